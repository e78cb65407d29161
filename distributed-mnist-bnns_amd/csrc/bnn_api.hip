// Library-level entry points: version, thread-local error string.
#include <cstdarg>
#include <cstdio>

#include "bnn_common.h"

namespace bnn {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

}  // namespace bnn

BNN_API int bnn_version(void) { return 1; }

BNN_API const char* bnn_last_error(void) { return bnn::g_err; }
