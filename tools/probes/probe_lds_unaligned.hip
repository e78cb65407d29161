// Does ds_read_b128 at a 2-byte-aligned LDS address return the 16 bytes at that address on gfx950?
// (Decides whether the conv filter kernel can read kw-shifted input windows from one image.)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short bf8 __attribute__((ext_vector_type(8)));
__global__ void k(short* out, int off) {
  __shared__ __attribute__((aligned(16))) short s[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) s[i] = (short)i;
  __syncthreads();
  const bf8 v = *reinterpret_cast<const bf8*>(s + 8 * threadIdx.x + off);
  for (int j = 0; j < 8; ++j) out[8 * threadIdx.x + j] = v[j];
}
int main() {
  short* d;
  hipMalloc(&d, 512 * sizeof(short));
  short h[512];
  int bad_total = 0;
  for (int off = 0; off < 8; ++off) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, off);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 512; ++i) bad += h[i] != (short)(i + off);
    printf("offset %d elements: %d mismatches (first: got %d want %d)\n", off, bad, h[0], off);
    bad_total += bad;
  }
  hipFree(d);
  return bad_total ? 1 : 0;
}
