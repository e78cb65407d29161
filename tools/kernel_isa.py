"""Static instruction mix of libbnn kernels (gfx950 code object): counts of VALU / SALU / LDS /
global / MFMA / branch instructions in each matching kernel's body, optionally its disassembly.

    python tools/kernel_isa.py SUBSTRING [--dump]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

LIB = os.environ.get("BNN_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "distributed-mnist-bnns_amd", "lib", "libbnn.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def classify(op):
    if "mfma" in op:
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_waitcnt") or op.startswith("s_barrier"):
        return "wait/barrier"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return "other"


def main():
    sub = sys.argv[1]
    dump = "--dump" in sys.argv
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "libbnn.so")
        subprocess.run(["cp", LIB, src], check=True)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", src], cwd=d, check=True, capture_output=True)
        for co in sorted(os.listdir(d)):
            if not co.endswith("gfx950"):
                continue
            text = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--demangle", os.path.join(d, co)],
                                  capture_output=True, text=True).stdout
            for block in re.split(r"\n(?=[0-9a-f]{16} <)", text):
                head = block.split("\n", 1)[0]
                if sub not in head or ".kd" in head:
                    continue
                cnt = collections.Counter()
                for line in block.split("\n")[1:]:
                    m = re.match(r"\s+([a-z_0-9]+)\b", line)
                    if m:
                        cnt[classify(m.group(1))] += 1
                print(head[:160])
                print("   ", ", ".join(f"{k} {v}" for k, v in sorted(cnt.items(), key=lambda kv: -kv[1])))
                if dump:
                    print(block)


if __name__ == "__main__":
    main()
