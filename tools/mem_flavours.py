"""Census of the global memory instructions (with their cache-policy bits sc0 / sc1 / nt) in the
libbnn kernels whose names contain any of the given substrings -- how a hand-off's producer stores
and its consumers load.

    python tools/mem_flavours.py SUBSTRING [SUBSTRING ...]
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


def main():
    pats = sys.argv[1:]
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
                if ".kd" in head or not any(p in head for p in pats):
                    continue
                c = collections.Counter()
                for line in block.split("\n")[1:]:
                    m = re.match(r"\s+((?:global|buffer|flat)_(?:load|store|atomic)\w*)(.*?)(//|$)", line)
                    if m:
                        bits = [t for t in m.group(2).replace(",", " ").split() if t in ("sc0", "sc1", "nt", "lds")]
                        c[" ".join([m.group(1)] + bits)] += 1
                name = head[18:].replace("bnn::(anonymous namespace)::", "").replace("void ", "", 1)
                print(name.split("(")[0])
                for k, v in sorted(c.items()):
                    print(f"    {v:4d} {k}")


if __name__ == "__main__":
    main()
