"""Per-kernel VGPR / AGPR / spill / scratch / LDS usage of libbnn.so's gfx950 code object.

    python tools/kernel_regs.py [name-substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

LIB = os.environ.get("BNN_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "distributed-mnist-bnns_amd", "lib", "libbnn.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    subs = sys.argv[1:]
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "libbnn.so")          # the bundles are extracted next to the input
        subprocess.run(["cp", LIB, src], check=True)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", src], cwd=d, check=True, capture_output=True)
        notes = "".join(subprocess.run([f"{LLVM}/llvm-readelf", "--notes", os.path.join(d, co)], check=True,
                                       capture_output=True, text=True).stdout
                        for co in sorted(os.listdir(d)) if co.endswith("gfx950"))   # one code object per TU
    kernels = re.split(r"\n\s+- \.", notes)
    for k in kernels:
        m = re.search(r"\.name:\s+(\S+)", k)
        if not m or m.group(1).endswith(".kd"):
            continue
        name = subprocess.run(["c++filt"], input=m.group(1), capture_output=True, text=True).stdout.strip()
        if subs and not any(s in name for s in subs):
            continue
        f = {key: re.search(rf"\.{key}:\s+(\d+)", k) for key in
             ("vgpr_count", "agpr_count", "vgpr_spill_count", "private_segment_fixed_size", "group_segment_fixed_size")}
        v = {key: (int(x.group(1)) if x else 0) for key, x in f.items()}
        print(f"vgpr {v['vgpr_count']:3d} agpr {v['agpr_count']:3d} spill {v['vgpr_spill_count']:3d} "
              f"scratch {v['private_segment_fixed_size']:4d} lds {v['group_segment_fixed_size']:6d}  {name[:150]}")


if __name__ == "__main__":
    main()
