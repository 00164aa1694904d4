"""Per-kernel resources (VGPRs, SGPRs, spills, scratch, LDS) of librsgpu.so's
gfx950 code object, read from its AMDGPU metadata notes (no recompile).

    python tools/co_resources.py [substring ...]
"""
import os
import re
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    lib = os.path.join(ROOT, "infinicache_amd", "librsgpu.so")
    libdir = os.path.dirname(lib)
    notes = ""
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", lib], check=True, stdout=subprocess.DEVNULL)
    try:  # one code object per HIP translation unit, extracted next to the library
        for f in sorted(os.listdir(libdir)):
            if f.startswith("librsgpu.so.") and "amdgcn" in f:
                notes += subprocess.run([f"{LLVM}/llvm-readobj", "--notes", os.path.join(libdir, f)],
                                        capture_output=True, text=True, check=True).stdout
    finally:
        for f in os.listdir(libdir):
            if f.startswith("librsgpu.so.") and f != "librsgpu.so":
                os.remove(os.path.join(libdir, f))
    pats = sys.argv[1:]
    for e in notes.split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", e).group(1)
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        if pats and not any(p in dem for p in pats):
            continue
        g = lambda k: (re.search(rf"\.{k}:\s+(\d+)", e) or [None, "?"])[1]
        print(f"{dem[:90]:90s} vgpr {g('vgpr_count'):>3} sgpr {g('sgpr_count'):>3} "
              f"vspill {g('vgpr_spill_count')} sspill {g('sgpr_spill_count')} "
              f"scratch {g('private_segment_fixed_size')} lds {g('group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
