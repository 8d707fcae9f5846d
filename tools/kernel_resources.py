"""VGPR / SGPR / spill / LDS figures of the kernels in a code object (llvm-readelf --notes
metadata, one entry per kernel).  python tools/kernel_resources.py <hsaco> [name-regex]"""
import re
import subprocess
import sys


def kernels(path):
    txt = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", path],
                         capture_output=True, text=True).stdout
    out = []
    for block in re.split(r"\n  - \.", txt)[1:]:
        f = dict(re.findall(r"^\s*\.?([a-z_]+):\s+(\S+)\s*$", "." + block, re.M))
        if "name" in f and "vgpr_count" in f:
            out.append(f)
    return out


if __name__ == "__main__":
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    for f in kernels(sys.argv[1]):
        if pat.search(f["name"]):
            print(f"{f['name']:32s} vgpr {f['vgpr_count']:>4} agpr {f.get('agpr_count', '0'):>3} "
                  f"sgpr {f.get('sgpr_count', '?'):>4} spill v{f.get('vgpr_spill_count', '?')}"
                  f"/s{f.get('sgpr_spill_count', '?')} lds {f.get('group_segment_fixed_size', '?')}")
