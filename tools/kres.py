#!/usr/bin/env python
"""Per-kernel resource table of a .hip file (compile only, no GPU):
VGPRs / SGPRs / spills / LDS / occupancy from hipcc's kernel-resource-usage
remarks.  Usage: python tools/kres.py FILE.hip [FILTER] [-D...]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else ""
extra = [a for a in sys.argv[2:] if a.startswith("-")]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics", "-c", src,
       "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"] + extra
r = subprocess.run(cmd, capture_output=True, text=True)
rows, cur = [], None
for ln in r.stderr.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", ln)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        name = t.split(":", 1)[1].strip()
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        name = re.sub(r"\(anonymous namespace\)::", "", name)
        name = re.sub(r"\(.*\)$", "", name)
        cur = {"name": name}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
if r.returncode:
    print(r.stderr[-3000:])
    sys.exit(1)
keys = ["VGPRs", "AGPRs", "SGPRs", "VGPRs Spill", "SGPRs Spill", "LDS Size [bytes/block]", "Occupancy [waves/SIMD]"]
print(f"{'kernel':70s} " + " ".join(f"{k.split()[0][:5]:>6s}" + ("sp" if "Spill" in k else "") for k in keys))
for row in rows:
    if flt and flt not in row["name"]:
        continue
    print(f"{row['name'][:70]:70s} " + " ".join(f"{row.get(k, '-'):>8s}" for k in keys))
