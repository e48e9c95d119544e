"""Print per-kernel VGPR/AGPR/scratch/occupancy/LDS of a HIP source (hipcc -Rpass-analysis)."""
import re
import subprocess
import sys

src = sys.argv[1]
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Iinclude",
                      "-x", "hip", "-c", src, "-o", "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0].split("\\")[0]] = int(m.group(1))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for r in rows:
    if flt in r["name"]:
        print(f"{r.get('VGPRs',0):4d}v {r.get('AGPRs',0):4d}a scr={r.get('ScratchSize',0):3d} occ={r.get('Occupancy',0)} "
              f"lds={r.get('LDS',0):6d}  {r['name'][:110]}")
