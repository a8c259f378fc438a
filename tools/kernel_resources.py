"""VGPRs / scratch / occupancy of every kernel in a HIP source (gfx950).

usage: python tools/kernel_resources.py libssa_amd/csrc/kernels.hip
"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-Iinclude", "-Ilibssa_amd/csrc", "--offload-arch=gfx950",
       "--cuda-device-only", "-c", "-o", "/dev/null", src, "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?): (.*?) \[", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    print(f"{name[:60]:60s} vgpr={r.get('VGPRs'):>4} agpr={r.get('AGPRs'):>3} scratch={r.get('ScratchSize [bytes/lane]'):>4} "
          f"sgpr_spill={r.get('SGPRs Spill'):>3} occ={r.get('Occupancy [waves/SIMD]')}")
