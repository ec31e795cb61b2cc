"""Per-kernel register / spill / LDS summary from hipcc -Rpass-analysis=kernel-resource-usage.
usage: python tools/kres.py <file.hip> [name filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17",
                      "-I/root/repo/include", "-I/root/repo/multi-modal-retrieval-predict-project_amd/csrc", "-c", src, "-o", "/dev/null",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        print(f"{k[:90]:90s} vgpr {v.get('VGPRs', 0):3d} agpr {v.get('AGPRs', 0):3d} spill {v.get('VGPRs Spill', 0):3d} "
              f"scratch {v.get('ScratchSize [bytes/lane]', 0):3d} occ {v.get('Occupancy [waves/SIMD]', 0)}")
