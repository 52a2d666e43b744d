"""Per-kernel resource usage (VGPR/AGPR/spill/LDS/occupancy) of one HIP source, gfx950."""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/include",
                      f"-I{ROOT}/flood-prediction-gan_amd/csrc", "-c", src, "-o", "/tmp/kres.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = {}
rows = []
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt"], input=v, capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    else:
        cur[k.split()[0] + ("S" if "Spill" in k else "")] = v
for r in rows:
    if flt in r["name"]:
        print(f"v{r.get('VGPRs','?'):>4} a{r.get('AGPRs','?'):>3} spill{r.get('VGPRsS','?'):>3} scr{r.get('ScratchSize','?'):>5} lds{r.get('LDS','?'):>7} occ{r.get('Occupancy','?'):>2}  {r['name'][:150]}")
