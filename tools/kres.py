"""Per-kernel VGPR / scratch / occupancy of one translation unit (compile-time check for spills):
  python tools/kres.py csrc/k_halo.hip [extra hipcc flags...]"""
import re
import subprocess
import sys
import os

DMX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "diffusion-model_amd", "dmx")
src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + os.path.join(DMX, "..", "..", "include"),
       "-I" + os.path.join(DMX, "csrc"), "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-c", "--offload-device-only",
       "-Rpass-analysis=kernel-resource-usage", "-o", "/tmp/kres.o", os.path.join(DMX, src)] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1).split(" ")[0], m.group(2)
    if k == "Function":
        cur = {"name": subprocess.run(["c++filt"], input=v, capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    else:
        cur[k] = v
for r in rows:
    flag = "  <-- SPILL" if r.get("ScratchSize", "0") != "0" else ""
    print(f"{r.get('VGPRs','?'):>4} v {r.get('AGPRs','?'):>3} a {r.get('ScratchSize','?'):>4} scr occ {r.get('Occupancy','?')}  {r['name'][:150]}{flag}")
