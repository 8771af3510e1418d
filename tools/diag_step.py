"""One event-timed eager CFG step at the bench shape -> per-family kernel times (diagnostic A/B
of library builds: DMX_LIB=libdmx_xxx.so python tools/diag_step.py TAG)."""
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "diffusion-model_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
import diff  # noqa: E402
from dmx import synth  # noqa: E402
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "run"
dev = torch.device("cuda:0")
m = UnetCondWithGeomHead()
m.load_state_dict(synth.unet_cond_geom_weights(0))
m.to(dev).eval()
nm = m.native()
d = diff.Diffuser(1000, device=dev)
tables = d.coef_tables(dev, True)
x, y, vals, mask = bench.make_inputs(64, 32, dev)
t = torch.full((64,), 1000, dtype=torch.long, device=dev)
for _ in range(3):
    recs = nm.step_profile(x.clone(), x.clone(), t, y, 0, vals, mask, 3.0, tables, None, seed=1)
fam = defaultdict(float)
for r in recs:
    fam[r["kernel"]] += r["ms"] * 1e3
tot = sum(fam.values())
out = {"tag": tag, "total_us": round(tot, 1), "kernels": {k: round(v, 1) for k, v in sorted(fam.items(), key=lambda kv: -kv[1])}}
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump({"records": recs, **out}, open(os.path.join(REPO, "gpurun_out", f"diag_{tag}.json"), "w"), indent=1)
print(json.dumps(out)[:1500])
