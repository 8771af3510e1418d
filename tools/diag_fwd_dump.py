"""Diagnostic: one B=64 CFG step (x3) of the synthetic config-2 model, latents written to the
path given (used to compare builds / env switches bit for bit, e.g. DMX_GN_FUSE=0 vs 1)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "diffusion-model_amd"), REPO):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

if __name__ == "__main__":
    import diff
    from dmx import synth
    from models.unet_cond_geom import UnetCondWithGeomHead
    from bench import make_inputs
    dev = torch.device("cuda:0")
    m = UnetCondWithGeomHead()
    m.load_state_dict(synth.unet_cond_geom_weights(0))
    m.to(dev).eval()
    d = diff.Diffuser(1000, device=dev)
    x, y, vals, mask = make_inputs(64, 32, dev)
    t = torch.full((64,), 537, dtype=torch.long, device=dev)
    torch.manual_seed(3)
    out = d.denoise_cond(m, x, t, y=y, guidance_scale=3.0, cond_vals=vals, cond_mask=mask)
    np.save(sys.argv[1], out.cpu().numpy())
