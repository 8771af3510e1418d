"""Golden vectors of the training step, from the reference modules
themselves (build container only; the reference never travels to the GPU box).

Run from the repo root:  python tests/golden/make_golden_train.py

train_step.npz holds two cases, each the body of train_latent_cond.py:136-163 run on the CPU
with the reference's own UnetCondWithGeomHead / UnetCond, F.mse_loss, masked_geom_mse and
torch.optim.Adam(lr=1e-4), weights = dmx.synth (U-Net seed 0):
  * "g": UnetCondWithGeomHead, B=2, 28x28 latents (the Up pad path), cond given, sample 1's
    label / condition dropped (the loop's CFG dropout), geom_lambda 0.5;
  * "c": UnetCond(cfg_drop_prob=0, remove_deep_conv=True), B=3, 16x16, no cond (cond_mlp
    takes no gradient), plain MSE.
Stored per case: the inputs, eps / geom / loss, and per parameter (state_dict order) the
gradient's sum and L2 norm, 16 sampled gradient entries, and the same 16 entries of the
parameter after two Adam steps (second step on a fresh noise draw).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
SAMPLES = 16


def _case(tag, model, B, hw, cond, lam, seed):
    from losses.geom_losses import masked_geom_mse  # noqa: E402  (reference)
    g = torch.Generator().manual_seed(seed)
    steps = []
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    names = [n for n, _ in model.named_parameters()]
    rec = {}
    for step in range(2):
        z_noisy = torch.randn((B, 4, hw, hw), generator=g)
        noise = torch.randn((B, 4, hw, hw), generator=g)
        t = torch.randint(1, 1001, (B,), generator=g)
        y = torch.randint(1, 4, (B,), generator=g)
        vals = torch.rand((B, 12), generator=g)
        mask = (torch.rand((B, 12), generator=g) > 0.3).float()
        drop = torch.zeros(B, dtype=torch.bool)
        if cond:
            drop[1] = True  # train_latent_cond.py:140-145 with this sample dropped
        y_used = torch.where(drop, torch.zeros_like(y), y)
        keep = (~drop).float().unsqueeze(1)
        if cond:
            out = model(z_noisy, t, y_used, cond_vals=vals * keep, cond_mask=mask * keep)
        else:
            out = model(z_noisy, t, y_used)
        eps, geom = out if isinstance(out, tuple) else (out, None)
        loss = F.mse_loss(eps, noise)
        if geom is not None:
            loss = loss + lam * masked_geom_mse(geom, vals, mask * keep)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        if step == 0:
            rng = np.random.default_rng(seed)
            ps = dict(model.named_parameters())
            idx = np.stack([rng.integers(0, ps[n].numel(), SAMPLES) for n in names])
            has = np.array([ps[n].grad is not None for n in names])
            gsum = np.array([float(ps[n].grad.double().sum()) if ps[n].grad is not None else 0.0 for n in names])
            gl2 = np.array([float(ps[n].grad.double().norm()) if ps[n].grad is not None else 0.0 for n in names])
            gval = np.stack([ps[n].grad.reshape(-1)[torch.from_numpy(i)].numpy() if ps[n].grad is not None
                             else np.zeros(SAMPLES, np.float32) for n, i in zip(names, idx)])
            rec.update({
                "x": z_noisy.numpy(), "noise": noise.numpy(), "t": t.numpy(), "y": y_used.numpy(),
                "vals": (vals * keep).numpy(), "mask": (mask * keep).numpy(), "vals_gt": vals.numpy(),
                "eps": eps.detach().numpy(), "loss": np.float64(loss.item()),
                "idx": idx, "has_grad": has, "g_sum": gsum, "g_l2": gl2, "g_val": gval,
            })
            if geom is not None:
                rec["geom"] = geom.detach().numpy()
        else:
            rec.update({"x2": z_noisy.numpy(), "noise2": noise.numpy(), "t2": t.numpy(), "y2": y_used.numpy(),
                        "vals2": (vals * keep).numpy(), "mask2": (mask * keep).numpy(), "vals_gt2": vals.numpy()})
        opt.step()
    ps = dict(model.named_parameters())
    rec["p_after"] = np.stack([ps[n].detach().reshape(-1)[torch.from_numpy(i)].numpy()
                               for n, i in zip(names, rec["idx"])])
    rec["names"] = np.array(names)
    rec["lam"] = np.float64(lam)
    return {f"{tag}_{k}": v for k, v in rec.items()}


def main():
    torch.set_num_threads(8)
    sys.path.insert(0, os.path.join(REPO, "diffusion-model_amd"))
    from dmx import synth  # our seeded weight generator (no reference code)
    sys.path.insert(0, REF)
    from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402  (reference)
    from models.unet_cond import UnetCond  # noqa: E402

    out = {}
    mg = UnetCondWithGeomHead()
    mg.load_state_dict(synth.unet_cond_geom_weights(0))
    mg.train()
    out.update(_case("g", mg, 2, 28, True, 0.5, 101))

    mc = UnetCond(cfg_drop_prob=0.0, remove_deep_conv=True)
    sd = synth.unet_cond_geom_weights(0, remove_deep_conv=True)
    mc.load_state_dict({k: v for k, v in sd.items() if not k.startswith("geom_head.")})
    mc.train()
    out.update(_case("c", mc, 3, 16, False, 0.0, 202))
    np.savez_compressed(os.path.join(HERE, "train_step.npz"), **out)
    print("[golden-train] loss g=%.6f c=%.6f" % (out["g_loss"], out["c_loss"]))


if __name__ == "__main__":
    main()
