"""The CPU oracle is pinned against golden vectors produced by importing the
reference itself (tests/golden/make_golden.py).  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import ref


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def test_weights_sha_match_golden():
    from dmx import synth
    keys = json.load(open(os.path.join(GOLDEN, "keys.json")))
    assert synth.state_dict_sha256({k: v.numpy() for k, v in synth.unet_cond_geom_weights(0).items()}) == \
        keys["sha256"]["unet_cond_geom_seed0"]
    assert synth.state_dict_sha256({k: v.numpy() for k, v in synth.vae_weights(1).items()}) == keys["sha256"]["vae_seed1"]


def test_schedule_bit_exact(golden):
    g = golden("schedule.npz")
    b, a, ab = ref.schedule(1000)
    assert np.array_equal(b.numpy(), g["betas"])
    assert np.array_equal(a.numpy(), g["alphas"])
    assert np.array_equal(ab.numpy(), g["alpha_bars"])


def test_rng_probe(golden):
    g = golden("rng_probe.npz")
    torch.manual_seed(int(g["seed"]))
    p = torch.randn(4096)
    assert np.array_equal(p[:16].numpy(), g["first"])


def test_forward_32_and_28(golden, unet_sd):
    for name in ("forward_32.npz", "forward_28.npz"):
        g = golden(name)
        with torch.no_grad():
            eps, geom = ref.unet_cond_geom_forward(unet_sd, torch.from_numpy(g["x"]), torch.from_numpy(g["t"]),
                                                   torch.from_numpy(g["y"]), torch.from_numpy(g["vals"]),
                                                   torch.from_numpy(g["mask"]))
        assert rel(eps, g["eps"]) < 1e-5, name
        assert rel(geom, g["geom"]) < 1e-5, name


def test_forward_uncond(golden):
    from dmx import synth
    sd = synth.unet_weights(0, in_ch=4)
    g = golden("forward_uncond.npz")
    with torch.no_grad():
        eps = ref.unet_forward(sd, torch.from_numpy(g["x"]), torch.from_numpy(g["t"]))
    assert rel(eps, g["eps"]) < 1e-5


def test_vae_decode(golden, vae_sd):
    g = golden("vae_decode.npz")
    with torch.no_grad():
        img16 = ref.vae_decode(vae_sd, torch.from_numpy(g["z16"]))
        img32 = ref.vae_decode(vae_sd, torch.from_numpy(g["z32"]))
    assert rel(img16, g["img16"]) < 1e-5
    u8 = ref.to_uint8(img32).permute(0, 2, 3, 1).numpy()
    d = np.abs(u8.astype(int) - g["u8_32"].astype(int))
    assert d.max() <= 1 and (d > 0).mean() < 1e-3


def test_denoise_cond_steps(golden, unet_sd):
    g = golden("denoise_cond.npz")
    _, alphas, abars = ref.schedule(1000)
    x, y = torch.from_numpy(g["x"]), torch.from_numpy(g["y"])
    vals, mask = torch.from_numpy(g["vals"]), torch.from_numpy(g["mask"])
    for tv in (1000, 500, 2, 1):
        t = torch.full((2,), tv, dtype=torch.long)
        with torch.no_grad():
            out = ref.cfg_step(unet_sd, x, t, y, alphas, abars, 3.0, 0, vals, mask, torch.from_numpy(g[f"noise_{tv}"]))
        assert rel(out, g[f"out_{tv}"]) < 1e-5, tv


def test_sampler_csv(golden):
    g = golden("sampler_csv.npz")
    table = np.loadtxt(os.path.join(GOLDEN, "entities.csv"), delimiter=",")
    for cid in (1, 2, 3):
        v, m = ref.build_vals_mask(table, cid, (400, 400))
        assert np.array_equal(v, g[f"vals_{cid}"]) and np.array_equal(m, g[f"mask_{cid}"])
        v, m = ref.build_vals_mask(table, cid, (320.0, 280.0))
        assert np.array_equal(v, g[f"vals_{cid}_320x280"])


def test_short_cond_trajectory_T20(golden, unet_sd):
    """sample_latent_cond with z_shape given, T=20 (draw order x_T then one per step)."""
    g = golden("sample_T20.npz")
    torch.manual_seed(int(g["seed"]))
    b, a, ab = ref.schedule(20)
    y = torch.tensor([1, 3])
    vals = torch.zeros((2, 12))
    mask = torch.zeros((2, 12))
    for i, cls in enumerate([1, 3]):
        for k in {1: ["x1", "y1", "x2", "y2"], 3: ["ax", "ay", "ar", "theta1", "theta2"]}[cls]:
            mask[i, ref.KEY_ORDER.index(k)] = 1.0
    x = torch.randn((2, 4, 32, 32))
    with torch.no_grad():
        for i in range(20, 0, -1):
            t = torch.full((2,), i, dtype=torch.long)
            x = ref.cfg_step(unet_sd, x, t, y, a, ab, 3.0, 0, vals, mask, torch.randn(x.shape))
    assert rel(x, g["latent_32"]) < 1e-5


@pytest.mark.parametrize("tag", ["64", "56"])
def test_vae_encode(golden, vae_sd, tag):
    """VAE.encode (models/vae.py:51-62) vs the reference's own outputs (make_golden_encode.py)."""
    g = golden("vae_encode.npz")
    with torch.no_grad():
        z, kl, mu, lv = ref.vae_encode(vae_sd, torch.from_numpy(g[f"x{tag}"]), torch.from_numpy(g[f"eps{tag}"]))
    assert torch.equal(z, torch.from_numpy(g[f"z{tag}"]))
    assert torch.equal(mu, torch.from_numpy(g[f"mu{tag}"]))
    assert float(kl) == float(g[f"kl{tag}"])


def test_vae_forward_composes_encode_decode(golden, vae_sd):
    """VAE.forward (models/vae.py:71-76) restated as encode -> decode -> MSE + 1e-6 KL; its encode half is
    pinned by the reference's encode outputs (parity of the loss arithmetic itself is unpinned)."""
    g = golden("vae_encode.npz")
    x, eps = torch.from_numpy(g["x64"]), torch.from_numpy(g["eps64"])
    with torch.no_grad():
        x_recon, z, loss, recon, kl = ref.vae_forward(vae_sd, x, eps)
        assert torch.equal(z, torch.from_numpy(g["z64"]))
        assert float(kl) == float(g["kl64"])
        assert torch.equal(x_recon, ref.vae_decode(vae_sd, z))
        assert float(loss) == float(((x_recon - x) ** 2).mean() + 1e-6 * kl)


# ---- eval_iou_noise metrics: oracle vs the reference's outputs --------
def test_eval_oracle_matches_reference_metrics(golden):
    import numpy as np
    from oracle import eval_ref
    g = golden("eval_metrics.npz")
    for i in range(g["metrics"].shape[0]):
        gm, qm = eval_ref.binarize(g["gray_gt"][i]), eval_ref.binarize(g["gray_gen"][i])
        assert np.array_equal(gm, g["mask_gt"][i]) and np.array_equal(qm, g["mask_gen"][i])
        m = eval_ref.compute_metrics(gm, qm, 2.0)
        got = np.array([m[k] for k in ("iou", "gt_iou", "far_noise_ratio", "gauss_recall", "inter", "union",
                                       "gt_area", "pred_area", "fp")])
        assert np.array_equal(got, g["metrics"][i]), i
    m = eval_ref.compute_metrics(g["ns_gt"], g["ns_gen"], 3.5)
    assert np.array_equal(np.array(list(m.values())), g["ns_metrics"])


def test_eval_oracle_empty_gt_distance_convention():
    """scipy's transform of an image with no GT pixel measures from the virtual feature (-1, 0):
    the convention the native kernel reproduces (csrc/eval.h)."""
    import numpy as np
    from oracle import eval_ref
    gt = np.zeros((5, 9), bool)
    y, x = np.mgrid[0:5, 0:9]
    assert np.array_equal(eval_ref.distance_map_to_gt(gt), np.sqrt(((y + 1) ** 2 + x ** 2).astype(np.float64)))
