"""The training-step oracle (oracle/train_ref.py) pinned to the reference's own loss.backward()
and Adam steps (tests/golden/train_step.npz, make_golden_train.py).  CPU only."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diffusion-model_amd"))

from oracle import train_ref  # noqa: E402
from dmx import synth  # noqa: E402

GOLD = np.load(os.path.join(HERE, "golden", "train_step.npz"))


def case_weights(tag):
    if tag == "g":
        return synth.unet_cond_geom_weights(0), True, False
    sd = synth.unet_cond_geom_weights(0, remove_deep_conv=True)
    return {k: v for k, v in sd.items() if not k.startswith("geom_head.")}, False, True


def case_inputs(tag, second=False):
    s = "2" if second else ""
    g = lambda k: torch.from_numpy(np.asarray(GOLD[f"{tag}_{k}{s}"]))  # noqa: E731
    vals = g("vals") if tag == "g" else None
    mask = g("mask") if tag == "g" else None
    gt = g("vals_gt") if tag == "g" else None
    return g("x"), g("t").long(), g("y").long(), vals, mask, g("noise"), gt


def grad_stats_close(tag, grads, names, rel=2e-4):
    """Per parameter: sum and L2 of the gradient and 16 sampled entries vs the reference's."""
    idx, has = GOLD[f"{tag}_idx"], GOLD[f"{tag}_has_grad"]
    gsum, gl2, gval = GOLD[f"{tag}_g_sum"], GOLD[f"{tag}_g_l2"], GOLD[f"{tag}_g_val"]
    scale = float(np.max(gl2))
    bad = []
    for k, n in enumerate(names):
        g = grads[n]
        if not has[k]:
            if g is not None:
                bad.append((n, "expected no gradient"))
            continue
        g = g.detach().double().cpu().reshape(-1)
        if abs(float(g.norm()) - gl2[k]) > rel * gl2[k] + 1e-9 * scale:
            bad.append((n, "l2", float(g.norm()), gl2[k]))
        if abs(float(g.sum()) - gsum[k]) > rel * gl2[k] * np.sqrt(g.numel()) + 1e-9 * scale:
            bad.append((n, "sum", float(g.sum()), gsum[k]))
        v = g[torch.from_numpy(idx[k])].numpy()
        if np.max(np.abs(v - gval[k])) > rel * gl2[k] + 1e-9 * scale:
            bad.append((n, "vals", float(np.max(np.abs(v - gval[k]))), gl2[k]))
    return bad


@pytest.mark.parametrize("tag", ["g", "c"])
def test_oracle_grads_match_reference(tag):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    sd, geom, shallow = case_weights(tag)
    names = list(GOLD[f"{tag}_names"])
    assert names == list(sd.keys())
    x, t, y, vals, mask, noise, gt = case_inputs(tag)
    loss, eps, gpred, grads = train_ref.loss_and_grads(
        sd, x, t, y, vals, mask, noise, gt, mask, float(GOLD[f"{tag}_lam"]), geom, shallow)
    assert abs(float(loss) - float(GOLD[f"{tag}_loss"])) <= 1e-5 * float(GOLD[f"{tag}_loss"])
    np.testing.assert_allclose(eps.numpy(), GOLD[f"{tag}_eps"], rtol=1e-4, atol=1e-5)
    if geom:
        np.testing.assert_allclose(gpred.numpy(), GOLD[f"{tag}_geom"], rtol=1e-4, atol=1e-5)
    assert grad_stats_close(tag, grads, names) == []


def test_oracle_two_adam_steps_match_reference():
    """Parameters after two torch Adam(lr=1e-4) steps on the oracle's gradients (the reference
    loop's optimizer) vs the reference's: first-step Adam updates are lr * sign(g), so entries
    whose gradient is at rounding level may flip; the bulk must agree to fp32 rounding."""
    tag = "g"
    sd, geom, shallow = case_weights(tag)
    names = list(sd.keys())
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    opt = torch.optim.Adam(params.values(), lr=1e-4)
    for second in (False, True):
        x, t, y, vals, mask, noise, gt = case_inputs(tag, second)
        opt.zero_grad(set_to_none=True)
        eps, g = train_ref.forward(params, x, t, y, vals, mask, geom, shallow)
        loss = torch.nn.functional.mse_loss(eps, noise) + float(GOLD[f"{tag}_lam"]) * train_ref.masked_geom_mse(g, gt, mask)
        loss.backward()
        opt.step()
    idx, after = GOLD[f"{tag}_idx"], GOLD[f"{tag}_p_after"]
    got = np.stack([params[n].detach().reshape(-1)[torch.from_numpy(i)].numpy() for n, i in zip(names, idx)])
    d = np.abs(got - after)
    assert d.max() <= 2.1e-4
    assert (d <= 1e-6 + 1e-5 * np.abs(after)).mean() >= 0.97
