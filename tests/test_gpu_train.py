"""The native training step (include/dmx.h dmx_train_forward / dmx_train_backward) driven the
way train_latent_cond.py:136-163 drives the reference: drop-in module in train mode,
F.mse_loss (+ masked_geom_mse), loss.backward(), torch Adam.  Checked against the reference's
own gradients / Adam steps (tests/golden/train_step.npz) and against the CPU oracle's full
gradient tensors (oracle/train_ref.py).  Tolerances: fp32 arithmetic on both sides, different
summation orders — per-tensor relative L2 of the gradient <= 1e-4 vs the oracle, the reference
statistics within 2e-4 of each tensor's L2 norm."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

from test_train_oracle import GOLD, case_inputs, case_weights, grad_stats_close  # noqa: E402


def _model(tag, dev):
    from models.unet_cond import UnetCond
    from models.unet_cond_geom import UnetCondWithGeomHead
    sd, geom, shallow = case_weights(tag)
    m = UnetCondWithGeomHead() if geom else UnetCond(cfg_drop_prob=0.0, remove_deep_conv=True)
    m.load_state_dict(sd)
    return m.to(dev).train(), geom


def _loss(m, geom, inputs, dev, lam):
    from losses.geom_losses import masked_geom_mse
    x, t, y, vals, mask, noise, gt = (v.to(dev) if v is not None else None for v in inputs)
    out = m(x, t, y, cond_vals=vals, cond_mask=mask) if vals is not None else m(x, t, y)
    eps, g = out if isinstance(out, tuple) else (out, None)
    loss = F.mse_loss(eps, noise)
    if g is not None:
        loss = loss + lam * masked_geom_mse(g, gt, mask)
    return loss, eps, g


@pytest.mark.parametrize("tag", ["g", "c"])
def test_native_step_matches_reference_and_oracle(cuda, tag):
    from oracle import train_ref
    m, geom = _model(tag, cuda)
    lam = float(GOLD[f"{tag}_lam"])
    loss, eps, g = _loss(m, geom, case_inputs(tag), cuda, lam)
    m.zero_grad(set_to_none=True)
    loss.backward()
    names = [n for n, _ in m.named_parameters()]
    grads = {n: p.grad for n, p in m.named_parameters()}
    assert abs(float(loss) - float(GOLD[f"{tag}_loss"])) <= 2e-5 * float(GOLD[f"{tag}_loss"])
    np.testing.assert_allclose(eps.detach().cpu().numpy(), GOLD[f"{tag}_eps"], rtol=1e-4, atol=2e-5)
    if geom:
        np.testing.assert_allclose(g.detach().cpu().numpy(), GOLD[f"{tag}_geom"], rtol=1e-4, atol=2e-5)
    assert grad_stats_close(tag, grads, names) == []
    # full tensors vs the oracle's autograd
    sd, geom_, shallow = case_weights(tag)
    x, t, y, vals, mask, noise, gt = case_inputs(tag)
    _, _, _, ref = train_ref.loss_and_grads(sd, x, t, y, vals, mask, noise, gt, mask, lam, geom_, shallow)
    worst = []
    for n in names:
        if ref[n] is None:
            assert grads[n] is None, n
            continue
        a, b = grads[n].detach().double().cpu(), ref[n].double()
        worst.append((float((a - b).norm() / max(float(b.norm()), 1e-30)), n))
    worst.sort(reverse=True)
    print("[train] worst rel-L2 vs oracle:", worst[:5])
    assert worst[0][0] <= 1e-4, worst[:5]


def test_native_grads_at_bench_shape_vs_oracle(cuda):
    """The bench.py training leg's shape: B = 32 latents of 28 x 28 (224^2 images through the VAE),
    t ~ U{1..1000}, CFG dropout (label 0 and zeroed conditions on dropped rows), geom_lambda 0.5
    — the wgrad split counts, two-pass colsums, GroupNorm-backward chunking and attention lengths
    of the reported training throughput — every gradient within 1e-4 rel-L2 of the oracle."""
    from losses.geom_losses import masked_geom_mse
    from oracle import train_ref
    from dmx import synth
    B, hw = 32, 28
    g = torch.Generator().manual_seed(21)
    x = torch.randn((B, 4, hw, hw), generator=g)
    t = torch.randint(1, 1001, (B,), generator=g)
    classes = torch.randint(1, 4, (B,), generator=g)
    drop = torch.rand(B, generator=g) < 0.1
    drop[:2] = True
    y = torch.where(drop, torch.zeros_like(classes), classes)
    keep = (~drop).float().unsqueeze(1)
    vals = torch.rand((B, 12), generator=g) * keep
    mask = (torch.rand((B, 12), generator=g) > 0.3).float() * keep
    noise = torch.randn((B, 4, hw, hw), generator=g)
    gt = torch.rand((B, 12), generator=g)
    sd = synth.unet_cond_geom_weights(0)
    from models.unet_cond_geom import UnetCondWithGeomHead
    m = UnetCondWithGeomHead()
    m.load_state_dict(sd)
    m.to(cuda).train()
    dv = [v.to(cuda) for v in (x, t, y, vals, mask, noise, gt)]
    eps, gp = m(dv[0], dv[1], dv[2], cond_vals=dv[3], cond_mask=dv[4])
    loss = F.mse_loss(eps, dv[5]) + 0.5 * masked_geom_mse(gp, dv[6], dv[4])
    m.zero_grad(set_to_none=True)
    loss.backward()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    rloss, _, _, ref = train_ref.loss_and_grads(sd, x, t, y, vals, mask, noise, gt, mask, 0.5, True, False)
    assert abs(float(loss) - float(rloss)) <= 2e-5 * float(rloss)
    worst = []
    for n, p in m.named_parameters():
        if ref[n] is None:
            assert p.grad is None, n
            continue
        a, b = p.grad.detach().double().cpu(), ref[n].double()
        worst.append((float((a - b).norm() / max(float(b.norm()), 1e-30)), n))
    worst.sort(reverse=True)
    print("[train bench shape] worst rel-L2 vs oracle:", worst[:5])
    assert worst[0][0] <= 1e-4, worst[:5]


def test_two_adam_steps_match_reference(cuda):
    tag = "g"
    m, geom = _model(tag, cuda)
    lam = float(GOLD[f"{tag}_lam"])
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    for second in (False, True):
        loss, _, _ = _loss(m, geom, case_inputs(tag, second), cuda, lam)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    names = [n for n, _ in m.named_parameters()]
    ps = dict(m.named_parameters())
    idx, after = GOLD[f"{tag}_idx"], GOLD[f"{tag}_p_after"]
    got = np.stack([ps[n].detach().cpu().reshape(-1)[torch.from_numpy(i)].numpy() for n, i in zip(names, idx)])
    d = np.abs(got - after)
    assert d.max() <= 2.1e-4
    assert (d <= 1e-6 + 1e-5 * np.abs(after)).mean() >= 0.97


def test_refresh_after_optimizer_step_equals_fresh_model(cuda):
    """optimizer.step() changes the parameters in place: the next inference forward repacks on the
    device (dmx_model_refresh) and must equal a model built from scratch from the same weights."""
    from models.unet_cond_geom import UnetCondWithGeomHead
    m, geom = _model("g", cuda)
    nm0 = m.native()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    loss, _, _ = _loss(m, geom, case_inputs("g"), cuda, 0.5)
    opt.zero_grad()
    loss.backward()
    opt.step()
    x, t, y, vals, mask, _, _ = (v.to(cuda) if v is not None else None for v in case_inputs("g"))
    m.eval()
    with torch.no_grad():
        e1, g1 = m(x, t, y, cond_vals=vals, cond_mask=mask)
    assert m.native() is nm0  # refreshed, not rebuilt
    fresh = UnetCondWithGeomHead().to(cuda).eval()
    fresh.load_state_dict(m.state_dict())
    with torch.no_grad():
        e2, g2 = fresh(x, t, y, cond_vals=vals, cond_mask=mask)
    assert torch.equal(e1, e2) and torch.equal(g1, g2)


def test_stale_tape_is_refused(cuda):
    from dmx import _lib
    m, geom = _model("g", cuda)
    inputs = case_inputs("g")
    l1, _, _ = _loss(m, geom, inputs, cuda, 0.5)
    l2, _, _ = _loss(m, geom, inputs, cuda, 0.5)
    with pytest.raises(_lib.DmxError, match="stale tape"):
        l1.backward()
    l2.backward()  # the current tape still works
    assert all(p.grad is not None for n, p in m.named_parameters())


def test_input_gradients_are_refused(cuda):
    m, geom = _model("g", cuda)
    x, t, y, vals, mask, _, _ = (v.to(cuda) if v is not None else None for v in case_inputs("g"))
    with pytest.raises(NotImplementedError):
        m(x.requires_grad_(True), t, y, cond_vals=vals, cond_mask=mask)


def test_unetcond_training_dropout_draws_like_reference(cuda):
    """UnetCond.forward in train mode with cfg_drop_prob > 0 draws torch.rand_like(y.float()) then
    torch.rand(B) for the condition (models/unet_cond.py:199-211) from the global generator."""
    from models.unet_cond import UnetCond
    m = UnetCond(cfg_drop_prob=0.5).to(cuda).train()
    x, t, y, vals, mask, _, _ = (v.to(cuda) if v is not None else None for v in case_inputs("g"))
    torch.manual_seed(5)
    with torch.no_grad():
        m(x, t, y, cond_vals=vals, cond_mask=mask)
    after = torch.cuda.get_rng_state(cuda)
    torch.manual_seed(5)
    torch.rand_like(y.float())
    torch.rand(vals.size(0), device=cuda)
    assert torch.equal(after, torch.cuda.get_rng_state(cuda))


def test_refreshed_training_weights_equal_fresh_model(cuda):
    """After optimizer.step() the training weights are re-derived on the device (dmx_model_refresh:
    the data-gradient packs straight from the forward weights — flipped 3x3 / transposed Linear —
    the forward and data-gradient f16 planes with their device-side scales): the next forward +
    backward must equal, bit for bit, that of a model built from scratch from the updated weights."""
    from models.unet_cond_geom import UnetCondWithGeomHead
    m, geom = _model("g", cuda)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    loss, _, _ = _loss(m, geom, case_inputs("g"), cuda, 0.5)
    opt.zero_grad()
    loss.backward()
    opt.step()
    nm0 = m.native()
    inputs = case_inputs("g", True)
    loss1, eps1, g1 = _loss(m, geom, inputs, cuda, 0.5)
    opt.zero_grad()
    loss1.backward()
    assert m.native() is nm0  # refreshed, not rebuilt
    grads1 = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    fresh = UnetCondWithGeomHead().to(cuda).train()
    fresh.load_state_dict(m.state_dict())
    loss2, eps2, g2 = _loss(fresh, geom, inputs, cuda, 0.5)
    fresh.zero_grad()
    loss2.backward()
    assert torch.equal(eps1, eps2) and torch.equal(g1, g2)
    for n, p in fresh.named_parameters():
        assert torch.equal(grads1[n], p.grad), n
