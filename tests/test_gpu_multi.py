"""The multi-GPU product path executed: ShardedCondSampler with world size 2 (gloo), both ranks on
cuda:0 (a one-GPU rehearsal of the one-process-per-GPU layout; RCCL refuses two ranks on one
device).  Rank 0 must receive the single-process result: latents within rel-L2 1e-5 (the shards
run different batch sizes, so GEMM split-K choices — summation orders — may differ), decoded
uint8 images within +-1 LSB.  Draw order per rank: tests/test_distributed_gloo.py (stub model)."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _job(mode, decode, B=5, T=4, hw=16):
    import diff
    from dmx import distributed as dd
    from dmx import synth
    from models.unet_cond_geom import UnetCondWithGeomHead
    from models.vae import VAE
    dev = torch.device("cuda:0")
    m = UnetCondWithGeomHead()
    m.load_state_dict(synth.unet_cond_geom_weights(0))
    m.to(dev).eval()
    v = None
    if decode:
        v = VAE()
        v.load_state_dict(synth.vae_weights(1))
        v.to(dev).eval()
    d = diff.Diffuser(T, device=dev)
    d.noise_source = mode
    g = torch.Generator().manual_seed(40)
    vals = torch.rand((B, 12), generator=g).to(dev)
    mask = (torch.rand((B, 12), generator=g) > 0.3).float().to(dev)
    torch.manual_seed(41)
    out = dd.ShardedCondSampler(d, m, v).sample({1: 3, 3: B - 3}, z_shape=(4, hw, hw), cond=vals, cond_mask=mask,
                                                decode=decode)
    return None if out is None else out.cpu()


def _worker(rank, world, port, mode, decode, q, kw=None):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = _job(mode, decode, **(kw or {}))
        # by value (numpy): a torch tensor would travel as a shared-memory fd that the parent can
        # only open while this process is still alive
        q.put((rank, None if out is None else out.numpy()))
    finally:
        dist.destroy_process_group()


def _run2(mode, decode, **kw):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, decode, q, kw)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (None if a is None else torch.from_numpy(a)) for r, a in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("mode", ["host", "device"])
def test_sharded_sampler_world2_on_one_gpu(cuda, mode):
    res = _run2(mode, decode=True)
    single = _job(mode, decode=True)
    assert res[1] is None and res[0].shape == single.shape == (5, 128, 128, 3)
    d = np.abs(res[0].numpy().astype(np.int32) - single.numpy().astype(np.int32))
    # The decoder takes its tiling / split-K decisions per sample (engine.hip vae_body, Run::tile_n),
    # so a sample's bytes do not depend on the shard it is decoded in (test_gpu_parity.py
    # test_vae_decode_batch_invariant); the U-Net step's decisions still follow the shard's batch
    # size, so latents may differ in summation order only.  Pixel contract of every other test.
    assert d.max() <= 1 and (d > 0).mean() <= 1e-3, (int(d.max()), float((d > 0).mean()))


def _config3_rank0_in_process(B=128, T=8, hw=32):
    """Rank 0 of a world of 2 emulated in this process (world / seed broadcast / gather patched to
    local no-ops): ShardedCondSampler's own shard range, global x_T draw and Philox sample offset."""
    from dmx import distributed as dd
    saved = (dd.world, dd.any_rank, dd.gather_rows, dd.dist.broadcast, dd.dist.get_backend)
    try:
        dd.world = lambda: (2, 0)
        dd.any_rank = lambda t, dev: bool(t)
        dd.gather_rows = lambda x, n: x
        dd.dist.broadcast = lambda *a, **k: None
        dd.dist.get_backend = lambda *a, **k: "gloo"
        return _job("device", False, B=B, T=T, hw=hw)
    finally:
        dd.world, dd.any_rank, dd.gather_rows, dd.dist.broadcast, dd.dist.get_backend = saved


def test_config3_per_rank_shape_world2_on_one_gpu(cuda):
    """BASELINE configs[2] at its per-rank shape: 64 samples per rank (B = 128 over
    world 2), 32 x 32 x 4 latents, CFG 3.0, T = 8 device-noise steps, VAE decode and the rank-0
    gather (diff.py:326-369).

    The U-Net takes its tiling / split-K decisions for a batch class (engine.hip dec_n: 128 samples
    for every CFG batch of >= 64), the decoder per sample, and the device noise is keyed by the
    global sample index: a rank's shard computes exactly the bytes of the same rows of a
    single-process B = 128 run.  Checked bit-wise twice: rank 0 emulated in this process, and the
    real two-process run with both ranks on this one GPU at once (which is how a run-to-run race in
    reduce_norm_kernel<1> was found and removed: DESIGN.md §7)."""
    kw = dict(B=128, T=8, hw=32)
    lsingle = _job("device", False, **kw)
    r0 = _config3_rank0_in_process(**kw)
    assert r0.shape == (64, 4, 32, 32)
    assert torch.equal(r0, lsingle[:64]), float((r0 - lsingle[:64]).norm() / lsingle[:64].norm())
    lat = _run2("device", False, **kw)
    assert lat[1] is None and lat[0].shape == lsingle.shape == (128, 4, 32, 32)
    assert torch.equal(lat[0], lsingle), float((lat[0] - lsingle).norm() / lsingle.norm())
    res = _run2("device", True, **kw)
    single = _job("device", True, **kw)
    assert res[1] is None and res[0].shape == single.shape == (128, 256, 256, 3)
    d = np.abs(res[0].numpy().astype(np.int32) - single.numpy().astype(np.int32))
    assert d.max() == 0, (int(d.max()), float((d > 0).mean()))


def test_sharded_sampler_latents_world2_host(cuda):
    res = _run2("host", decode=False)
    single = _job("host", decode=False)
    assert res[1] is None
    assert float((res[0] - single).norm() / single.norm()) < 1e-5


def test_sharded_world1_equals_diffuser_device_mode(cuda):
    """same seed -> same samples from ShardedCondSampler (world 1) and
    Diffuser.sample_latent_cond in device-noise mode (x_T drawn before the Philox seed in both)."""
    import diff
    from dmx import synth
    from models.unet_cond_geom import UnetCondWithGeomHead
    dev = torch.device("cuda:0")
    lat = _job("device", decode=False)
    m = UnetCondWithGeomHead()
    m.load_state_dict(synth.unet_cond_geom_weights(0))
    m.to(dev).eval()
    d = diff.Diffuser(4, device=dev)
    d.noise_source = "device"
    g = torch.Generator().manual_seed(40)
    vals = torch.rand((5, 12), generator=g).to(dev)
    mask = (torch.rand((5, 12), generator=g) > 0.3).float().to(dev)
    torch.manual_seed(41)
    ref_lat = d.sample_latent_cond(m, {1: 3, 3: 2}, z_shape=(4, 16, 16), vae=None, progress=False, cond=vals,
                                   cond_mask=mask)
    assert torch.equal(lat, ref_lat.cpu())


def test_sharded_world1_range_guard_equals_diffuser(cuda, unet_sd_overflow):
    """the sharded sampler runs the split-precision range guard.  An overflowing GroupNorm
    gamma trips it; world 1 must replay the chunk in fp32 exactly as Diffuser.sample_latent_cond."""
    import diff
    from dmx import distributed as dd
    from models.unet_cond_geom import UnetCondWithGeomHead
    dev = torch.device("cuda:0")
    outs = []
    for sharded in (True, False):
        m = UnetCondWithGeomHead()
        m.load_state_dict(unet_sd_overflow)
        m.to(dev).eval()
        d = diff.Diffuser(4, device=dev)
        g = torch.Generator().manual_seed(35)
        vals = torch.rand((2, 12), generator=g).to(dev)
        mask = torch.ones((2, 12), device=dev)
        torch.manual_seed(36)
        if sharded:
            s = dd.ShardedCondSampler(d, m, None)
            lat = s.sample({1: 1, 2: 1}, z_shape=(4, 16, 16), cond=vals, cond_mask=mask, decode=False)
            assert s.range_fallbacks == 1
        else:
            lat = d.sample_latent_cond(m, {1: 1, 2: 1}, z_shape=(4, 16, 16), vae=None, progress=False, cond=vals,
                                       cond_mask=mask)
            assert d.range_fallbacks == 1
        assert torch.isfinite(lat).all() and m.native().precision == "x3"
        outs.append(lat.cpu())
    assert torch.equal(outs[0], outs[1])


@pytest.fixture
def unet_sd_overflow():
    from dmx import synth
    sd = synth.unet_cond_geom_weights(0)
    sd["inc.double_conv.1.weight"] = sd["inc.double_conv.1.weight"] * 1e5
    return sd


# ---- data-parallel training step ----------------------------------
def _train_job(rank, world, B=4):
    """train_latent_cond.py's loss on this rank's half of a B = 4 batch (28x28x4 latents),
    loss.backward() through dmx_train_backward, then GradAllReducer (gloo here, RCCL in bench).
    The geom mask is NOT uniform (the two halves have different mask sums): the geom term is
    normalised by ``global_mask_mean`` (one scalar all-reduce), so the average of the two
    half-batch gradients is the full-batch gradient (up to fp32 summation order)."""
    import torch.nn.functional as F
    from dmx import distributed as dd
    from dmx import synth
    from losses.geom_losses import masked_geom_mse
    from models.unet_cond_geom import UnetCondWithGeomHead
    dev = torch.device("cuda:0")
    m = UnetCondWithGeomHead()
    m.load_state_dict(synth.unet_cond_geom_weights(0))
    m.to(dev).train()
    dd.broadcast_module(m)
    g = torch.Generator().manual_seed(90)
    z = torch.randn((B, 4, 28, 28), generator=g)
    t = torch.randint(1, 1001, (B,), generator=g)
    y = torch.randint(1, 4, (B,), generator=g)
    vals = torch.rand((B, 12), generator=g)
    noise = torch.randn((B, 4, 28, 28), generator=g)
    mask = (torch.rand((B, 12), generator=g) > 0.4).float()
    mask[:B // 2, :4] = 0.0  # rank 0's half holds fewer mask entries than rank 1's
    s, e = dd.shard_range(B, world, rank)
    sl = [a[s:e].to(dev) for a in (z, t, y, vals, mask, noise)]
    eps, geom = m(sl[0], sl[1], sl[2], cond_vals=sl[3], cond_mask=sl[4])
    denom = dd.global_mask_mean(sl[4]) if world > 1 else None
    loss = F.mse_loss(eps, sl[5]) + 0.5 * masked_geom_mse(geom, sl[3], sl[4], denom=denom)
    loss.backward()
    dd.GradAllReducer(m.parameters()).reduce()
    return {n: p.grad.detach().cpu() for n, p in m.named_parameters() if p.grad is not None}


def _train_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, {n: g.numpy() for n, g in _train_job(rank, world).items()}))  # by value, see _worker
    finally:
        dist.destroy_process_group()


def test_data_parallel_training_grads_world2_on_one_gpu(cuda):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: {n: torch.from_numpy(a) for n, a in g.items()} for r, g in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = _train_job(0, 1)
    assert set(res[0]) == set(res[1]) == set(single)
    for n, gs in single.items():
        assert torch.equal(res[0][n], res[1][n]), n  # replicas hold identical averaged gradients
        err = float((res[0][n] - gs).norm() / gs.norm().clamp_min(1e-30))
        assert err <= 1e-4, (n, err)  # the single-GPU native-gradient bound (test_gpu_train.py)
