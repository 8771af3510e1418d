"""HIP path vs the oracle / the reference's golden vectors (MI355X only).

Tolerances (fp32 everywhere):
  * single network forwards / single steps: rel-L2 <= 2e-5 (different but fp32-exact
    accumulation orders; measured ~1e-6)
  * latents after a full T=1000 CFG trajectory: rel-L2 <= 1e-4 (north-star bound)
  * decoded uint8 pixels: |diff| <= 1 LSB on <= 0.1% of values (truncating quantiser)
  * the DDPM/CFG update itself (given eps): bit-exact
"""
import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu

TOL = 2e-5


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def u8_close(a, b, frac=1e-3):
    d = np.abs(np.asarray(a, np.int32) - np.asarray(b, np.int32))
    return d.max() <= 1 and (d > 0).mean() <= frac, (int(d.max()), float((d > 0).mean()))


@pytest.fixture(scope="module")
def model(cuda, unet_sd):
    from models.unet_cond_geom import UnetCondWithGeomHead
    m = UnetCondWithGeomHead()
    m.load_state_dict(unet_sd)
    return m.to(cuda).eval()


@pytest.fixture(scope="module")
def vae(cuda, vae_sd):
    from models.vae import VAE
    v = VAE()
    v.load_state_dict(vae_sd)
    return v.to(cuda).eval()


def test_library_is_native(cuda):
    import ctypes
    from dmx import _lib
    lib = _lib.load()
    assert lib.dmx_abi_version() == 1
    assert isinstance(lib, ctypes.CDLL)


@pytest.fixture(params=["x3", "fp32"])
def prec(request, model):
    """Both GEMM arithmetics: fp16 hi/lo x3 split (default) and fp32 MFMA."""
    nm = model.native()
    old = nm.precision
    nm.set_precision(request.param)
    yield request.param
    nm.set_precision(old)


@pytest.mark.parametrize("name", ["forward_32.npz", "forward_28.npz"])
def test_unet_forward_golden(golden, model, cuda, name, prec):
    g = golden(name)
    dev = lambda k: torch.from_numpy(g[k]).to(cuda)
    with torch.no_grad():
        eps, geom = model(dev("x"), dev("t"), dev("y"), cond_vals=dev("vals"), cond_mask=dev("mask"))
    assert rel(eps, g["eps"]) < TOL
    assert rel(geom, g["geom"]) < TOL


def test_unet_forward_vs_oracle_no_cond(model, cuda, unet_sd):
    g = torch.Generator().manual_seed(3)
    x = torch.randn((5, 4, 32, 32), generator=g)
    t = torch.tensor([1, 2, 500, 999, 1000])
    y = torch.tensor([0, 1, 2, 3, 1])
    with torch.no_grad():
        eps, geom = model(x.to(cuda), t.to(cuda), y.to(cuda))
        e2, g2 = ref.unet_cond_geom_forward(unet_sd, x, t, y)
    assert rel(eps, e2) < TOL and rel(geom, g2) < TOL


@pytest.mark.parametrize("hw", [32, 28, 20])
def test_unet_forward_bench_batch_vs_oracle(model, cuda, unet_sd, prec, hw):
    """One forward of 128 samples (the CFG batch of B=64): the batch at which the 16x16 / 32x32 convs
    take their large-grid kernels — in x3 mode the Winograd F(2x2, 3x3) convs (igemm_wino.h) — checked
    on eps itself (a CFG step's latent hides eps errors behind its (1-a)/sqrt(1-ab) factor).  28x28:
    the 28 / 14 / 7 / 3 maps in the Winograd geometries of 32 / 16 / 8 / 4 (zero-padded rows and
    columns, partial GroupNorm rows) and the Up path's pad; 20x20: 20 / 10 / 5 / 2 maps (a 2 x 2 map in
    the 4-wide geometry, 5 x 5 in the 8-wide one, 3 bands of which the last holds 4 rows)."""
    g = torch.Generator().manual_seed(128 + hw)
    N = 128
    x = torch.randn((N, 4, hw, hw), generator=g)
    t = torch.randint(1, 1001, (N,), generator=g)
    y = torch.randint(0, 4, (N,), generator=g)
    vals = torch.rand((N, 12), generator=g)
    mask = (torch.rand((N, 12), generator=g) > 0.5).float()
    with torch.no_grad():
        eps, geom = model(x.to(cuda), t.to(cuda), y.to(cuda), cond_vals=vals.to(cuda), cond_mask=mask.to(cuda))
        e2, g2 = ref.unet_cond_geom_forward(unet_sd, x, t, y, vals, mask)
    ee, eg = rel(eps, e2), rel(geom, g2)
    print(f"[forward N=128 {hw}x{hw} {prec}] eps rel-L2 {ee:.2e}, geom {eg:.2e}")
    assert ee < TOL and eg < TOL


def test_bench_batch_forward_is_deterministic(model, cuda):
    """Five repeats of the N = 128 forward are bit-identical (the large-grid kernels — Winograd convs
    with GroupNorm-on-load, split-K slabs — must not race: a race shows up as run-to-run drift of a
    few samples; tools/det_check.py is the longer version of this check)."""
    g = torch.Generator().manual_seed(129)
    N = 128
    x = torch.randn((N, 4, 32, 32), generator=g).to(cuda)
    t = torch.randint(1, 1001, (N,), generator=g).to(cuda)
    y = torch.randint(0, 4, (N,), generator=g).to(cuda)
    vals = torch.rand((N, 12), generator=g).to(cuda)
    mask = (torch.rand((N, 12), generator=g) > 0.5).float().to(cuda)
    outs = []
    with torch.no_grad():
        for _ in range(5):
            eps, geom = model(x, t, y, cond_vals=vals, cond_mask=mask)
            outs.append((eps.cpu(), geom.cpu()))
    for e, gm in outs[1:]:
        assert torch.equal(e, outs[0][0]) and torch.equal(gm, outs[0][1])


def test_large_batch_class_is_shard_exact(model, cuda):
    """A 512-sample forward (a single-process B = 256 CFG batch) takes the 128-sample class decisions
    (engine.hip dec_n): samples 0..127 come out bit-identical to a 128-sample forward of the same
    inputs, and the workspace grows linearly with the batch (split slabs of splits * M * Cout floats;
    ADVICE r4: bound it)."""
    g = torch.Generator().manual_seed(512)
    N = 512
    x = torch.randn((N, 4, 32, 32), generator=g).to(cuda)
    t = torch.randint(1, 1001, (N,), generator=g).to(cuda)
    y = torch.randint(0, 4, (N,), generator=g).to(cuda)
    vals = torch.rand((N, 12), generator=g).to(cuda)
    mask = (torch.rand((N, 12), generator=g) > 0.5).float().to(cuda)
    nm = model.native()
    with torch.no_grad():
        e128, g128 = model(x[:128], t[:128], y[:128], cond_vals=vals[:128], cond_mask=mask[:128])
        ws128 = nm.workspace_bytes()
        e512, g512 = model(x, t, y, cond_vals=vals, cond_mask=mask)
        ws512 = nm.workspace_bytes()
    print(f"[batch class] workspace 128: {ws128 / 2**30:.2f} GiB, 512: {ws512 / 2**30:.2f} GiB")
    assert torch.equal(e512[:128], e128) and torch.equal(g512[:128], g128)
    assert ws512 <= 4.2 * ws128


def test_uncond_unet_golden(golden, cuda):
    from dmx import synth
    from models.unet import Unet
    m = Unet(in_ch=4)
    m.load_state_dict(synth.unet_weights(0, in_ch=4))
    m.to(cuda).eval()
    g = golden("forward_uncond.npz")
    with torch.no_grad():
        eps = m(torch.from_numpy(g["x"]).to(cuda), torch.from_numpy(g["t"]).to(cuda))
    assert rel(eps, g["eps"]) < TOL


def test_vae_decode_golden(golden, vae, cuda):
    g = golden("vae_decode.npz")
    with torch.no_grad():
        img16 = vae.decode(torch.from_numpy(g["z16"]).to(cuda))
        u8 = vae.decode_uint8(torch.from_numpy(g["z32"]).to(cuda))
    assert rel(img16, g["img16"]) < TOL
    ok, info = u8_close(u8.cpu().numpy(), g["u8_32"])
    assert ok, info


@pytest.mark.parametrize("tag", ["64", "56"])
@pytest.mark.parametrize("vprec", ["x3", "fp32"])
def test_vae_encode_golden(golden, vae, vae_sd, cuda, tag, vprec):
    """VAE.encode (models/vae.py:51-62; conv4x4-s2 implicit GEMM) vs the reference's outputs, including
    its randn_like draw: z rel-L2 <= 2e-5, KL rel <= 2e-5; the global RNG advanced like the reference."""
    g = golden("vae_encode.npz")
    nm = vae.native()
    old = nm.precision
    nm.set_precision(vprec)
    try:
        x = torch.from_numpy(g[f"x{tag}"]).to(cuda)
        torch.manual_seed(int(g[f"seed{tag}"]))
        eps = torch.randn(g[f"eps{tag}"].shape).to(cuda)  # the draw the drop-in makes on `cuda`
        zn, kln = nm.encode(x, eps)
        exp_z = ref.vae_encode(vae_sd, x.cpu(), eps.cpu())[0]
        assert rel(zn, exp_z) < TOL
        eg = torch.from_numpy(g[f"eps{tag}"])
        zg, klg = nm.encode(x, eg.to(cuda))
        assert rel(zg, g[f"z{tag}"]) < TOL
        assert abs(float(klg.mean()) - float(g[f"kl{tag}"])) <= TOL * abs(float(g[f"kl{tag}"]))
    finally:
        nm.set_precision(old)


def test_vae_encode_dropin_draws_like_reference(vae, cuda):
    """VAE.encode draws eps with torch on x's device: the RNG state afterwards equals one randn of z's shape."""
    x = torch.rand((2, 3, 32, 32), generator=torch.Generator().manual_seed(5)).to(cuda)
    torch.manual_seed(9)
    z, kl = vae.encode(x)
    after = torch.randn(3, device=cuda)
    torch.manual_seed(9)
    _ = torch.randn((2, 4, 4, 4), device=cuda)
    assert torch.equal(after, torch.randn(3, device=cuda))
    assert z.shape == (2, 4, 4, 4) and kl.dim() == 0 and torch.isfinite(z).all()


def test_vae_forward_vs_oracle(golden, vae, vae_sd, cuda):
    """Drop-in VAE.forward (models/vae.py:71-76: encode -> decode -> MSE + 1e-6 KL) vs the oracle given
    the same randn_like draw: x_recon, z and loss rel <= 2e-5."""
    g = golden("vae_encode.npz")
    x = torch.from_numpy(g["x64"]).to(cuda)
    torch.manual_seed(3)
    with torch.no_grad():
        x_recon, z, loss, parts = vae(x)
    torch.manual_seed(3)
    eps = torch.randn(z.shape, device=cuda).cpu()
    exp_recon, exp_z, exp_loss, exp_mse, exp_kl = ref.vae_forward(vae_sd, x.cpu(), eps)
    assert rel(z, exp_z) < TOL and rel(x_recon, exp_recon) < TOL
    assert abs(float(loss) - float(exp_loss)) <= TOL * abs(float(exp_loss))
    assert abs(float(parts["kl"]) - float(exp_kl)) <= TOL * abs(float(exp_kl))


def test_vae_decode_vs_oracle_odd_batch(vae, cuda, vae_sd):
    z = torch.randn((3, 4, 8, 8), generator=torch.Generator().manual_seed(4))
    with torch.no_grad():
        img = vae.decode(z.to(cuda))
        exp = ref.vae_decode(vae_sd, z)
    assert rel(img, exp) < TOL


@pytest.mark.parametrize("hw", [16, 32])
@pytest.mark.parametrize("vprec", ["x3", "fp32"])
def test_vae_decode_batch_invariant(vae, cuda, hw, vprec):
    """a latent's decoded image does not depend on the batch it is decoded in —
    the same 5 latents decoded as n=5, as n=3 + n=2 and one by one give identical fp32 images and
    uint8 bytes (the decoder's tile / split-K decisions are per sample; diff.py:353 decodes in
    chunks of 4, the sharded sampler in shards of any size)."""
    nat = vae.native()
    z = torch.randn((5, 4, hw, hw), generator=torch.Generator().manual_seed(6)).to(cuda)

    def dec(zz):
        img, u8 = nat.decode(zz.contiguous(), want_img=True, want_u8=True)
        return img.cpu(), u8.cpu()

    with nat.precision_override(vprec):
        full = dec(z)
        parts = [dec(z[:3]), dec(z[3:])]
        ones = [dec(z[i:i + 1]) for i in range(5)]
    for split in (parts, ones):
        assert torch.equal(torch.cat([p[0] for p in split]), full[0])
        assert torch.equal(torch.cat([p[1] for p in split]), full[1])


def test_denoise_cond_golden_steps(golden, model, cuda):
    import diff
    g = golden("denoise_cond.npz")
    d = diff.Diffuser(1000, device=cuda)
    x = torch.from_numpy(g["x"]).to(cuda)
    y = torch.from_numpy(g["y"]).to(cuda)
    vals, mask = torch.from_numpy(g["vals"]).to(cuda), torch.from_numpy(g["mask"]).to(cuda)
    for tv in (1000, 500, 2, 1):
        t = torch.full((2,), tv, dtype=torch.long, device=cuda)
        torch.manual_seed(100 + tv)  # same global-generator draw as the reference
        out = d.denoise_cond(model, x, t, y=y, guidance_scale=3.0, null_label=0, cond_vals=vals, cond_mask=mask)
        assert rel(out, g[f"out_{tv}"]) < TOL, tv


def test_ddpm_update_bit_exact(cuda):
    """K1 given eps: one rounding per reference op, same order => bit-identical to torch-CPU."""
    import diff
    from dmx import engine
    d = diff.Diffuser(1000, device=cuda)
    g = torch.Generator().manual_seed(9)
    B = 6
    x, eu, ec, nz = (torch.randn((B, 4, 16, 16), generator=g) for _ in range(4))
    t = torch.tensor([1, 2, 3, 500, 999, 1000])
    out = engine.ddpm_update(x.to(cuda), eu.to(cuda), ec.to(cuda), 3.0, t.to(cuda),
                             d.coef_tables(cuda, True), nz.to(cuda)).cpu()
    _, a, ab = ref.schedule(1000)
    eps = eu + 3.0 * (ec - eu)
    exp = ref.ddpm_update(x, eps, t, a, ab, nz)
    assert torch.equal(out, exp)
    # unconditional variant (diff.py:39 wrap-around alpha_bar_prev)
    out2 = engine.ddpm_update(x.to(cuda), eu.to(cuda), None, 0.0, t.to(cuda), d.coef_tables(cuda, False),
                              nz.to(cuda)).cpu()
    assert torch.equal(out2, ref.ddpm_update(x, eu, t, a, ab, nz, clamp_prev=False))


def test_cfg_step_full_batch_vs_oracle(model, cuda, unet_sd, prec):
    """One CFG step at the benchmark shape B=64, 32x32x4 (2B = 128 sample-forwards)."""
    import diff
    d = diff.Diffuser(1000, device=cuda)
    g = torch.Generator().manual_seed(21)
    B = 64
    x = torch.randn((B, 4, 32, 32), generator=g)
    y = torch.tensor([1 + i % 3 for i in range(B)])
    vals = torch.rand((B, 12), generator=g)
    mask = (torch.rand((B, 12), generator=g) > 0.5).float()
    t = torch.full((B,), 640, dtype=torch.long)
    torch.manual_seed(77)
    out = d.denoise_cond(model, x.to(cuda), t.to(cuda), y=y.to(cuda), guidance_scale=3.0,
                         cond_vals=vals.to(cuda), cond_mask=mask.to(cuda))
    torch.manual_seed(77)
    noise = torch.randn(x.shape)
    _, a, ab = ref.schedule(1000)
    with torch.no_grad():
        exp = ref.cfg_step(unet_sd, x, t, y, a, ab, 3.0, 0, vals, mask, noise)
    assert rel(out, exp) < TOL


@pytest.mark.parametrize("B,hw", [(3, 32), (9, 32), (5, 16), (33, 32), (33, 28)])
def test_cfg_step_ragged_batches_vs_oracle(model, cuda, unet_sd, B, hw):
    """Batches that are not a multiple of the low-resolution halo convs' whole-sample tiles (16
    samples of 4 x 4, 4 of 8 x 8: igemm_halo.h MS) — the last tile holds fewer samples, which stage
    as zeros and whose rows the epilogue drops — and the split-K slab reduction behind them.
    B = 33 (a 66-sample CFG forward) is in the benchmark's batch class (>= 64 samples): its 3x3 convs
    run the Winograd kernels, whose 8 x 8 blocks stack four samples, so the last block holds 2
    (igemm_wino.h nsamp guards).  B = 33 at 28x28: the same with the maps narrower
    than the Winograd geometries (7 x 7 in the 8-wide blocks, 3 x 3 in the 4-wide ones)."""
    import diff
    d = diff.Diffuser(1000, device=cuda)
    g = torch.Generator().manual_seed(300 + B)
    x = torch.randn((B, 4, hw, hw), generator=g)
    y = torch.tensor([1 + i % 3 for i in range(B)])
    vals = torch.rand((B, 12), generator=g)
    mask = (torch.rand((B, 12), generator=g) > 0.5).float()
    t = torch.full((B,), 333, dtype=torch.long)
    torch.manual_seed(78)
    out = d.denoise_cond(model, x.to(cuda), t.to(cuda), y=y.to(cuda), guidance_scale=3.0,
                         cond_vals=vals.to(cuda), cond_mask=mask.to(cuda))
    torch.manual_seed(78)
    noise = torch.randn(x.shape)
    _, a, ab = ref.schedule(1000)
    with torch.no_grad():
        exp = ref.cfg_step(unet_sd, x, t, y, a, ab, 3.0, 0, vals, mask, noise)
    err = rel(out, exp)
    print(f"[ragged B={B} {hw}x{hw}] CFG step rel-L2 vs oracle {err:.2e}")
    assert err < TOL


def test_trajectory_T1000_golden(golden, model, vae, cuda, prec):
    """Full T=1000 CFG trajectory (B=2) on the reference's own draws: latents <= 1e-4, pixels +-1."""
    import diff
    g = golden("traj_T1000_B2.npz")
    d = diff.Diffuser(1000, device=cuda)
    y = torch.from_numpy(g["y"]).to(cuda)
    vals, mask = torch.from_numpy(g["vals"]).to(cuda), torch.from_numpy(g["mask"]).to(cuda)
    torch.manual_seed(int(g["seed"]))
    x = torch.randn((2, 4, 32, 32)).to(cuda)
    for i in range(1000, 0, -1):
        t = torch.full((2,), i, dtype=torch.long, device=cuda)
        x = d.denoise_cond(model, x, t, y=y, guidance_scale=3.0, null_label=0, cond_vals=vals, cond_mask=mask)
        if i in (900, 500, 100):
            assert rel(x, g[f"x_{i}"]) < 1e-4, i
    err = rel(x, g["x_final"])
    u8 = vae.decode_uint8(x).cpu().numpy()
    ok, info = u8_close(u8, g["u8"])
    print(f"[trajectory T=1000 {prec}] final latents rel-L2 vs reference {err:.2e}, pixels {info}")
    assert err < 1e-4
    assert ok, info


@pytest.mark.parametrize("name", ["traj_T1000_B32.npz", "traj_T1000_B32_28.npz"])
def test_trajectory_T1000_B32_winograd_class_golden(golden, model, vae, cuda, name):
    """T=1000 CFG trajectory at B=32 (a 64-sample CFG forward: the batch class whose 3x3 convs run the
    Winograd kernels bench.py times) on the reference's own draws (tests/golden/make_golden_r5.py,
    diff.py:326-344 loop of denoise_cond): latents at t = 900 / 500 / 100 (samples 0..7) and after
    t = 1 (all 32) within 1e-4 rel-L2, decoded uint8 images of samples 0..5 within +-1 LSB on <= 0.1 %.
    x3 mode (the default, fp32 semantics).  traj_T1000_B32_28.npz: the same at
    28x28 latents (the reference sampler's shape; Winograd geometries with zero-padded columns)."""
    import diff
    g = golden(name)
    nm = model.native()
    assert nm.precision == "x3"
    B, sub = int(g["y"].shape[0]), int(g["sub"])
    d = diff.Diffuser(1000, device=cuda)
    y = torch.from_numpy(g["y"]).to(cuda)
    vals, mask = torch.from_numpy(g["vals"]).to(cuda), torch.from_numpy(g["mask"]).to(cuda)
    torch.manual_seed(int(g["seed"]))
    hw = int(g["x_final"].shape[-1])
    x = torch.randn((B, 4, hw, hw)).to(cuda)
    errs = {}
    for i in range(1000, 0, -1):
        t = torch.full((B,), i, dtype=torch.long, device=cuda)
        x = d.denoise_cond(model, x, t, y=y, guidance_scale=3.0, null_label=0, cond_vals=vals, cond_mask=mask)
        if i in (900, 500, 100):
            errs[i] = rel(x[:sub], g[f"x_{i}"])
    errs[1] = rel(x, g["x_final"])
    n_img = int(g["u8"].shape[0])
    u8 = vae.decode_uint8(x[:n_img].contiguous()).cpu().numpy()
    ok, info = u8_close(u8, g["u8"])
    print(f"[trajectory T=1000 B=32 {hw}x{hw} x3] latents rel-L2 vs reference {errs}, pixels {info}")
    assert all(e < 1e-4 for e in errs.values()), errs
    assert ok, info


def test_sample_latent_cond_T20_28_path(golden, model, vae, cuda):
    """z_shape=None (28x28 latents via the replayed encode draw), pixels via PIL, and z_shape given."""
    import diff
    g = golden("sample_T20.npz")
    d = diff.Diffuser(20, device=cuda)
    torch.manual_seed(int(g["seed"]))
    imgs = d.sample_latent_cond(model, (2, 2), vae=vae, to_pil=True, progress=False, guidance_scale=3.0,
                                cond=torch.from_numpy(g["vals"]).to(cuda), cond_mask=torch.from_numpy(g["mask"]).to(cuda))
    u8 = np.stack([np.asarray(im) for im in imgs])
    ok, info = u8_close(u8, g["u8_28"])
    assert ok, info
    torch.manual_seed(int(g["seed"]))
    lat = d.sample_latent_cond(model, {1: 1, 3: 1}, z_shape=(4, 32, 32), vae=None, progress=False)
    assert rel(lat, g["latent_32"]) < 1e-4


def test_uncond_sample_latent_T100_golden(golden, cuda):
    """Config 1: unconditional Unet, T=100, B=4 (diff.py:87-125)."""
    import diff
    from dmx import synth
    from models.unet import Unet
    m = Unet(in_ch=4)
    m.load_state_dict(synth.unet_weights(0, in_ch=4))
    m.to(cuda).eval()
    g = golden("uncond_T100.npz")
    d = diff.Diffuser(100, device=cuda)
    torch.manual_seed(int(g["seed"]))
    z = d.sample_latent(m, z_shape=(4, 4, 32, 32), vae=None, progress=False)
    assert rel(z, g["latent"]) < 1e-4


@pytest.mark.parametrize("B,hw", [(4, 32), (64, 32), (64, 28)])
def test_graph_loop_equals_eager_and_is_deterministic(model, cuda, B, hw):
    """Device-noise mode: hipGraph replay == eager launches, bit for bit, and reruns are identical
    (19 steps: two launches of the 8-step graph and three of the one-step graph).  B = 64 is the
    benchmark's timed region (bench.py: the 8-step graph at B = 64 — Winograd convs, Philox noise,
    cond-MLP rows computed once per graph); (64, 28): bench.py's latent28 leg."""
    from dmx import engine  # noqa: F401
    import diff
    d = diff.Diffuser(1000, device=cuda)
    nm = model.native()
    g = torch.Generator().manual_seed(2)
    x0 = torch.randn((B, 4, hw, hw), generator=g).to(cuda)
    y = torch.tensor([1 + i % 3 for i in range(B)], device=cuda)
    vals = torch.rand((B, 12), generator=g).to(cuda)
    mask = (torch.rand((B, 12), generator=g) > 0.3).float().to(cuda) if B > 4 else torch.ones((B, 12), device=cuda)
    tables = d.coef_tables(cuda, True)
    outs = []
    for use_graph in (True, False, True):
        x = x0.clone()
        t = torch.full((1,), 1000, dtype=torch.long, device=cuda)
        nm.sample_loop(x, t, y, 0, vals, mask, 3.0, tables, 19, seed=1234, use_graph=use_graph)
        torch.cuda.synchronize()
        assert int(t.item()) == 981
        outs.append(x.cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert torch.isfinite(outs[0]).all()


def test_philox_noise_statistics_and_shard_invariance(model, cuda):
    """Perf-mode noise: N(0,1) moments, and sample i's noise does not depend on the shard it runs in."""
    from dmx import engine
    import diff
    d = diff.Diffuser(1000, device=cuda)
    B = 8
    x = torch.zeros((B, 4, 32, 32), device=cuda)
    eu = torch.zeros_like(x)
    t = torch.full((B,), 2, dtype=torch.long, device=cuda)
    tab = d.coef_tables(cuda, True)
    full = engine.ddpm_update(x, eu, None, 0.0, t, tab, None, seed=99, sample_offset=0)
    part = engine.ddpm_update(x[4:], eu[4:], None, 0.0, t[4:], tab, None, seed=99, sample_offset=4)
    assert torch.equal(full[4:], part)
    z = (full / tab[2][1]).flatten().double()
    assert abs(float(z.mean())) < 0.02 and abs(float(z.std()) - 1.0) < 0.02


def test_edge_cases_batch1_per_sample_t_nonzero_null(model, cuda, unet_sd):
    import diff
    d = diff.Diffuser(1000, device=cuda)
    for B, tv, null in ((1, [1], 0), (3, [1, 500, 1000], 2)):
        g = torch.Generator().manual_seed(B)
        x = torch.randn((B, 4, 32, 32), generator=g)
        y = torch.tensor([3, 1, 2][:B])
        vals = torch.rand((B, 12), generator=g)
        mask = torch.ones((B, 12))
        t = torch.tensor(tv)
        torch.manual_seed(11)
        out = d.denoise_cond(model, x.to(cuda), t.to(cuda), y=y.to(cuda), guidance_scale=2.5, null_label=null,
                             cond_vals=vals.to(cuda), cond_mask=mask.to(cuda))
        torch.manual_seed(11)
        _, a, ab = ref.schedule(1000)
        with torch.no_grad():
            exp = ref.cfg_step(unet_sd, x, t, y, a, ab, 2.5, null, vals, mask, torch.randn(x.shape))
        assert rel(out, exp) < TOL, B


def test_reference_error_behaviour(model, cuda):
    import diff
    d = diff.Diffuser(1000, device=cuda)
    x = torch.zeros((1, 4, 32, 32), device=cuda)
    y = torch.ones((1,), dtype=torch.long, device=cuda)
    with pytest.raises(AssertionError):
        d.denoise_cond(model, x, torch.tensor([0], device=cuda), y=y, guidance_scale=3.0)
    with pytest.raises(AssertionError):
        d.denoise_cond(model, x, torch.tensor([1001], device=cuda), y=y, guidance_scale=3.0)
    with pytest.raises(UnboundLocalError):  # diff.py:152-156 with y given and guidance 0
        d.denoise_cond(model, x, torch.tensor([5], device=cuda), y=y, guidance_scale=0.0)
    with pytest.raises(TypeError):  # y=None: eps is the (eps, geom) tuple of the geom model
        d.denoise_cond(model, x, torch.tensor([5], device=cuda), y=None, guidance_scale=0.0)
    with pytest.raises(ValueError):
        d.sample_latent_cond(model, {1: 0}, z_shape=(4, 32, 32))
