"""Diagnostic: does a sample's result depend on the batch it is computed in?

One process, deterministic:
  1. VAE decode of the same 5 latents as n=5, as n=3 + n=2, and one by one (uint8 + fp32);
  2. one host-noise CFG step of the same 5 samples as n=5 and as n=3 + n=2;
  3. the test_gpu_multi host-mode job with the two shards run one after another in this process
     (world faked to 2) against the single-process job — latents and images.
Then the real two-process rehearsal, with each rank's pre-gather latents saved."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "diffusion-model_amd"), REPO, os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def cmp_u8(a, b):
    d = np.abs(a.astype(np.int32) - b.astype(np.int32))
    return int(d.max()), float((d > 0).mean())


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def decode_dep():
    from dmx import synth
    from models.vae import VAE
    dev = torch.device("cuda:0")
    v = VAE()
    v.load_state_dict(synth.vae_weights(1))
    v.to(dev).eval()
    nat = v.native()
    g = torch.Generator().manual_seed(5)
    z = torch.randn((5, 4, 16, 16), generator=g).to(dev)

    def dec(zz):
        img, u8 = nat.decode(zz.contiguous(), want_img=True, want_u8=True)
        return img.cpu(), u8.cpu().numpy()

    i5, u5 = dec(z)
    a, b = dec(z[:3]), dec(z[3:])
    i32, u32 = torch.cat([a[0], b[0]]), np.concatenate([a[1], b[1]])
    ones = [dec(z[i:i + 1]) for i in range(5)]
    i1, u1 = torch.cat([o[0] for o in ones]), np.concatenate([o[1] for o in ones])
    print("decode n5 vs 3+2: img equal", torch.equal(i5, i32), "rel", rel(i32, i5), "u8", cmp_u8(u32, u5), flush=True)
    print("decode n5 vs 1x5: img equal", torch.equal(i5, i1), "rel", rel(i1, i5), "u8", cmp_u8(u1, u5), flush=True)
    i5b, u5b = dec(z)
    print("decode n5 repeat: equal", torch.equal(i5, i5b), cmp_u8(u5b, u5), flush=True)
    return nat, z


def step_dep():
    import diff
    from dmx import synth
    from models.unet_cond_geom import UnetCondWithGeomHead
    dev = torch.device("cuda:0")
    m = UnetCondWithGeomHead()
    m.load_state_dict(synth.unet_cond_geom_weights(0))
    m.to(dev).eval()
    nm = m.native()
    d = diff.Diffuser(4, device=dev)
    tables = d.coef_tables(dev, clamp_prev=True)
    g = torch.Generator().manual_seed(7)
    x = torch.randn((5, 4, 16, 16), generator=g).to(dev)
    noise = torch.randn((5, 4, 16, 16), generator=g).to(dev)
    vals = torch.rand((5, 12), generator=g).to(dev)
    msk = (torch.rand((5, 12), generator=g) > 0.3).float().to(dev)
    y = torch.tensor([1, 1, 1, 3, 3], device=dev)

    def st(s, e, t):
        out = torch.empty_like(x[s:e])
        tt = torch.full((e - s,), t, dtype=torch.long, device=dev)
        nm.step(x[s:e].contiguous(), out, tt, y[s:e], 0, vals[s:e].contiguous(), msk[s:e].contiguous(), 3.0,
                tables, noise[s:e].contiguous())
        torch.cuda.synchronize()
        return out.cpu()

    for t in (4, 1):
        full = st(0, 5, t)
        part = torch.cat([st(0, 3, t), st(3, 5, t)])
        print(f"step t={t} n5 vs 3+2: equal", torch.equal(full, part), "rel", rel(part, full), flush=True)


def fake_sharded(mode, decode):
    """test_gpu_multi._job with world faked to 2: both shards in this process, one after the other."""
    from dmx import distributed as dd
    import test_gpu_multi as tm
    saved = (dd.world, dd.gather_rows)
    outs = []
    try:
        for r in range(2):
            dd.world = (lambda rr: (lambda: (2, rr)))(r)
            dd.gather_rows = lambda local, total, dst=0: local
            outs.append(tm._job(mode, decode))
    finally:
        dd.world, dd.gather_rows = saved
    return torch.cat(outs)


def real_two_process(mode):
    """The test's two-rank run; every rank's decode input (its final latents) is saved beside the images."""
    import test_gpu_multi as tm
    return tm._run2(mode, decode=True)


if __name__ == "__main__":
    decode_dep()
    step_dep()
    import test_gpu_multi as tm
    for mode in ("host", "device"):
        single_lat = tm._job(mode, decode=False)
        single_img = tm._job(mode, decode=True).numpy()
        for rep in range(2):
            fl = fake_sharded(mode, decode=False)
            fi = fake_sharded(mode, decode=True).numpy()
            print(f"{mode} rep{rep} in-process shards: latents equal", torch.equal(fl, single_lat), "rel",
                  rel(fl, single_lat), "u8", cmp_u8(fi, single_img), flush=True)
        for rep in range(3):
            r = real_two_process(mode)[0].numpy()
            print(f"{mode} rep{rep} two-process: u8", cmp_u8(r, single_img), flush=True)
