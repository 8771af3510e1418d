"""Diagnostic: VAE decode (uint8) determinism — repeated in one process, and in two concurrent
processes on the same GPU (each decoding the same latents)."""
import os
import socket
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "diffusion-model_amd"), REPO):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def dec(reps=4, B=3):
    from dmx import synth
    from models.vae import VAE
    dev = torch.device("cuda:0")
    v = VAE()
    v.load_state_dict(synth.vae_weights(1))
    v.to(dev).eval()
    g = torch.Generator().manual_seed(5)
    z = torch.randn((B, 4, 16, 16), generator=g).to(dev)
    outs = []
    for _ in range(reps):
        _, u8 = v.native().decode(z, want_img=False, want_u8=True)
        img, _ = v.native().decode(z, want_img=True, want_u8=False)
        outs.append((u8.cpu().numpy(), img.cpu().numpy()))
    return outs


def worker(rank, q):
    q.put((rank, dec()))


def cmp(a, b):
    d = np.abs(a[0].astype(np.int32) - b[0].astype(np.int32))
    return int(d.max()), float((d > 0).mean()), float(np.abs(a[1] - b[1]).max())


if __name__ == "__main__":
    import torch.multiprocessing as mp
    single = dec()
    print("single repeats:", [cmp(single[0], s) for s in single[1:]], flush=True)
    ctx = mp.get_context("spawn")
    for rep in range(3):
        q = ctx.Queue()
        ps = [ctx.Process(target=worker, args=(r, q)) for r in range(2)]
        for p in ps:
            p.start()
        res = dict(q.get(timeout=200) for _ in ps)
        for p in ps:
            p.join()
        print(rep, "concurrent vs single:", [cmp(single[0], s) for r in (0, 1) for s in res[r]], flush=True)
