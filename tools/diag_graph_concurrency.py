"""Diagnostic: do the parallel branches of a captured hipGraph run concurrently on MI355X?
Two chains of K small latency-bound kernels (torch elementwise ops on 64 KB tensors), captured
(a) both on one stream, (b) on two streams forked / joined inside the capture; replay times."""
import time

import torch


def chain(x, k):
    for _ in range(k):
        x.mul_(1.0000001).add_(1e-7)


def timed(g, reps=50):
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


if __name__ == "__main__":
    dev = torch.device("cuda:0")
    K = 100
    for n in (16384, 4 * 1024 * 1024):
        a = torch.ones(n, device=dev)
        b = torch.ones(n, device=dev)
        s0 = torch.cuda.Stream()
        s1 = torch.cuda.Stream()
        # warm
        with torch.cuda.stream(s0):
            chain(a, 2)
            chain(b, 2)
        torch.cuda.synchronize()
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1, stream=s0):
            chain(a, K)
            chain(b, K)
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2, stream=s0):
            ev = torch.cuda.Event()
            ev.record(s0)
            s1.wait_event(ev)
            chain(a, K)
            with torch.cuda.stream(s1):
                chain(b, K)
            ev2 = torch.cuda.Event()
            ev2.record(s1)
            s0.wait_event(ev2)
        g0 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g0, stream=s0):
            chain(a, K)
        t1, t2, t0 = timed(g1), timed(g2), timed(g0)
        print(f"n={n}: one chain {t0:.1f} us, two chains serial {t1:.1f} us, two chains forked {t2:.1f} us "
              f"(concurrency gain {t1 / t2:.2f}x)", flush=True)
