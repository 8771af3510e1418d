"""Multi-GPU paths (one process per GPU, torch.distributed / RCCL over xGMI).

Sampling is sample-sharded; training is data-parallel (``GradAllReducer``, SURVEY.md §8f
rank 2: every rank runs the train_latent_cond.py step on its own micro-batch, gradients
are averaged with bucketed all-reduces before the optimizer step).

The CFG loop has no cross-sample coupling (GroupNorm/LayerNorm are per sample), so a
job of B samples is split into contiguous shards [start, end) per rank:

  * C1 — frozen weights are broadcast once from rank 0 (``broadcast_module``);
  * no per-step collective;
  * C2 — decoded images / latents are gathered once at the end (``gather_rows``).

Noise stays shard-invariant in both modes:
  * ``"device"``: Philox keyed by the *global* sample index (``sample_offset = start``);
  * ``"host"``: every rank draws the full global (B, C, H, W) tensor from the CPU
    generator each step and keeps its slice — torch.randn is prefix-stable, so every
    sample sees exactly the draw the single-process reference would give it.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import torch
import torch.distributed as dist


def _diff():
    """The drop-in sampler module (diffusion-model_amd/diff.py), imported from this package's
    parent directory whatever sys.path holds (the host-noise sharded loop needs its prefetcher)."""
    try:
        import diff
        return diff
    except ImportError:
        import importlib.util
        import os
        import sys
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "diff.py")
        spec = importlib.util.spec_from_file_location("diff", path)
        if "diff" in sys.modules:  # (registered by another importer meanwhile)
            return sys.modules["diff"]
        mod = importlib.util.module_from_spec(spec)
        # registered while it executes (its own imports may resolve "diff"), removed again if
        # executing it fails, so no half-initialised module stays behind for a later `import diff`
        sys.modules["diff"] = mod
        try:
            spec.loader.exec_module(mod)
        except BaseException:
            if sys.modules.get("diff") is mod:
                del sys.modules["diff"]
            raise
        return mod


def world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def shard_range(total: int, world_size: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [start, end) of `total` samples for `rank` (first ranks get the extra)."""
    base, extra = divmod(total, world_size)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def broadcast_module(module: torch.nn.Module, src: int = 0) -> None:
    """C1: broadcast every parameter/buffer of `module` from `src` once per job, packed: the
    tensors of each (device, dtype) are flattened into ONE contiguous buffer and sent with one
    ``dist.broadcast`` (191 U-Net tensors = one 93.7 MB message instead of 191 small ones; on
    xGMI's point-to-point links a broadcast is per-link bound, so one large message is the cheap
    form).  gloo has no CUDA broadcast path here: its buffer travels through host memory."""
    tensors = list(module.parameters()) + list(module.buffers())
    broadcast_tensors([t.data for t in tensors], src=src)


def broadcast_tensors(tensors: List[torch.Tensor], src: int = 0) -> int:
    """Broadcast `tensors` from `src` in place as one flattened buffer per (device, dtype) group;
    returns the number of collectives issued (0 at world size 1)."""
    ws, _ = world()
    if ws == 1 or not tensors:
        return 0
    groups = {}
    for t in tensors:
        groups.setdefault((t.device, t.dtype), []).append(t)
    n = 0
    with torch.no_grad():
        for (dev, _), ts in groups.items():
            flat = torch._utils._flatten_dense_tensors(ts)
            on_host = dist.get_backend() == "gloo" and dev.type == "cuda"
            if on_host:
                flat = flat.cpu()
            dist.broadcast(flat, src=src)
            n += 1
            if on_host:
                flat = flat.to(dev)
            for t, v in zip(ts, torch._utils._unflatten_dense_tensors(flat, ts)):
                t.copy_(v)
    return n


def gather_rows(local: torch.Tensor, total: int, dst: int = 0) -> Optional[torch.Tensor]:
    """C2: concatenate every rank's shard (dim 0) on `dst` in global order; None elsewhere.

    One ``dist.gather`` to `dst` (only `dst` receives the shards).  Shards may differ by one
    row, and ranks beyond `total` hold an empty shard: every shard is padded to the largest
    size so the collective is uniform, and `dst` trims the padding.  With the gloo backend the
    shards travel through host memory (gloo's gather is CPU-only)."""
    ws, rank = world()
    if ws == 1:
        return local
    sizes = [shard_range(total, ws, r)[1] - shard_range(total, ws, r)[0] for r in range(ws)]
    if local.shape[0] != sizes[rank]:
        raise ValueError(f"rank {rank}: shard has {local.shape[0]} rows, shard_range gives {sizes[rank]}")
    dev = local.device
    if dist.get_backend() == "gloo" and local.is_cuda:
        local = local.cpu()
    pad = torch.zeros((max(sizes),) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(ws)] if rank == dst else None
    dist.gather(pad, gather_list=bufs, dst=dst)
    if rank != dst:
        return None
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)], dim=0).to(dev)


def host_noise_slice(shape_global, start: int, end: int, device) -> torch.Tensor:
    """One global CPU-generator draw, sliced to this shard (reference draw order)."""
    return torch.randn(tuple(shape_global))[start:end].to(device)


def sharded_loop(step: Callable[[torch.Tensor, int, Optional[torch.Tensor]], torch.Tensor], x_global_shape,
                 T: int, device, noise_source: str = "host") -> torch.Tensor:
    """Run the T loop on this rank's shard.

    step(x_shard, t, noise_shard_or_None) -> x_shard'.  In host mode x_T and every
    per-step noise are drawn globally and sliced; returns this rank's final shard."""
    ws, rank = world()
    s, e = shard_range(int(x_global_shape[0]), ws, rank)
    x = host_noise_slice(x_global_shape, s, e, device)  # x_T (diff.py:327)
    for i in range(T, 0, -1):
        noise = host_noise_slice(x_global_shape, s, e, device) if noise_source == "host" else None
        x = step(x, i, noise)
    return x


def any_rank(flag: bool, device) -> bool:
    """True when `flag` is set on any rank (one tiny MAX all-reduce; the sampler's range guard)."""
    ws, _ = world()
    if ws == 1:
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32)
    if dist.get_backend() != "gloo":
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(t.item())


class ShardedCondSampler:
    """Multi-GPU ``sample_latent_cond``: same arguments, this rank's shard runs on its GPU,
    rank 0 receives all decoded uint8 images (HWC) or latents."""

    def __init__(self, diffuser, model, vae=None):
        self.d, self.model, self.vae = diffuser, model, vae
        self.range_fallbacks = 0
        # resolved here, before any collective: a missing module fails on every rank at once
        self._prefetch = _diff()._NoisePrefetch

    def sample(self, class_counts, z_shape=None, guidance_scale: float = 3.0, null_label: int = 0, cond=None,
               cond_mask=None, decode: bool = True, dummy_input_hw=(224, 224)) -> Optional[torch.Tensor]:
        """Arguments as Diffuser.sample_latent_cond (diff.py:174-369); returns on rank 0 the
        (B, 8H, 8W, 3) uint8 images (decode and a VAE given) or the (B, C, H, W) latents,
        None on the other ranks.  Draw order per rank equals the single-process sampler's
        (optional encode draw, x_T, then the seed (device mode) or one global draw per step
        (host mode)), so every sample sees the single-process draws.  The U-Net takes its split-K
        / tile decisions for a batch class (engine.hip ``dec_n``: 128 samples for every CFG batch
        of >= 64, the batch itself below) and the VAE decode per sample (``Run::tile_n``), so
        shards of >= 64 samples (config 3: 64 per rank) give rank 0 exactly the single-process
        bytes (test_gpu_multi.py, bit-equal); smaller shards equal it up to fp32 summation order
        (latents within rel-L2 1e-5 in the tests).

        The T loop runs in Diffuser.GUARD_CHUNK pieces with the single-process sampler's
        split-precision range guard: after each chunk every rank's range flag is OR-ed across
        ranks (one 4-byte all-reduce per chunk) and, if any rank saw a non-finite output, EVERY
        rank replays the chunk from its start in exact-fp32 mode (same x, same CPU-generator
        state / Philox seed) — exactly what the single process does for the whole batch."""
        ws, rank = world()
        d = self.d
        items = d._norm_counts(class_counts)
        y_list: List[int] = []
        for cls, num in items:
            y_list += [cls] * num
        B = len(y_list)
        dev = torch.device(d.device)
        vals, msk = d._build_cond(y_list, cond, cond_mask, None, None, dev)
        s, e = shard_range(B, ws, rank)
        y = torch.tensor(y_list[s:e], device=dev, dtype=torch.long)
        v, m = vals[s:e].float().contiguous(), msk[s:e].float().contiguous()
        if z_shape is None:
            if self.vae is None:
                raise ValueError("z_shape 省略時は vae が必要です。")
            z_shape = d._latent_shape(self.vae, dummy_input_hw, dev)
        C, H, W = z_shape
        nm = self.model.native() if e > s else None
        guard = d._guard_target(self.model) if nm is not None else None
        tables = d.coef_tables(dev, clamp_prev=True)
        T = d.num_timesteps
        x = torch.randn((B, C, H, W))[s:e].to(dev).contiguous()  # x_T (diff.py:327), global draw
        if d.noise_source == "device":
            seed = torch.tensor([d._seed()], dtype=torch.long)  # drawn after x_T, as _run_cond_loop does
            if ws > 1:
                if dist.get_backend() != "gloo":
                    seed = seed.to(dev)
                dist.broadcast(seed, src=0)
            seed = int(seed.item())
            t_dev = torch.full((1,), T, dtype=torch.long, device=dev)

            def run(i_from, i_to, xs):  # device Philox loop, graph-replayed, t decremented in-graph
                if xs.shape[0] > 0:
                    t_dev.fill_(i_from)
                    nm.sample_loop(xs, t_dev, y, null_label, v, m, float(guidance_scale), tables, i_from - i_to,
                                   seed=seed, sample_offset=s, use_graph=d.use_graph)
                return xs
        else:
            def run(i_from, i_to, xs):
                """One global CPU-generator draw per step (this shard's rows kept), made one step
                ahead on a helper thread into pinned buffers (diff._NoisePrefetch: same generator,
                same order), so the host draw of the global tensor overlaps the GPU step."""
                pf = self._prefetch((B, C, H, W), i_from - i_to, rows=(s, e)) if dev.type == "cuda" else None
                try:
                    for i in range(i_from, i_to, -1):
                        noise = pf.next(dev) if pf is not None else host_noise_slice((B, C, H, W), s, e, dev)
                        if xs.shape[0] > 0:  # an empty shard (B < world size) only keeps the draw order
                            out = torch.empty_like(xs)
                            tt = torch.full((xs.shape[0],), i, dtype=torch.long, device=dev)
                            nm.step(xs, out, tt, y, null_label, v, m, float(guidance_scale), tables, noise)
                            xs = out
                finally:
                    if pf is not None:
                        pf.close()
                return xs

        with torch.no_grad():
            i = T
            while i >= 1:
                j = max(i - d.GUARD_CHUNK, 0)
                x0, rng = x.clone(), torch.get_rng_state()
                x = run(i, j, x)
                tripped = guard.range_tripped() if guard is not None else False
                if any_rank(tripped, dev):
                    torch.set_rng_state(rng)
                    x = x0
                    if guard is not None:
                        with guard.precision_override("fp32"):
                            x = run(i, j, x)
                        guard.range_tripped()  # clear
                    else:
                        x = run(i, j, x)
                    self.range_fallbacks += 1
                i = j
        if decode and self.vae is not None:
            if e > s:
                _, u8 = self.vae.native().decode(x, want_img=False, want_u8=True)
            else:
                u8 = torch.empty((0, 8 * H, 8 * W, 3), dtype=torch.uint8, device=dev)
            return gather_rows(u8, B)
        return gather_rows(x, B)


def global_mask_mean(mask: torch.Tensor, group=None) -> torch.Tensor:
    """Mean over ranks of the local ``mask.sum()`` (a detached scalar on mask's device): the
    denominator that makes rank-averaged gradients of ``masked_geom_mse`` equal the global
    batch's (see ``GradAllReducer``).  World size 1: the local sum."""
    s = mask.detach().sum().reshape(1).to(torch.float64)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(s, group=group)
        s = s / dist.get_world_size(group)
    return s.to(mask.dtype).reshape(())


class GradAllReducer:
    """Data-parallel gradient averaging for the training step (train_latent_cond.py:136-163 run
    on every rank with its own batch).

    After ``loss.backward()`` each rank holds dLoss_r/dθ of its local loss; ``reduce()``
    replaces every ``p.grad`` with the mean over ranks.  For the per-sample mean terms of the
    training loss (the noise MSE) that is the gradient of the global-batch loss when the local
    batches have equal sizes (the single-process reference trained on the concatenated batch
    gives the same gradient up to fp32 summation order).  It is NOT for a term normalised by a
    data-dependent local count: ``masked_geom_mse`` divides by the rank's own mask sum, and the
    rank mean of sum_r / mask_r differs from (sum of sums) / (sum of masks) whenever the ranks'
    mask sums differ.  Pass ``denom=global_mask_mean(geom_mask)`` to ``masked_geom_mse`` (one
    scalar all-reduce) to normalise the geom term globally; the reduced gradient is then the
    global batch's.  Then every rank
    applies the same optimizer step to identical parameters (start them identical with
    ``broadcast_module``), so replicas never drift.

    Layout: parameters are packed, in reverse registration order (roughly the order the
    backward finishes them), into buckets of about ``bucket_mb`` MB; each bucket is flattened
    into one contiguous buffer and all-reduced asynchronously as soon as it is packed, so the
    packing of bucket k+1 overlaps the wire time of bucket k (RCCL runs on its own stream).  On
    xGMI's point-to-point links a ring all-reduce is per-link bound, so a few large buckets beat
    many small ones; 25 MB gives 4 buckets for the 93.7 MB of U-Net gradients.

    A gradient that is None on every rank stays None (the optimizer skips that parameter, as
    with the reference's unused branches, e.g. ``cond_mlp`` without conditions); one that is
    None on some ranks only is reduced as zeros there.  One tiny all-reduce of the presence
    mask per step decides which."""

    def __init__(self, params, bucket_mb: float = 25.0, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.bucket_bytes = int(bucket_mb * (1 << 20))

    def _buckets(self, present):
        cur, size = [], 0
        for i in reversed(range(len(self.params))):
            if not present[i]:
                continue
            p = self.params[i]
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= self.bucket_bytes:
                yield cur
                cur, size = [], 0
        if cur:
            yield cur

    def reduce(self) -> None:
        ws = dist.get_world_size(self.group) if dist.is_initialized() else 1
        if ws == 1 or not self.params:
            return
        dev = self.params[0].device
        on_host = dist.get_backend(self.group) == "gloo" and dev.type == "cuda"  # gloo: host buffers
        mask = torch.tensor([p.grad is not None for p in self.params], dtype=torch.int32)
        if not on_host:
            mask = mask.to(dev)
        dist.all_reduce(mask, op=dist.ReduceOp.MAX, group=self.group)
        present = mask.cpu().tolist()
        pending = []
        for bucket in self._buckets(present):
            grads = []
            for p in bucket:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
                grads.append(p.grad)
            flat = torch._utils._flatten_dense_tensors(grads)
            if on_host:
                flat = flat.cpu()
            pending.append((dist.all_reduce(flat, group=self.group, async_op=True), flat, grads))
        for work, flat, grads in pending:
            work.wait()
            flat = flat.to(dev) if on_host else flat
            flat.div_(ws)
            for g, r in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
                g.copy_(r)
