"""World-size-2 gloo tests of the sample-sharded multi-GPU logic (CPU, no GPU needed):
shard partition, weight broadcast (C1), gather (C2) and shard-invariant host noise."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dmx import distributed as dd


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _ByValue:
    """A tensor shipped as a numpy array."""

    def __init__(self, a):
        self.a = a


def _convert(obj, f):
    if isinstance(obj, _ByValue):
        return f(obj)
    if isinstance(obj, dict):
        return {k: _convert(v, f) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_convert(v, f) for v in obj)
    return f(obj)


def _worker(rank, world, port, fn, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # tensors travel by value (numpy): a torch tensor would be a shared-memory fd that the
        # parent can only open while this process is still alive
        q.put((rank, _convert(fn(rank, world), lambda v: _ByValue(v.numpy()) if torch.is_tensor(v) else v)))
    finally:
        dist.destroy_process_group()


def run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    back = (lambda v: torch.from_numpy(v.a) if isinstance(v, _ByValue) else v)
    res = {r: _convert(v, back) for r, v in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_shard_range_partitions():
    for total in (1, 7, 64, 512, 513):
        for ws in (1, 2, 3, 8):
            spans = [dd.shard_range(total, ws, r) for r in range(ws)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _bcast_gather(rank, world):
    m = torch.nn.Linear(4, 3)
    if rank == 0:
        with torch.no_grad():
            m.weight.fill_(1.5)
            m.bias.fill_(-2.0)
    dd.broadcast_module(m)
    local = torch.arange(dd.shard_range(5, world, rank)[0], dd.shard_range(5, world, rank)[1]).float().unsqueeze(1)
    full = dd.gather_rows(local, 5)
    return float(m.weight.sum()), float(m.bias.sum()), None if full is None else full.flatten().tolist()


def _bcast_packed(rank, world):
    """C1 packed: a module with mixed dtypes goes out as one flattened buffer per dtype."""
    m = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.Linear(3, 2))
    m.register_buffer("steps", torch.zeros(2, dtype=torch.long))
    if rank == 0:
        with torch.no_grad():
            for i, p in enumerate(m.parameters()):
                p.copy_(torch.arange(p.numel(), dtype=p.dtype).reshape(p.shape) * (i + 1))
            m.steps.fill_(7)
    ts = [t.data for t in list(m.parameters()) + list(m.buffers())]
    n = dd.broadcast_tensors(ts)
    return n, [t.flatten().tolist() for t in ts]


def test_broadcast_is_one_packed_message_per_dtype_world2():
    res = run(_bcast_packed)
    assert res[0][0] == res[1][0] == 2  # float32 parameters + the int64 buffer
    assert res[0][1] == res[1][1]
    assert res[1][1][-1] == [7.0, 7.0] or res[1][1][-1] == [7, 7]


def test_broadcast_and_gather_world2():
    res = run(_bcast_gather)
    for r in (0, 1):
        assert res[r][0] == 1.5 * 12 and res[r][1] == -6.0
    assert res[0][2] == [0.0, 1.0, 2.0, 3.0, 4.0] and res[1][2] is None


def _toy_step(x, t, noise):
    return 0.9 * x + 0.05 * t * 1e-3 + 0.1 * noise


def _sharded_host_noise(rank, world):
    torch.manual_seed(123)
    x = dd.sharded_loop(_toy_step, (5, 2, 3, 3), 6, "cpu", "host")
    return dd.gather_rows(x, 5)


def test_host_noise_is_shard_invariant_world2():
    """Each sample's x_T and per-step noise equal the single-process draw order (diff.py:327,158)."""
    res = run(_sharded_host_noise)
    torch.manual_seed(123)
    x = torch.randn((5, 2, 3, 3))
    for i in range(6, 0, -1):
        x = _toy_step(x, i, torch.randn((5, 2, 3, 3)))
    assert torch.equal(res[0], x)


# ---- ShardedCondSampler plumbing with a stub native model (CPU) -------------------------
class _FakeNative:
    """Stands in for dmx NativeModel: a per-sample deterministic step (the real one is covered by
    tests/test_gpu_multi.py on the GPU)."""

    def step(self, xs, out, tt, y, null_label, v, m, g, tables, noise):
        out.copy_(0.9 * xs + 0.1 * noise + 0.01 * y.view(-1, 1, 1, 1) + 0.001 * (v * m).sum(1).view(-1, 1, 1, 1))

    def sample_loop(self, x, t_dev, y, null_label, v, m, g, tables, steps, seed=0, sample_offset=0, use_graph=True):
        idx = torch.arange(sample_offset, sample_offset + x.shape[0], dtype=torch.float32).view(-1, 1, 1, 1)
        x.mul_(0.5).add_(idx + float(seed % 997) * 1e-3 + 0.01 * y.view(-1, 1, 1, 1))
        t_dev.sub_(steps)

    def decode(self, x, want_img=False, want_u8=True):
        u8 = (x.mean(1, keepdim=True).clamp(0, 1) * 255).to(torch.uint8).expand(-1, 3, -1, -1)
        u8 = u8.repeat_interleave(8, 2).repeat_interleave(8, 3).permute(0, 2, 3, 1).contiguous()
        return None, u8


class _FakeModel:
    _n = _FakeNative()

    def native(self):
        return self._n


def _sharded_sampler(rank, world, B=5, mode="host", decode=True):
    import diff
    d = diff.Diffuser(4, device="cpu")
    d.noise_source = mode
    torch.manual_seed(7)
    s = dd.ShardedCondSampler(d, _FakeModel(), _FakeModel() if decode else None)
    counts = {1: B // 2 + B % 2, 3: B // 2} if B > 1 else (2, 1)
    out = s.sample(counts, z_shape=(2, 3, 3), decode=decode)
    return None if out is None else out.clone()


def _sharded_b1(rank, world):
    return _sharded_sampler(rank, world, B=1, mode="host", decode=True)


def _sharded_device(rank, world):
    return _sharded_sampler(rank, world, B=5, mode="device", decode=False)


def _sharded_host_lat(rank, world):
    return _sharded_sampler(rank, world, B=5, mode="host", decode=False)


@pytest.mark.parametrize("fn", [_sharded_host_lat, _sharded_device, _sharded_b1])
def test_sharded_sampler_world2_equals_single_process(fn):
    """Rank 0 gets exactly the single-process result (host and device noise, decode, B < world)."""
    res = run(fn)
    single = fn(0, 1)
    assert res[1] is None
    assert torch.equal(res[0], single)


class _GuardNative(_FakeNative):
    """A stub native model with the split-precision range guard: in "x3" mode a step on a class-3
    sample raises the range flag and adds a visible error; "fp32" mode is exact.  Only the rank
    holding the class-3 samples trips, so both ranks must replay (the sharded sampler
    runs the single-process guard)."""

    def __init__(self):
        self.precision = "x3"
        self.flag = False

    def _mark(self, xs, y):
        if self.precision == "x3":
            xs.add_(1e-3)  # the split-precision error every x3 step carries (absent in fp32 mode)
            if bool((y == 3).any()):
                self.flag = True
                xs.add_(0.25)

    def step(self, xs, out, tt, y, null_label, v, m, g, tables, noise):
        super().step(xs, out, tt, y, null_label, v, m, g, tables, noise)
        self._mark(out, y)

    def sample_loop(self, x, t_dev, y, null_label, v, m, g, tables, steps, seed=0, sample_offset=0, use_graph=True):
        super().sample_loop(x, t_dev, y, null_label, v, m, g, tables, steps, seed, sample_offset, use_graph)
        self._mark(x, y)

    def range_tripped(self, reset=True):
        f = self.flag
        if reset:
            self.flag = False
        return f

    def precision_override(self, prec):
        import contextlib

        @contextlib.contextmanager
        def cm():
            old, self.precision = self.precision, prec
            try:
                yield self
            finally:
                self.precision = old
        return cm()


class _GuardModel:
    _dmx_kind = 2  # looks like a dmx UnetCondWithGeomHead to diff._native_kind

    def __init__(self):
        self._n = _GuardNative()

    def native(self):
        return self._n


def _guarded(rank, world, mode):
    import diff
    d = diff.Diffuser(4, device="cpu")
    d.noise_source = mode
    torch.manual_seed(7)
    s = dd.ShardedCondSampler(d, _GuardModel(), None)
    out = s.sample({1: 3, 3: 2}, z_shape=(2, 3, 3), decode=False)
    return None if out is None else (out.clone(), s.range_fallbacks)


def _guarded_host(rank, world):
    return _guarded(rank, world, "host")


def _guarded_device(rank, world):
    return _guarded(rank, world, "device")


@pytest.mark.parametrize("fn", [_guarded_host, _guarded_device])
def test_sharded_sampler_range_guard_replays_on_every_rank(fn):
    """A range trip on rank 1 only makes every rank replay the chunk in fp32: rank 0's gathered
    latents equal the single-process guarded run, and carry no x3 error."""
    res = run(fn)
    single, nfall = fn(0, 1)
    assert nfall == 1 and res[1] is None
    out, nf0 = res[0]
    assert nf0 == 1
    assert torch.equal(out, single)


def test_gather_rows_rejects_wrong_shard():
    res = run(_bad_gather)
    assert res[0] == "ValueError" and res[1] == "ValueError"


def _bad_gather(rank, world):
    try:
        dd.gather_rows(torch.zeros(4, 2), 5)
    except ValueError:
        return "ValueError"
    return "ok"


# ---- data-parallel training: GradAllReducer ----------------------
class _Toy(torch.nn.Module):
    """Two-layer MLP with a branch used only by some ranks (`extra`) and one never used (`dead`)."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(3)
        self.l1 = torch.nn.Linear(6, 16)
        self.l2 = torch.nn.Linear(16, 3)
        self.extra = torch.nn.Linear(6, 3)
        self.dead = torch.nn.Linear(6, 3)

    def forward(self, x, use_extra):
        out = self.l2(torch.nn.functional.gelu(self.l1(x)))
        return out + self.extra(x) if use_extra else out


def _toy_batch():
    g = torch.Generator().manual_seed(11)
    return torch.randn((12, 6), generator=g), torch.randn((12, 3), generator=g)


def _dp_grads(rank, world, bucket_mb):
    m = _Toy()
    dd.broadcast_module(m)
    x, y = _toy_batch()
    s, e = dd.shard_range(12, world, rank)
    loss = torch.nn.functional.mse_loss(m(x[s:e], use_extra=(rank == 0)), y[s:e])
    loss.backward()
    dd.GradAllReducer(m.parameters(), bucket_mb=bucket_mb).reduce()
    return {n: (None if p.grad is None else p.grad.clone()) for n, p in m.named_parameters()}


def _dp_small_buckets(rank, world):
    return _dp_grads(rank, world, 0.0005)  # ~500 B buckets: several buckets, async in flight together


def _dp_one_bucket(rank, world):
    return _dp_grads(rank, world, 25.0)


@pytest.mark.parametrize("fn,world", [(_dp_small_buckets, 2), (_dp_one_bucket, 2), (_dp_small_buckets, 3)])
def test_grad_allreduce_equals_full_batch_mean(fn, world):
    """Averaged per-rank gradients == the gradient of the full-batch mean loss (equal shards);
    a branch used on one rank only is reduced as zeros elsewhere; a never-used one stays None."""
    res = run(fn, world)
    m = _Toy()
    x, y = _toy_batch()
    per = 12 // world  # full-batch reference: rank 0's shard uses `extra`, the others do not
    out = torch.cat([m(x[:per], use_extra=True), m(x[per:], use_extra=False)])
    torch.nn.functional.mse_loss(out, y).backward()
    for n, p in m.named_parameters():
        for r in range(world):
            if p.grad is None:
                assert res[r][n] is None, n
            else:
                assert torch.allclose(res[r][n], p.grad, rtol=1e-5, atol=1e-7), n
    for r in range(1, world):
        assert torch.equal(res[0]["l1.weight"], res[r]["l1.weight"])


def _geom_batch():
    g = torch.Generator().manual_seed(5)
    pred_in = torch.randn((8, 4), generator=g)
    gt = torch.randn((8, 4), generator=g)
    mask = (torch.rand((8, 4), generator=g) < torch.linspace(0.1, 0.9, 8)[:, None]).float()
    return pred_in, gt, mask


def _dp_geom(rank, world):
    from losses.geom_losses import masked_geom_mse
    w = torch.nn.Parameter(torch.linspace(-1.0, 1.0, 4))
    x, gt, mask = _geom_batch()
    s, e = dd.shard_range(8, world, rank)
    loss = masked_geom_mse(x[s:e] * w, gt[s:e], mask[s:e], denom=dd.global_mask_mean(mask[s:e]))
    loss.backward()
    dd.GradAllReducer([w]).reduce()
    return w.grad.clone()


def test_grad_allreduce_masked_geom_global_denominator():
    """masked_geom_mse with the all-reduced mask denominator: the rank-averaged gradient equals
    the single-process gradient of the whole batch's masked mean although the two shards' mask
    sums differ (the reference's local denominator would not)."""
    from losses.geom_losses import masked_geom_mse
    res = run(_dp_geom, 2)
    w = torch.nn.Parameter(torch.linspace(-1.0, 1.0, 4))
    x, gt, mask = _geom_batch()
    assert mask[:4].sum() != mask[4:].sum()
    masked_geom_mse(x * w, gt, mask).backward()
    for r in range(2):
        assert torch.allclose(res[r], w.grad, rtol=1e-5, atol=1e-7)
