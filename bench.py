"""Benchmark: CFG denoising steps/s (T=1000, 32x32x4 latents, B=64 per GPU) on MI355X.

A "step" is one Diffuser.denoise_cond over the batch (reference diff.py:127-162):
two U-Net forwards (uncond + cond, batched as one 2B = 128-sample native forward)
plus the CFG mix and the DDPM update, with on-device Philox noise; the timed steps
run as replayed hipGraphs (the diff.py:332-344 loop without host round trips).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N  (one rank per GPU)

Each rank runs its own B=64 shard (weak scaling: samples are independent — no
per-step collective); frozen weights are broadcast from rank 0 over RCCL once.
`value` = batch-steps/s of the whole job = N * K / max-over-ranks time.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(REPO, "diffusion-model_amd"), REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X dense fp32 MFMA (MI355X_MICROARCH.md, chip table)
F16_MFMA_PEAK_TFLOPS = 2500.0   # MI355X dense fp16/bf16 MFMA (spec, no sparsity)
HBM_PEAK_GBS = 8000.0
UNET_GFLOP_PER_SAMPLE = 3.7097  # reference FLOPs per sample-forward


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--hw", type=int, default=32)
    ap.add_argument("--T", type=int, default=1000)
    ap.add_argument("--guidance", type=float, default=3.0)
    ap.add_argument("--cpu-steps", type=int, default=5, help="oracle steps timed for cpu_baseline, median (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0: os.cpu_count(), capped by OMP_NUM_THREADS where the host sets the process's share")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--config5-steps", type=int, default=100,
                    help="steps timed in BASELINE config 5 (B=1, VAE decode of every x_t) (0 = skip)")
    ap.add_argument("--config4-steps", type=int, default=100,
                    help="steps timed in BASELINE config 4 (fp16 arithmetic) beside the headline (0 = skip)")
    ap.add_argument("--legs-steps", type=int, default=30,
                    help="steps timed for the fp32-MFMA and host-noise legs beside the headline (0 = skip)")
    ap.add_argument("--train-steps", type=int, default=10, help="training-step leg (0 = skip)")
    ap.add_argument("--train-batch", type=int, default=32)
    ap.add_argument("--no-e2e", dest="e2e", action="store_false",
                    help="skip the end-to-end config-2 sample (T steps + decode + uint8 + PIL) leg")
    ap.add_argument("--sharded-T", type=int, default=50,
                    help="steps of the ShardedCondSampler leg (config 3 path incl. decode + gather; 0 = skip)")
    ap.add_argument("--png-steps", type=int, default=100,
                    help="steps of the generate_steps drop-in (async PNG pipeline) timed for config 5 (0 = skip)")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("DMX_BENCH_ONE_DEVICE") == "1":
        # rehearsal of the multi-rank path on a one-GPU box: every rank on cuda:0, gloo
        # collectives (RCCL refuses two ranks on one device); never used for a reported number
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        backend = os.environ.get("DMX_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def make_inputs(B, hw, dev, seed=0):
    """Synthetic config-2 inputs: x_T ~ N(0,1), y cycles 1,2,3,
    cond U[0,1) masked to the class keys of diff.py:235-239."""
    from diff import CLASS_KEYS, KEY_ORDER
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((B, 4, hw, hw), generator=g)
    y = torch.tensor([1 + i % 3 for i in range(B)], dtype=torch.long)
    mask = torch.zeros((B, 12))
    for i in range(B):
        for k in CLASS_KEYS[int(y[i])]:
            mask[i, KEY_ORDER.index(k)] = 1.0
    vals = torch.rand((B, 12), generator=g) * mask
    return x.to(dev), y.to(dev), vals.to(dev), mask.to(dev)


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(args):
    """The oracle (reference-equivalent torch-CPU restatement, bit-exact with the reference on this
    container) timed on the host cores: 1 warm-up + the median of --cpu-steps CFG steps at the
    benchmark shape (BASELINE.md:48-53).  Threads: os.cpu_count(), capped by OMP_NUM_THREADS where
    the host sets this process's share (16 per GPU on the MI355X pool)."""
    from dmx import synth
    from oracle import ref
    share = int(os.environ.get("OMP_NUM_THREADS") or 0)
    threads = args.cpu_threads or min(os.cpu_count() or 1, share or (os.cpu_count() or 1))
    torch.set_num_threads(threads)
    sd = synth.unet_cond_geom_weights(0)
    x, y, vals, mask = make_inputs(args.batch, args.hw, "cpu")
    _, a, ab = ref.schedule(args.T)
    t = torch.full((args.batch,), args.T, dtype=torch.long)
    times = []
    with torch.no_grad():
        ref.cfg_step(sd, x, t, y, a, ab, args.guidance, 0, vals, mask, torch.randn(x.shape))  # warm-up
        for _ in range(args.cpu_steps):
            t0 = time.perf_counter()
            x = ref.cfg_step(sd, x, t, y, a, ab, args.guidance, 0, vals, mask, torch.randn(x.shape))
            times.append(time.perf_counter() - t0)
    med = sorted(times)[len(times) // 2]
    return {"value": round(1.0 / med, 4), "unit": "CFG batch-steps/s (B=%d)" % args.batch, "cores": threads,
            "kind": "port", "cpu_model": _cpu_model(), "host_cpu_count": os.cpu_count(),
            "sample": f"median of {args.cpu_steps} CFG steps at B={args.batch}, {args.hw}x{args.hw}x4, after 1 "
                      f"warm-up (oracle/ref.py, torch-CPU fp32, {threads} threads); step times "
                      f"{[round(v, 3) for v in times]} s"}


def legs(nm, model, x, y, vals, mask, args, tables, seed):
    """Beside the headline: the same config-2 step in exact-fp32 MFMA mode (precision 0, graph
    replay) and on the default drop-in path (Diffuser.denoise_cond with host CPU-generator noise:
    one eager dmx_step per step plus the host draw and its H2D copy)."""
    import diff
    out = {}
    k = args.legs_steps
    with nm.precision_override("fp32"):
        xs = x.clone()
        t_dev = torch.full((1,), args.T, dtype=torch.long, device=x.device)
        nm.sample_loop(xs, t_dev, y, 0, vals, mask, args.guidance, tables, 3, seed=seed)
        torch.cuda.synchronize()
        t_dev.fill_(args.T)
        t0 = time.perf_counter()
        nm.sample_loop(xs, t_dev, y, 0, vals, mask, args.guidance, tables, k, seed=seed)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    out["fp32_mfma"] = {"value": round(k / dt, 3), "unit": "CFG batch-steps/s (B=%d)" % args.batch,
                        "ms_per_step": round(dt / k * 1e3, 4), "steps": k,
                        "dtype": "f32 (exact fp32 MFMA v_mfma_f32_32x32x2_f32 / 16x16x4_f32)"}
    # the sampler's own loop (diff.py:332-344 as Diffuser.sample_latent_cond drives it): a k-step schedule has
    # the same per-step work as the T = 1000 one
    d = diff.Diffuser(k, device=x.device)
    counts = [(c, int((y == c).sum())) for c in (1, 2, 3)]
    d.sample_latent_cond(model, counts, z_shape=(4, args.hw, args.hw), progress=False, cond=vals, cond_mask=mask)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    xs = d.sample_latent_cond(model, counts, z_shape=(4, args.hw, args.hw), progress=False, cond=vals,
                              cond_mask=mask)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert torch.isfinite(xs).all(), "non-finite latents (host-noise leg)"
    out["host_noise"] = {"value": round(k / dt, 3), "unit": "CFG batch-steps/s (B=%d)" % args.batch,
                         "ms_per_step": round(dt / k * 1e3, 4), "steps": k,
                         "path": "Diffuser.sample_latent_cond loop: eager dmx_step per step, noise from torch's CPU "
                                 "generator in the reference's draw order (helper-thread draws, pinned async H2D)"}
    # the reference sampler's own latent shape (diff.py:315-322: the 224 dummy through VAE.encode gives
    # 28 x 28 x 4), same batch and loop (graph replay, device noise)
    x28, y28, v28, m28 = make_inputs(args.batch, 28, x.device, seed=7)
    t_dev = torch.full((1,), args.T, dtype=torch.long, device=x.device)
    nm.sample_loop(x28, t_dev, y28, 0, v28, m28, args.guidance, tables, 3, seed=seed)
    torch.cuda.synchronize()
    t_dev.fill_(args.T)
    t0 = time.perf_counter()
    nm.sample_loop(x28, t_dev, y28, 0, v28, m28, args.guidance, tables, k, seed=seed)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert torch.isfinite(x28).all(), "non-finite latents (28x28 leg)"
    out["latent28"] = {"value": round(k / dt, 3), "unit": "CFG batch-steps/s (B=%d, 28x28x4)" % args.batch,
                       "ms_per_step": round(dt / k * 1e3, 4), "steps": k,
                       "pixel_rate_vs_main": None,  # filled in by main(): per-latent-pixel rate / the main leg's
                       "note": "reference default sampler shape (diff.py:315-322); the 28 / 14 / 7 / 3 maps run the "
                               "Winograd convs in their 32 / 16 / 8 / 4 geometries (zero-padded columns)"}
    return out


def train_leg(args, dev, world=1, rank=0):
    """The training step of train_latent_cond.py:114-163 on the drop-ins, B = 32 224x224 synthetic
    images per GPU: frozen VAE encode (micro-batches of 8, no_grad), t ~ U{1..1000}, add_noise, CFG
    dropout (p = 0.1), UnetCondWithGeomHead forward + F.mse_loss + geom_lambda * masked_geom_mse,
    backward (native dmx_train_backward), torch Adam(lr=1e-4) step.  world > 1: data-parallel — every
    rank its own batch, gradients averaged by dmx.distributed.GradAllReducer (bucketed async RCCL
    all-reduces over xGMI) before the Adam step; value = images/s of the whole job (max over ranks).
    Also the native forward + backward alone, and (world > 1) the gradient all-reduce alone."""
    import diff
    from dmx import distributed as dd
    from dmx import synth
    from losses.geom_losses import masked_geom_mse
    from models.unet_cond_geom import UnetCondWithGeomHead
    from models.vae import VAE
    B = args.train_batch
    g = torch.Generator().manual_seed(7 + rank)
    model = UnetCondWithGeomHead()
    model.load_state_dict(synth.unet_cond_geom_weights(0))
    model.to(dev).train()
    dd.broadcast_module(model)
    reducer = dd.GradAllReducer(model.parameters())
    vae = VAE()
    vae.load_state_dict(synth.vae_weights(1))
    vae.to(dev).eval()
    for p in vae.parameters():
        p.requires_grad = False
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    diffuser = diff.Diffuser(1000, device=dev)
    images = torch.rand((B, 3, 224, 224), generator=g).to(dev)
    vals = torch.rand((B, 12), generator=g).to(dev)
    mask = (torch.rand((B, 12), generator=g) > 0.3).float().to(dev)
    classes = torch.randint(1, 4, (B,), generator=g).to(dev)

    def step():
        with torch.no_grad():
            z = torch.cat([vae.encode(mb)[0] for mb in images.split(8, dim=0)], dim=0)
        t = torch.randint(1, 1001, (B,), device=dev)
        z_noisy, noise = diffuser.add_noise(z, t)
        drop = torch.rand(B, device=dev) < 0.1
        y_used = torch.where(drop, torch.zeros_like(classes), classes)
        keep = (~drop).float().unsqueeze(1)
        eps, geom = model(z_noisy, t, y_used, cond_vals=vals * keep, cond_mask=mask * keep)
        m_used = mask * keep
        # world > 1: the geom term normalised by the GLOBAL mask mean, so the rank-averaged
        # gradient is the global batch's (dmx.distributed.GradAllReducer)
        denom = dd.global_mask_mean(m_used) if world > 1 else None
        loss = F.mse_loss(eps, noise) + 0.5 * masked_geom_mse(geom, vals, m_used, denom=denom)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        reducer.reduce()
        opt.step()
        return loss

    def synced():
        torch.cuda.synchronize()
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    def max_over_ranks(v):
        if world == 1:
            return v
        import torch.distributed as dist
        e = torch.tensor([v], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        return float(e.item())

    for _ in range(2):
        step()
    synced()
    k = args.train_steps
    t0 = time.perf_counter()
    for _ in range(k):
        loss = step()
    synced()
    dt = max_over_ranks((time.perf_counter() - t0) / k)
    assert torch.isfinite(loss), "non-finite training loss"
    ar_ms = None
    if world > 1:  # the gradient all-reduce alone (grads of the last step still in place)
        synced()
        t0 = time.perf_counter()
        for _ in range(k):
            reducer.reduce()
        synced()
        ar_ms = max_over_ranks((time.perf_counter() - t0) / k) * 1e3
    # native forward + backward alone (same shapes)
    nm = model.native()
    z = torch.randn((B, 4, 28, 28), generator=g).to(dev)
    t = torch.randint(1, 1001, (B,), generator=g).to(dev)
    d_eps, d_geom = torch.randn_like(z), torch.randn((B, nm.geom_dim), device=dev)
    for _ in range(2):
        _, _, tape = nm.train_forward(z, t, classes, vals, mask)
        nm.train_backward(tape, d_eps, d_geom)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        _, _, tape = nm.train_forward(z, t, classes, vals, mask)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(k):
        _, _, tape = nm.train_forward(z, t, classes, vals, mask)
        nm.train_backward(tape, d_eps, d_geom)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    fwd = (t1 - t0) / k
    fb = (t2 - t1) / k
    res = {"value": round(world * B / dt, 2),
           "unit": "training images/s (B=%d per GPU, 224x224 -> 28x28x4 latents)" % B,
           "ms_per_step": round(dt * 1e3, 3), "steps": k, "n_gpus": world,
            "native_forward_ms": round(fwd * 1e3, 3), "native_backward_ms": round((fb - fwd) * 1e3, 3),
            "dtype": "f32 semantics (GEMMs and the forward attention cores as x3 split-f16 MFMA products with fp32 accumulation; attention backward on fp32 MFMA; fp32 elsewhere)",
            "path": "train_latent_cond.py step on the drop-ins: VAE.encode x4, add_noise, forward, mse + "
                    "masked_geom_mse, loss.backward() (dmx_train_backward), torch Adam"}
    if world > 1:
        res["parallelism"] = f"data-parallel x{world}: bucketed async all-reduce of 93.7 MB fp32 gradients"
        res["grad_allreduce_ms"] = round(ar_ms, 3)
    return res


MFMA_FAMILIES = ("igemm_x3_kernel", "igemm_pp_kernel", "igemm_f32_kernel", "attention_x3_kernel",
                 "attention16_kernel", "attention_kernel", "tok_ln_qkv_kernel", "tok_ln_qkv_lds_kernel",
                 "tok_attn_out_kernel", "igemm_halo_kernel", "igemm_halo_cs_kernel", "wino_kernel")
X3_FAMILIES = ("igemm_pp_kernel", "attention16_kernel", "igemm_halo_kernel", "igemm_halo_cs_kernel", "wino_kernel")
# Winograd F(2x2, 3x3): the algorithmic work is the reference's direct conv (2 M Cout 9 Cin); the
# kernel issues 16 / 36 of those multiply-adds on the matrix cores
WINO_EXECUTED = 16.0 / 36.0


def family(name):
    return name.split("<", 1)[0]


def _entry(fam, a, pmc_fam):
    """Roofline entry of one kernel family: algorithmic work per launch / average launch time."""
    avg_ms = a["ms"] / a["n"]
    if fam in MFMA_FAMILIES:
        per_launch = a["flops"] / a["n"]
        achieved = per_launch / (avg_ms * 1e-3) / 1e12
        if "x3" in fam or fam.startswith("tok_") or fam in X3_FAMILIES:
            # fp32 operands as fp16 hi+lo: 3 f16 MFMAs per algorithmic fp32 multiply-add
            peak, mfma = F16_MFMA_PEAK_TFLOPS / 3.0, "f16 x3 split (peak = 2500/3 TF of fp32 work)"
        else:
            peak, mfma = FP32_MFMA_PEAK_TFLOPS, "f32"
        e = {"kernel": fam, "bound": "mfma", "mfma_dtype": mfma, "achieved": round(achieved, 3),
             "peak": round(peak, 1), "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
             "flops_per_launch": per_launch}
        if fam == "wino_kernel":
            e["work"] = "direct-conv FLOPs (reference work); executed MFMA work = 16/36 of it"
            e["executed_frac_of_peak"] = round(achieved * WINO_EXECUTED / peak, 4)
    else:
        per_launch = a["bytes"] / a["n"]
        achieved = per_launch / (avg_ms * 1e-3) / 1e9
        e = {"kernel": fam, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
             "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "bytes_per_launch": per_launch}
    e["traffic"] = round(pmc_fam / a["n"]) if pmc_fam is not None else None
    e["launches"] = a["n"]
    e["avg_launch_us"] = round(avg_ms * 1e3, 2)
    return e


def _pmc_by_label(pmc, labels):
    """PMC bytes keyed by bench.py's kernel labels.  rocprofv3 names carry every template argument
    (wave layout, prefetch depth), the labels only the leading ones: a label takes the PMC entry whose
    template arguments start with the label's (the mean if several launch configurations match)."""
    def split(name):
        fam, _, rest = name.partition("<")
        return fam, [a.strip() for a in rest.rstrip(">").split(",")] if rest else []
    out = {}
    for lab in labels:
        if lab in pmc:
            out[lab] = pmc[lab]
            continue
        fam, args = split(lab)
        hits = [v for k, v in pmc.items() if split(k)[0] == fam and split(k)[1][:len(args)] == args]
        if hits:
            out[lab] = sum(hits) / len(hits)
    return out


def roofline(records, pmc=None):
    """Dominant kernel = the kernel family (name without template arguments: every tile /
    epilogue instantiation of the implicit-GEMM conv is one kernel) with the largest summed
    duration in one eager, HIP-event-timed step (events on the launch stream);
    achieved = its algorithmic FLOPs (MFMA-bound) or bytes (HBM-bound) per launch / its average
    event-timed launch duration.  `traffic` = PMC HBM bytes per launch (profiles/pmc_traffic.json,
    averaged over the family's launches in the step) or null."""
    agg, fams = {}, {}
    pmc = _pmc_by_label(pmc, {r["kernel"] for r in records}) if pmc is not None else None
    for r in records:
        for key, d in ((r["kernel"], agg), (family(r["kernel"]), fams)):
            a = d.setdefault(key, {"ms": 0.0, "flops": 0.0, "bytes": 0.0, "n": 0, "pmc": 0.0, "pmc_ok": True})
            a["ms"] += r["ms"]
            a["flops"] += r["flops"]
            a["bytes"] += r["bytes"]
            a["n"] += 1
            if pmc is not None and r["kernel"] in pmc:
                a["pmc"] += pmc[r["kernel"]]
            else:
                a["pmc_ok"] = False
    total_ms = sum(v["ms"] for v in agg.values())
    total_flops = sum(v["flops"] for v in agg.values())
    ranked = sorted(fams.items(), key=lambda kv: -kv[1]["ms"])
    fam, a = ranked[0]
    rl = _entry(fam, a, a["pmc"] if a["pmc_ok"] else None)
    rl["share_of_step"] = round(a["ms"] / total_ms, 3)
    rl["step_kernel_ms"] = round(total_ms, 3)
    rl["step_tflops_eager"] = round(total_flops / (total_ms * 1e-3) / 1e12, 3)
    # the next families by time, each against its own roofline
    rl["others"] = [dict(_entry(f, v, v["pmc"] if v["pmc_ok"] else None), share_of_step=round(v["ms"] / total_ms, 3))
                    for f, v in ranked[1:5]]
    for o in rl["others"]:
        o.pop("flops_per_launch", None)
        o.pop("bytes_per_launch", None)
    return rl, agg


def lib_sha256() -> str:
    import hashlib
    from dmx import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def load_pmc():
    """PMC HBM bytes per launch (profiles/pmc_traffic.json, tools/pmc_traffic.py) — only when that
    file was measured on THIS library build (its lib_sha256 equals the loaded libdmx.so's);
    otherwise `traffic` stays null and the note says why."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, "no profiles/pmc_traffic.json"
    doc = json.load(open(path))
    have, want = doc.get("lib_sha256"), lib_sha256()
    if have != want:
        return None, f"stale: profiles/pmc_traffic.json is of build {str(have)[:12]}, loaded build {want[:12]}"
    return doc.get("traffic_bytes_per_launch"), f"profiles/pmc_traffic.json (build {want[:12]})"


def e2e_sample(model, args, dev):
    """One full BASELINE config-2 sample end to end (reference diff.py:326-369 as the drop-in runs it):
    Diffuser.sample_latent_cond with device (Philox) noise — x_T draw, the T-step CFG loop (graph
    replay, range-guarded chunks), empty_cache, the VAE decode of all B latents (uint8 HWC on the
    device), the D2H copy and the PIL conversion — as wall seconds.  The decode + D2H + PIL tail is
    also timed alone."""
    import diff
    from dmx import synth
    from models.vae import VAE
    vae = VAE()
    vae.load_state_dict(synth.vae_weights(1))
    vae = vae.to(dev).eval()
    _, y, vals, mask = make_inputs(args.batch, args.hw, dev, seed=11)
    counts = [(c, int((y == c).sum())) for c in (1, 2, 3)]
    order = torch.argsort(y, stable=True)  # the sampler lays out classes in count order
    vals, mask = vals[order].contiguous(), mask[order].contiguous()
    kw = dict(z_shape=(4, args.hw, args.hw), vae=vae, to_pil=True, progress=False, cond=vals, cond_mask=mask)
    warm = diff.Diffuser(diff.Diffuser.GUARD_CHUNK, device=dev)
    warm.noise_source = "device"
    warm.sample_latent_cond(model, counts, **kw)  # graph capture, decode workspace
    d = diff.Diffuser(args.T, device=dev)
    d.noise_source = "device"
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    imgs = d.sample_latent_cond(model, counts, **kw)
    dt = time.perf_counter() - t0
    assert len(imgs) == args.batch and imgs[0].size == (8 * args.hw, 8 * args.hw)
    z = torch.randn((args.batch, 4, args.hw, args.hw), generator=torch.Generator().manual_seed(3)).to(dev)
    d._decode(vae, z, True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    d._decode(vae, z, True)
    tail = time.perf_counter() - t1
    return {"workload": f"config 2 end to end: one sample_latent_cond call, B={args.batch}, T={args.T}, CFG "
                        f"{args.guidance}, device noise, VAE decode to {8 * args.hw}x{8 * args.hw} uint8 + PIL",
            "seconds": round(dt, 4), "images_per_s": round(args.batch / dt, 2),
            "loop_steps_per_s": round(args.T / max(dt - tail, 1e-9), 2),
            "decode_d2h_pil_ms": round(tail * 1e3, 2), "range_fallbacks": d.range_fallbacks}


def sharded_sample(model, args, dev, world, rank):
    """BASELINE config 3 path (multi-GPU): dmx.distributed.ShardedCondSampler.sample over a global batch
    of B x world (B per rank), device noise, a T_s-step CFG loop, per-rank VAE decode and the C2
    gather of all uint8 images on rank 0 (dist.gather; RCCL under torchrun).  Reports the whole call
    (max over ranks) and the gather alone."""
    import diff
    from dmx import distributed as dd
    from dmx import synth
    from models.vae import VAE
    vae = VAE()
    vae.load_state_dict(synth.vae_weights(1))
    vae = vae.to(dev).eval()
    Bg = args.batch * world
    T = args.sharded_T
    counts = [(1, Bg - 2 * (Bg // 3)), (2, Bg // 3), (3, Bg // 3)]

    def run():
        d = diff.Diffuser(T, device=dev)
        d.noise_source = "device"
        torch.manual_seed(21)
        return dd.ShardedCondSampler(d, model, vae).sample(counts, z_shape=(4, args.hw, args.hw),
                                                            guidance_scale=args.guidance, decode=True)

    def synced():
        torch.cuda.synchronize()
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    def max_over_ranks(v):
        if world == 1:
            return v
        import torch.distributed as dist
        e = torch.tensor([v], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        return float(e.item())

    run()
    synced()
    t0 = time.perf_counter()
    imgs = run()
    synced()
    dt = max_over_ranks(time.perf_counter() - t0)
    if rank == 0:
        assert imgs is not None and imgs.shape == (Bg, 8 * args.hw, 8 * args.hw, 3)
    s, e = dd.shard_range(Bg, world, rank)
    u8 = torch.zeros((e - s, 8 * args.hw, 8 * args.hw, 3), dtype=torch.uint8, device=dev)
    dd.gather_rows(u8, Bg)
    synced()
    t1 = time.perf_counter()
    dd.gather_rows(u8, Bg)
    synced()
    g = max_over_ranks(time.perf_counter() - t1)
    return {"workload": f"config 3 path: ShardedCondSampler.sample, global B={Bg} ({args.batch} per rank), T={T}, "
                        f"device noise, per-rank decode, uint8 gather to rank 0",
            "seconds": round(dt, 4), "steps_per_s": round(T / dt, 2),
            "job_batch_steps_per_s": round(world * T / dt, 2),
            "images_per_s": round(Bg / dt, 2), "gather_ms": round(g * 1e3, 3),
            "gather_bytes": Bg * 64 * args.hw * args.hw * 3, "n_gpus": world,
            "backend": (__import__("torch.distributed").distributed.get_backend() if world > 1 else "none")}


def config5(nm, args, tables, seed):
    """BASELINE config 5 (generate_steps.py:158-187): B=1, and before every denoise_cond the
    current latent x_t is decoded by the frozen VAE to a 256x256 uint8 image (the PNG write
    itself is host I/O, excluded).  Per step: one VAE decode launch sequence + one CFG step
    (replayed hipGraph); units = denoising steps/s with per-step decode."""
    from dmx import synth
    from models.vae import VAE
    dev = torch.device("cuda", torch.cuda.current_device())
    vae = VAE()
    vae.load_state_dict(synth.vae_weights(1))
    vae = vae.to(dev).eval()
    vn = vae.native()
    x, y, vals, mask = make_inputs(1, args.hw, dev, seed=5)
    t_dev = torch.full((1,), args.T, dtype=torch.long, device=dev)

    def run(k):
        for _ in range(k):
            vn.decode(x, want_img=False, want_u8=True)
            nm.sample_loop(x, t_dev, y, 0, vals, mask, args.guidance, tables, 1, seed=seed)

    run(5)
    torch.cuda.synchronize()
    t_dev.fill_(args.T)
    t0 = time.perf_counter()
    run(args.config5_steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert torch.isfinite(x).all(), "non-finite latents (config 5)"
    res = {"workload": "config 5: generate_steps path, B=1, VAE decode (uint8 256x256) of x_t before every CFG step",
           "value": round(args.config5_steps / dt, 2), "unit": "denoising steps/s (B=1, decode every step)",
           "ms_per_step": round(dt / args.config5_steps * 1e3, 4), "steps": args.config5_steps, "dtype": "f32 (x3)",
           "gflop_per_step": round(2 * UNET_GFLOP_PER_SAMPLE + 11.52, 2), "png": "excluded (kernels only)"}
    if args.png_steps > 0:
        res["with_png"] = config5_png(args, vae)
    return res


def config5_png(args, vae):
    """The generate_steps.py drop-in end to end (save_reverse_steps_for_csv_row, every step saved:
    decode + 1 pixel PNG + 4 latent-channel PNGs per step through the async pipeline), both noise
    sources; PNG encode and file writes included."""
    import tempfile
    import generate_steps as gs
    from dmx import synth
    from models.unet_cond_geom import UnetCondWithGeomHead
    dev = torch.device("cuda", torch.cuda.current_device())
    m = UnetCondWithGeomHead()
    m.load_state_dict(synth.unet_cond_geom_weights(0))
    m.to(dev).eval()
    csv = os.path.join(REPO, "tests", "golden", "entities.csv")
    out = {}
    for mode in ("host", "device"):
        with tempfile.TemporaryDirectory() as tmp:
            kw = dict(csv_path=csv, row_index=0, class_id=1, model=m, vae=vae, device="cuda",
                      z_shape=(1, 4, args.hw, args.hw), out_root=tmp, progress=False, noise_source=mode)
            gs.save_reverse_steps_for_csv_row(num_timesteps=5, run_name="warm", **kw)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gs.save_reverse_steps_for_csv_row(num_timesteps=args.png_steps, run_name="run", **kw)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            n_png = sum(len(f) for _, _, f in os.walk(os.path.join(tmp, "run")))
        out[mode + "_noise"] = {"value": round(args.png_steps / dt, 2), "unit": "denoising steps/s incl. 5 PNGs/step",
                                "ms_per_step": round(dt / args.png_steps * 1e3, 4), "steps": args.png_steps,
                                "pngs": n_png}
    return out


def config4(nm, x, y, vals, mask, args, tables, seed):
    """BASELINE config 4: the same CFG step with fp16 GEMM/attention operands (one f16 MFMA,
    fp32 accumulate, fp32 norms/softmax/scheduler); tolerance study in tests/test_gpu_f16.py.
    Reported beside the headline, never as `value` (reduced precision)."""
    old = nm.precision
    nm.set_precision("f16")
    try:
        xs = x.clone()
        t_dev = torch.full((1,), args.T, dtype=torch.long, device=x.device)
        nm.sample_loop(xs, t_dev, y, 0, vals, mask, args.guidance, tables, 5, seed=seed)  # warm-up + capture
        torch.cuda.synchronize()
        t_dev.fill_(args.T)
        t0 = time.perf_counter()
        nm.sample_loop(xs, t_dev, y, 0, vals, mask, args.guidance, tables, args.config4_steps, seed=seed)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        assert torch.isfinite(xs).all(), "non-finite latents (config 4)"
    finally:
        nm.set_precision(old)
    return {"workload": "config 4: config 2 with fp16 weights/activations, fp32 accumulate + scheduler",
            "value": round(args.config4_steps / dt, 3), "unit": "CFG batch-steps/s (B=%d)" % args.batch,
            "ms_per_step": round(dt / args.config4_steps * 1e3, 4), "steps": args.config4_steps, "dtype": "f16",
            "tolerance": "latents rel-L2 <= 2e-3 after T=1000, measured 7.1e-4 (tests/test_gpu_f16.py)"}


def main():
    args = parse()
    world, rank, local = dist_setup(args)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    import diff
    from dmx import synth
    from models.unet_cond_geom import UnetCondWithGeomHead

    model = UnetCondWithGeomHead()
    if rank == 0 or world == 1:
        model.load_state_dict(synth.unet_cond_geom_weights(0))
    model.to(dev).eval()
    if world > 1:  # C1: broadcast the frozen weights once over RCCL (xGMI), one packed buffer
        from dmx import distributed as dd
        dd.broadcast_module(model)
    nm = model.native()
    d = diff.Diffuser(args.T, device=dev)
    tables = d.coef_tables(dev, True)
    x, y, vals, mask = make_inputs(args.batch, args.hw, dev, seed=rank)
    t_dev = torch.full((1,), args.T, dtype=torch.long, device=dev)
    seed = 1234

    # warm-up (also captures the step graph)
    nm.sample_loop(x, t_dev, y, 0, vals, mask, args.guidance, tables, max(args.warmup, 1), seed=seed,
                   sample_offset=rank * args.batch)
    torch.cuda.synchronize()
    t_dev.fill_(args.T)

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nm.sample_loop(x, t_dev, y, 0, vals, mask, args.guidance, tables, args.steps, seed=seed,
                   sample_offset=rank * args.batch)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    assert torch.isfinite(x).all(), "non-finite latents"

    value = world * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    out = {
        "metric": "denoising steps/sec (CFG, T=1000, 32x32x4 latent, B=64)",
        "value": round(value, 3),
        "unit": "CFG batch-steps/s (B=64 per GPU; 2 U-Net forwards + update each)",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32 (GEMMs: fp32 operands split fp16 hi+lo on the matrix cores, fp32 accumulate)", "data": "synthetic (seeded synthetic weights, x_T~N(0,1), Philox step noise)",
        "config": {"workload": "config 2: UnetCondWithGeomHead CFG=3.0 denoising step, B=64, 32x32x4, T=1000",
                   "global_batch": args.batch * world, "latent": [4, args.hw, args.hw], "T": args.T,
                   "parallelism": f"sample-sharded x{world} (no per-step collective)"},
        "sample_steps_per_s": round(value * args.batch, 1),
        "tflops_effective": round(value * 2 * args.batch * UNET_GFLOP_PER_SAMPLE / 1e3, 2),
    }
    if world == 1 and args.config4_steps > 0:
        out["config4"] = config4(nm, x, y, vals, mask, args, tables, seed)
    if world == 1 and args.config5_steps > 0:
        out["config5"] = config5(nm, args, tables, seed)
    if world == 1 and args.legs_steps > 0:
        out.update(legs(nm, model, x, y, vals, mask, args, tables, seed))
        if "latent28" in out:
            # (the main leg runs at args.hw x args.hw: 32 x 32 by default)
            out["latent28"]["pixel_rate_vs_main"] = round(out["latent28"]["value"] * 28 * 28 / (value * args.hw * args.hw), 3)
            out["latent28"]["main_hw"] = args.hw
    if world == 1 and args.e2e:
        out["e2e"] = e2e_sample(model, args, dev)
    if args.sharded_T > 0:
        out["sharded_sample"] = sharded_sample(model, args, dev, world, rank)
    if args.train_steps > 0:
        out["train_step"] = train_leg(args, dev, world, rank)
    if rank == 0:
        if not args.no_profile:
            xp = x.clone()
            tp = torch.full((args.batch,), args.T, dtype=torch.long, device=dev)
            nm.step_profile(xp, xp, tp, y, 0, vals, mask, args.guidance, tables, None, seed=seed)  # warm
            recs = nm.step_profile(xp, xp, tp, y, 0, vals, mask, args.guidance, tables, None, seed=seed)
            pmc, pmc_note = load_pmc()
            rl, agg = roofline(recs, pmc)
            rl["traffic_source"] = pmc_note
            out["roofline"] = rl
            if os.environ.get("DMX_BENCH_BREAKDOWN"):
                with open(os.environ["DMX_BENCH_BREAKDOWN"], "w") as f:
                    json.dump({"records": recs, "by_kernel": agg}, f, indent=1)
        if args.cpu_steps > 0 and world == 1:
            out["cpu_baseline"] = cpu_baseline(args)
            out["gpu_over_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
