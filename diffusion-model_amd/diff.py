"""Drop-in ``diff`` module: the DDPM scheduler and samplers of the reference
(reference diff.py:10-369) running on the MI355X-native engine.

Call surface, defaults, exception types and RNG draw order are the reference's.
What changes is where the work happens:

* ``denoise_cond`` with CFG on a dmx network batches the uncond/cond forwards into
  one 2B-sample native forward and fuses out-head + CFG mix + DDPM update into one
  kernel (libdmx ``dmx_step``); any other (duck-typed) model is called exactly like
  the reference and only the update runs natively (``dmx_ddpm_update``).
* ``noise_source``:
    - ``"host"`` (default): every Gaussian draw comes from the global torch CPU
      generator in the reference's order (optional encode draw, x_T, one draw per
      step) and is copied to the device — results match the reference PyTorch-CPU
      path on identical seeds;
    - ``"device"``: counter-based Philox on the GPU keyed by (seed, t, global sample
      index); the T loop then runs as replayed hipGraphs with no host round trip.
* Schedule tables are built on the host with the reference's fp32 torch ops, so
  the per-t coefficients are bit-identical to the reference CPU path.
"""
from __future__ import annotations

import os
import queue
import sys
import threading
from typing import Dict, Iterable, List, Optional, Tuple, Union

import numpy as np
import torch
from tqdm import tqdm

_ROOT = os.path.dirname(os.path.abspath(__file__))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from dmx import engine as _engine  # noqa: E402

KEY_ORDER = ["x1", "y1", "x2", "y2", "cx", "cy", "cr", "ax", "ay", "ar", "theta1", "theta2"]
CLASS_KEYS = {1: ["x1", "y1", "x2", "y2"], 2: ["cx", "cy", "cr"], 3: ["ax", "ay", "ar", "theta1", "theta2"]}


def _native_kind(model) -> int:
    """libdmx kind of a dmx drop-in network, 0 for foreign (duck-typed) models."""
    return int(getattr(type(model), "_dmx_kind", 0)) if hasattr(model, "native") else 0


class _NoisePrefetch:
    """The next `n` per-step noise draws of a sampler chunk, made on a helper thread from the
    global CPU generator — in the reference's order, nothing else draws meanwhile — into pinned
    buffers, so the host draw (~2 ms at B=64, single-threaded in torch) overlaps the GPU step
    instead of preceding it.  torch.randn(shape, out=buf) consumes the generator exactly like
    torch.randn(shape)."""

    def __init__(self, shape, n: int, depth: int = 2, rows=None):
        self.shape, self.n = tuple(int(v) for v in shape), int(n)
        self.rows = rows  # (start, end): only these rows of each draw go to the device (a rank's shard)
        self.bufs = [torch.empty(self.shape, pin_memory=True) for _ in range(depth + 2)]
        self.events = [None] * len(self.bufs)
        self.q: "queue.Queue" = queue.Queue(maxsize=depth)
        self.err = None
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()

    def _run(self):
        try:
            for k in range(self.n):
                j = k % len(self.bufs)
                if self.events[j] is not None:
                    self.events[j].synchronize()  # the H2D copy that last read this buffer is done
                torch.randn(self.shape, out=self.bufs[j])
                self.q.put(k)
        except BaseException as e:  # surfaced to the consumer
            self.err = e
            self.q.put(-1)

    def next(self, device):
        k = self.q.get()
        if k < 0:
            raise self.err
        j = k % len(self.bufs)
        src = self.bufs[j] if self.rows is None else self.bufs[j][self.rows[0]:self.rows[1]]
        out = src.to(device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        self.events[j] = ev
        return out

    def close(self):
        while self.thread.is_alive():  # the consumer stopped early: let the producer finish its draws
            try:
                self.q.get(timeout=0.05)
            except queue.Empty:
                pass
        self.thread.join()


class Diffuser:
    def __init__(self, num_timesteps=1000, beta_start=0.0001, beta_end=0.02, device="cpu"):
        # diff.py:11-16, evaluated on the CPU (torch's CPU cumprod accumulates in double)
        self.num_timesteps = num_timesteps
        self.device = device
        betas = torch.linspace(beta_start, beta_end, num_timesteps)
        alphas = 1 - betas
        alpha_bars = torch.cumprod(alphas, dim=0)
        self.betas = betas.to(device)
        self.alphas = alphas.to(device)
        self.alpha_bars = alpha_bars.to(device)
        self._host = (alphas, alpha_bars)
        self._tables: Dict[Tuple[str, bool], Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = {}
        self.noise_source = "host"
        self.use_graph = True
        self.range_fallbacks = 0  # chunks recomputed in fp32 by the range guard

    # ---- schedule tables (per t-1) ---------------------------------------------------------
    def coef_tables(self, device, clamp_prev: bool = True):
        """(c1, c2, sd) with c1 = (1-a)/sqrt(1-ab), c2 = sqrt(a), sd = posterior std.

        clamp_prev=True follows denoise_cond (diff.py:144), False follows denoise's
        wrap-around ``alpha_bars[t_idx-1]`` (diff.py:39)."""
        key = (str(device), clamp_prev)
        if key not in self._tables:
            a, ab = self._host
            idx = torch.arange(self.num_timesteps)
            prev = torch.clamp(idx - 1, min=0) if clamp_prev else idx - 1
            abp = ab[prev]
            c1 = (1 - a) / torch.sqrt(1 - ab)
            c2 = torch.sqrt(a)
            sd = torch.sqrt((1 - a) * (1 - abp) / (1 - ab))
            self._tables[key] = tuple(v.contiguous().to(device) for v in (c1, c2, sd))
        return self._tables[key]

    # ---- RNG -------------------------------------------------------------------------------
    _NOISE_RING = 3

    def _randn(self, shape, device):
        """One Gaussian draw in the reference's order (host mode) — diff.py:104,158,327.

        The draw is the global CPU generator's (torch.randn(shape, out=...) consumes it exactly like
        torch.randn(shape)).  For a GPU destination it lands in a small ring of pinned host buffers
        and goes up with a non-blocking copy, so the host draws step k+1's noise while the GPU runs
        step k (a pageable copy would block the host until the stream drained)."""
        shape = tuple(int(v) for v in shape)
        dev = torch.device(device)
        if dev.type != "cuda":
            return torch.randn(shape).to(dev)
        ring = self.__dict__.setdefault("_noise_ring", {})
        key = (shape, str(dev))
        slots = ring.get(key)
        if slots is None:
            slots = ring[key] = [[torch.empty(shape, pin_memory=True), None] for _ in range(self._NOISE_RING)]
            self.__dict__.setdefault("_noise_next", {})[key] = 0
        k = self._noise_next[key]
        self._noise_next[key] = (k + 1) % len(slots)
        buf, ev = slots[k]
        if ev is not None:
            ev.synchronize()  # the copy that last read this pinned slot has finished
        torch.randn(shape, out=buf)
        out = buf.to(dev, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        slots[k][1] = ev
        return out

    def _step_noise(self, x):
        if self.noise_source == "host":
            pf = self.__dict__.get("_prefetch")
            if pf is not None and x.is_cuda and tuple(x.shape) == pf.shape:
                return pf.next(x.device)
            return self._randn(x.shape, x.device)
        return None

    def _seed(self) -> int:
        return int(torch.randint(0, 2 ** 62, (1,)).item())

    # ---- training-side helper (not on the sampling path) ------------------------------------
    def add_noise(self, x_0, t):
        """diff.py:18-30 — forward diffusion used by training (plain torch; not a dmx path)."""
        assert (t >= 1).all() and (t <= self.num_timesteps).all()
        ab = self.alpha_bars[t - 1].view(-1, 1, 1, 1)
        noise = torch.randn_like(x_0, device=self.device)
        return torch.sqrt(ab) * x_0 + torch.sqrt(1 - ab) * noise, noise

    # ---- one step -----------------------------------------------------------------------------
    def denoise(self, model, x, t):
        """Unconditional DDPM step (diff.py:32-56)."""
        T = self.num_timesteps
        assert (t >= 1).all() and (t <= T).all()
        tables = self.coef_tables(x.device, clamp_prev=False)
        model.eval()
        if _native_kind(model) and x.is_cuda and getattr(model, "_dmx_kind", 0) == 3:
            model.train()
            noise = self._step_noise(x)
            out = torch.empty_like(x)
            model.native().step(x, out, t.to(x.device), None, 0, None, None, 0.0, tables, noise,
                                seed=self._seed() if noise is None else 0)
            return out
        with torch.no_grad():
            eps = model(x, t)
        model.train()
        noise = self._step_noise(x)
        return _engine.ddpm_update(x, eps, None, 0.0, t, tables, noise, seed=self._seed() if noise is None else 0)

    def reverse_to_img(self, x):
        """diff.py:58-64: x*255 -> clamp(0,255) -> uint8 (truncation) -> PIL."""
        from PIL import Image
        a = (x * 255).clamp(0, 255).to(torch.uint8).cpu().numpy()
        if a.ndim == 3:
            a = np.transpose(a, (1, 2, 0))
            if a.shape[2] == 1:
                a = a[:, :, 0]
        return Image.fromarray(a)

    def denoise_cond(self, model, x, t, y=None, guidance_scale=0.0, null_label=0, cond_vals=None, cond_mask=None):
        """One DDPM step with optional classifier-free guidance (diff.py:127-162)."""
        T = self.num_timesteps
        assert (t >= 1).all() and (t <= T).all()  # (reads t back: a device sync, as in the reference)
        return self._denoise_cond(model, x, t, y, guidance_scale, null_label, cond_vals, cond_mask)

    def _denoise_cond(self, model, x, t, y=None, guidance_scale=0.0, null_label=0, cond_vals=None, cond_mask=None):
        """denoise_cond after the range check — the samplers' own loops build t from a host-known
        step in [1, T] and call this directly, so the host never waits on the device per step."""
        tables = self.coef_tables(x.device, clamp_prev=True)
        with torch.no_grad():
            if guidance_scale and y is not None and guidance_scale > 0:
                kind = _native_kind(model)
                if kind in (1, 2) and x.is_cuda:
                    noise = self._step_noise(x)
                    out = torch.empty_like(x)
                    use = cond_vals is not None and cond_mask is not None
                    model.native().step(x.contiguous(), out, t.to(x.device), y.to(x.device), null_label,
                                        cond_vals if use else None, cond_mask if use else None,
                                        float(guidance_scale), tables, noise,
                                        seed=self._seed() if noise is None else 0)
                    return out
                y_null = torch.full_like(y, null_label)
                eps_uncond, _ = model(x, t, y_null, cond_vals=cond_vals, cond_mask=cond_mask)
                eps_cond, _ = model(x, t, y, cond_vals=cond_vals, cond_mask=cond_mask)
                noise = self._step_noise(x)
                return _engine.ddpm_update(x, eps_uncond, eps_cond, float(guidance_scale), t, tables, noise,
                                           seed=self._seed() if noise is None else 0)
            else:
                # plain conditional/unconditional — mirrors diff.py:152-156 literally, including
                # its UnboundLocalError when y is given without guidance
                if y is None:
                    y = torch.full((x.size(0),), null_label, device=x.device, dtype=torch.long)
                    eps = model(x, t, y, cond_vals=cond_vals, cond_mask=cond_mask)
        noise = self._step_noise(x)
        if not isinstance(eps, torch.Tensor):
            raise TypeError(f"unsupported operand type(s) for *: 'Tensor' and '{type(eps).__name__}'")
        return _engine.ddpm_update(x, eps, None, 0.0, t, tables, noise, seed=self._seed() if noise is None else 0)

    # ---- loops --------------------------------------------------------------------------------
    def sample(self, model, x_shape=(20, 3, 80, 80)):
        """Pixel-space sampler (diff.py:66-85)."""
        batch_size = x_shape[0]
        x = self._randn(x_shape, self.device)
        for i in tqdm(range(self.num_timesteps, 0, -1)):
            t = torch.tensor([i] * batch_size, device=self.device, dtype=torch.long)
            x = self.denoise(model, x, t)
        return [self.reverse_to_img(x[i]) for i in range(batch_size)]

    def sample_latent(self, model, z_shape=(1000, 4, 28, 28), vae=None, to_pil=True, progress=True):
        """Latent sampler, unconditional model (diff.py:87-125)."""
        batch_size = z_shape[0]
        x = self._randn(z_shape, self.device)
        bar = tqdm(total=self.num_timesteps) if progress else None

        def run(i_from, i_to, x):
            for i in range(i_from, i_to, -1):
                t = torch.full((batch_size,), i, device=self.device, dtype=torch.long)
                x = self.denoise(model, x, t)
                if bar is not None:
                    bar.update(1)
            return x

        with torch.no_grad():
            x = self._guarded_host_loop(model, x, run)
        if bar is not None:
            bar.close()
        if vae is None:
            return x
        return self._decode(vae, x, to_pil)

    # ---- split-precision range guard ------------------------------------------------------
    GUARD_CHUNK = 50

    @staticmethod
    def _guard_target(model):
        """The NativeModel whose range flag guards this loop (None: foreign model or exact fp32)."""
        if not _native_kind(model):
            return None
        nm = model.native()
        return nm if nm.precision != "fp32" else None

    def _guarded_host_loop(self, model, x, run, on_replay=None):
        """T steps in chunks of GUARD_CHUNK.  After each chunk the model's range flag is read
        (dmx_model_range_check); if an operand left the f16 range of the split-precision modes
        the chunk is replayed from its start — same x, same CPU-generator state, hence the same
        draws — in exact-fp32 MFMA mode.  `run(i_from, i_to, x)` advances t = i_from .. i_to + 1."""
        T = self.num_timesteps
        nm = self._guard_target(model) if x.is_cuda else None
        prefetch = x.is_cuda and self.noise_source == "host" and _native_kind(model) != 0
        i = T
        while i >= 1:
            j = max(i - self.GUARD_CHUNK, 0)
            x0, rng = x, torch.get_rng_state()
            x = self._run_chunk(run, i, j, x, prefetch)
            if nm is not None and nm.range_tripped():
                if on_replay is not None:
                    on_replay()
                torch.set_rng_state(rng)
                with nm.precision_override("fp32"):
                    x = self._run_chunk(run, i, j, x0, prefetch)
                nm.range_tripped()  # clear
                self.range_fallbacks += 1
            i = j
        return x

    def _run_chunk(self, run, i, j, x, prefetch):
        if not prefetch:
            return run(i, j, x)
        self._prefetch = _NoisePrefetch(x.shape, i - j)
        try:
            return run(i, j, x)
        finally:
            pf, self._prefetch = self._prefetch, None
            pf.close()

    def sample_cond(self, model, x_shape, y, guidance_scale=0.0, null_label=0):
        """diff.py:165-172."""
        batch_size = x_shape[0]
        assert y.shape[0] == batch_size
        x = self._randn(x_shape, self.device)
        for i in range(self.num_timesteps, 0, -1):
            t = torch.full((batch_size,), i, device=self.device, dtype=torch.long)
            x = self.denoise_cond(model, x, t, y=y, guidance_scale=guidance_scale, null_label=null_label)
        return x

    def _decode(self, vae, x, to_pil):
        """Decode latents; dmx VAEs emit the uint8 HWC images directly (diff.py:346-369)."""
        if _native_kind(vae) == 4 and x.is_cuda:
            img, u8 = vae.native().decode(x, want_img=not to_pil, want_u8=to_pil)
            if to_pil:
                from PIL import Image
                arr = u8.cpu().numpy()
                return [Image.fromarray(arr[i]) for i in range(arr.shape[0])]
            return img
        vae.eval()
        outs = []
        with torch.inference_mode():
            for s in range(0, x.shape[0], 4):
                outs.append(vae.decode(x[s:s + 4]))
        images = torch.cat(outs, dim=0)
        return [self.reverse_to_img(images[i]) for i in range(images.shape[0])] if to_pil else images

    @staticmethod
    def _norm_counts(cc) -> List[Tuple[int, int]]:
        """diff.py:206-218."""
        if isinstance(cc, dict):
            items = list(cc.items())
        elif isinstance(cc, tuple) and len(cc) == 2:
            items = [cc]
        elif isinstance(cc, list):
            items = list(cc)
        else:
            raise ValueError("class_counts は {cls:num}, (cls,num), そのリストのいずれか。")
        items = [(int(c), int(n)) for c, n in items if int(n) > 0]
        if not items:
            raise ValueError("生成枚数が0です。")
        return items

    def _build_cond(self, y_list, cond, cond_mask, key_order, class_keys, device):
        """(B,K) vals/mask from tensor / dict / list inputs (diff.py:229-312)."""
        B = len(y_list)
        if key_order is None:
            key_order = list(KEY_ORDER)
        K = len(key_order)
        kidx = {k: i for i, k in enumerate(key_order)}
        if class_keys is None:
            class_keys = CLASS_KEYS
        vals = cond.to(device) if isinstance(cond, torch.Tensor) else None
        msk = cond_mask.to(device) if isinstance(cond_mask, torch.Tensor) else None
        if vals is not None:
            if vals.ndim != 2 or vals.shape[0] != B or vals.shape[1] != K:
                raise ValueError(f"cond Tensor 形状は (B={B}, K={K}) 必須: got {tuple(vals.shape)}")
            if msk is None:
                msk = (vals != 0).float()
            elif msk.ndim != 2 or msk.shape != vals.shape:
                raise ValueError("cond_mask Tensor 形状は cond と同じ (B,K) 必須。")
            return vals, msk
        vals = torch.zeros((B, K), device=device, dtype=torch.float32)
        if msk is None:
            msk = torch.zeros((B, K), device=device, dtype=torch.float32)
        if isinstance(cond, dict):
            for i, cls in enumerate(y_list):
                if cls in cond:
                    for k, v in cond[cls].items():
                        if k not in kidx:
                            continue
                        vals[i, kidx[k]] = float(v)
                        explicit = isinstance(cond_mask, dict) and cls in cond_mask and k in cond_mask[cls]
                        msk[i, kidx[k]] = float(cond_mask[cls][k]) if explicit else 1.0
                if isinstance(cond_mask, dict) and cls in cond_mask:
                    for k, mv in cond_mask[cls].items():
                        if k in kidx:
                            msk[i, kidx[k]] = float(mv)
        elif isinstance(cond, list):
            if len(cond) != B:
                raise ValueError(f"cond(list) の長さ {len(cond)} が生成枚数 {B} と不一致。")
            for i, d in enumerate(cond):
                for k, v in d.items():
                    if k not in kidx:
                        continue
                    vals[i, kidx[k]] = float(v)
                    explicit = isinstance(cond_mask, list) and i < len(cond_mask) and k in cond_mask[i]
                    msk[i, kidx[k]] = float(cond_mask[i][k]) if explicit else 1.0
            if isinstance(cond_mask, list) and len(cond_mask) == B:
                for i, d in enumerate(cond_mask):
                    for k, mv in d.items():
                        if k in kidx:
                            msk[i, kidx[k]] = float(mv)
        else:
            for i, cls in enumerate(y_list):
                for k in class_keys.get(cls, []):
                    if k in kidx:
                        msk[i, kidx[k]] = 1.0
        return vals, msk

    def _latent_shape(self, vae, dummy_input_hw, device):
        """z_shape inference (diff.py:315-322).  For a dmx VAE the encoder is not run:
        the shape follows from its conv arithmetic and its randn_like draw
        (models/vae.py:56) is replayed so the global RNG stream stays aligned."""
        H, W = dummy_input_hw
        if _native_kind(vae) == 4:
            from models.vae import latent_hw
            h, w = latent_hw(H, W)
            if self.noise_source == "host":
                torch.randn((1, vae.z_channels, h, w))
            return vae.z_channels, h, w
        with torch.no_grad():
            z, _ = vae.encode(torch.zeros(1, 3, H, W, device=device))
        return tuple(z.shape[1:])

    def sample_latent_cond(
        self,
        model,
        class_counts: Union[Dict[int, int], Tuple[int, int], List[Tuple[int, int]]],
        z_shape: Tuple[int, int, int] = None,
        vae=None,
        to_pil: bool = True,
        progress: bool = True,
        guidance_scale: float = 3.0,
        null_label: int = 0,
        dummy_input_hw: Tuple[int, int] = (224, 224),
        cond=None,
        cond_mask=None,
        key_order: Optional[List[str]] = None,
        class_keys: Optional[Dict[int, List[str]]] = None,
    ):
        """Class + numeric-condition latent sampler (diff.py:174-369)."""
        device = self.device
        items = self._norm_counts(class_counts)
        y_list: List[int] = []
        for cls, num in items:
            y_list += [cls] * num
        B = len(y_list)
        y = torch.tensor(y_list, device=device, dtype=torch.long)
        vals, msk = self._build_cond(y_list, cond, cond_mask, key_order, class_keys, device)

        if z_shape is None:
            if vae is None:
                raise ValueError("z_shape 省略時は vae が必要です。")
            C, Hlat, Wlat = self._latent_shape(vae, dummy_input_hw, device)
        else:
            C, Hlat, Wlat = z_shape

        x = self._randn((B, C, Hlat, Wlat), device)
        x = self._run_cond_loop(model, x, y, vals, msk, guidance_scale, null_label, progress)
        if vae is None:
            return x
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        return self._decode(vae, x, to_pil)

    def _run_cond_loop(self, model, x, y, vals, msk, guidance_scale, null_label, progress):
        """The T loop (diff.py:328-344), range-guarded in chunks (_guarded_host_loop)."""
        T = self.num_timesteps
        native = _native_kind(model) in (1, 2) and x.is_cuda and guidance_scale and guidance_scale > 0
        bar = tqdm(total=T, desc="Sampling (cond+numeric)") if progress else None
        if native and self.noise_source == "device":
            # whole loop on the device: Philox noise, hipGraph replay, t decremented in-graph
            nm = model.native()
            x = x.contiguous().clone()
            t_dev = torch.full((1,), T, device=x.device, dtype=torch.long)
            tables = self.coef_tables(x.device, clamp_prev=True)
            seed = self._seed()
            v, m = vals.float().contiguous(), msk.float().contiguous()
            guard = self._guard_target(model)
            done = 0
            with torch.no_grad():
                while done < T:
                    k = min(self.GUARD_CHUNK, T - done)
                    x0 = x.clone() if guard is not None else None
                    nm.sample_loop(x, t_dev, y, null_label, v, m, float(guidance_scale), tables, k, seed=seed,
                                   use_graph=self.use_graph)
                    if guard is not None and guard.range_tripped():
                        x.copy_(x0)
                        t_dev.fill_(T - done)
                        with guard.precision_override("fp32"):
                            nm.sample_loop(x, t_dev, y, null_label, v, m, float(guidance_scale), tables, k,
                                           seed=seed, use_graph=self.use_graph)
                        guard.range_tripped()
                        self.range_fallbacks += 1
                    done += k
                    if bar is not None:
                        bar.update(k)
            if bar is not None:
                bar.close()
            return x

        def run(i_from, i_to, x):
            for i in range(i_from, i_to, -1):  # i in [1, T]: denoise_cond's assert holds by construction
                t = torch.full((x.shape[0],), i, device=x.device, dtype=torch.long)
                x = self._denoise_cond(model, x, t, y, guidance_scale, null_label, vals, msk)
                if bar is not None:
                    bar.update(1)
            return x

        with torch.no_grad():
            x = self._guarded_host_loop(model, x, run)
        if bar is not None:
            bar.close()
        return x
