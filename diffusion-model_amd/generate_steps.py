"""Drop-in ``generate_steps`` (reference generate_steps.py:1-191): the per-step trajectory dump
(BASELINE config 5) with an asynchronous output pipeline.

Same functions, keyword arguments, defaults, directory layout and PNG contents as the
reference:

    <out_root>/<run_name>/pixel/t{i}.png            decoded x_t before step i (224x224 RGB at 28x28)
    <out_root>/<run_name>/latent/ch{c:02d}/t{i}.png  per-channel min-max of x_t (grayscale)

What changes is how the frames leave the GPU.  The reference decodes, quantises, copies to the
host and encodes five PNGs synchronously before every denoising step.  Here, per saved step:

  1. on the compute stream: the native VAE decode with the uint8 quantiser fused into its last
     kernel (dmx_vae_decode, u8 HWC) and the latent min-max frames (dmx_latent_frames_u8),
     both into a device slot of a small ring;
  2. on a copy stream: one D2H copy of the slot into pinned host memory, ordered after (1)
     by an event — the next denoising step is enqueued immediately;
  3. on writer threads: wait for the copy's event, encode and write the five PNGs.

A slot is reused only after its writer finished, so at most RING frames are in flight.  The
frames are byte-identical to the reference's quantisation (the pixel quantiser is the fused
x*255 -> clamp -> truncating uint8 of reverse_to_img; the latent frames are pinned by
tests/golden/steps_T12.npz).
"""
from __future__ import annotations

import os
from concurrent.futures import Future, ThreadPoolExecutor
from pathlib import Path
from typing import List, Optional, Sequence

import numpy as np
import torch
from PIL import Image
from tqdm import tqdm

from diff import Diffuser, _native_kind
from entityCsvSampler import EntityCsvSampler


class NoiseOnlyWrapper(torch.nn.Module):
    """generate_steps.py:23-32 (defined, unused by the reference's loop)."""

    def __init__(self, model: torch.nn.Module):
        super().__init__()
        self.model = model

    def forward(self, x, t, y, cond_vals=None, cond_mask=None):
        out = self.model(x, t, y, cond_vals=cond_vals, cond_mask=cond_mask)
        if isinstance(out, (tuple, list)):
            return out[0]
        return out


def latent_frames_u8(z: torch.Tensor) -> torch.Tensor:
    """(n, c, h, w) fp32 -> (n, c, h, w) uint8 per-channel min-max frames (generate_steps.py:54-64),
    on z's device: the native kernel on a GPU tensor, the same fp32 arithmetic in torch on the host."""
    if z.is_cuda:
        from dmx import _lib
        from dmx.engine import _stream
        lib = _lib.load()
        zc = z.detach().to(torch.float32).contiguous()
        out = torch.empty(zc.shape, dtype=torch.uint8, device=zc.device)
        n, c, h, w = zc.shape
        with torch.cuda.device(zc.device):
            _lib.check(lib.dmx_latent_frames_u8(zc.data_ptr(), out.data_ptr(), n, c, h, w, _stream(zc.device)))
        return out
    zc = z.detach().to(torch.float32)
    lo = zc.amin(dim=(2, 3), keepdim=True)
    hi = zc.amax(dim=(2, 3), keepdim=True)
    nrm = torch.where(hi > lo, (zc - lo) / (hi - lo), torch.zeros_like(zc))
    return torch.from_numpy((nrm.numpy() * 255).astype(np.uint8))


def save_latent_channels_by_dir(z: torch.Tensor, step: int, latent_root: str):
    """generate_steps.py:36-66: latent/ch{c:02d}/t{step}.png, per-channel min-max grayscale."""
    frames = latent_frames_u8(z[:1]).cpu().numpy()[0]
    for c in range(frames.shape[0]):
        ch_dir = os.path.join(latent_root, f"ch{c:02d}")
        os.makedirs(ch_dir, exist_ok=True)
        Image.fromarray(frames[c], mode="L").save(os.path.join(ch_dir, f"t{step}.png"))


class FrameWriter:
    """Ring of device slots -> pinned host slots -> PNG writer threads (see module docstring)."""

    def __init__(self, device: torch.device, pix_shape, lat_shape, pixel_dir: str, latent_dir: str, ring: int = 4,
                 workers: int = 4):
        self.device = device
        self.pixel_dir, self.latent_dir = pixel_dir, latent_dir
        n_pix, n_lat = int(np.prod(pix_shape)), int(np.prod(lat_shape))
        self.pix_shape, self.lat_shape = tuple(pix_shape), tuple(lat_shape)
        self.ring = ring
        self.dev = [torch.empty(n_pix + n_lat, dtype=torch.uint8, device=device) for _ in range(ring)]
        self.host = [torch.empty(n_pix + n_lat, dtype=torch.uint8, pin_memory=True) for _ in range(ring)]
        self.events: List[Optional[torch.cuda.Event]] = [None] * ring
        self.pending: List[Optional[Future]] = [None] * ring
        self.copy_stream = torch.cuda.Stream(device)
        self.pool = ThreadPoolExecutor(max_workers=workers)
        self.n_pix = n_pix
        self.k = 0
        for c in range(self.lat_shape[0]):
            os.makedirs(os.path.join(latent_dir, f"ch{c:02d}"), exist_ok=True)

    def slot(self) -> int:
        s = self.k % self.ring
        if self.pending[s] is not None:
            self.pending[s].result()  # the writer of this slot's previous frame is done
            self.pending[s] = None
        return s

    def submit(self, x: torch.Tensor, vae, step: int) -> None:
        """Decode x (1, C, H, W) and its latent frames into a slot; copy and write asynchronously."""
        s = self.slot()
        buf = self.dev[s]
        pix = buf[: self.n_pix].view(self.pix_shape)
        lat = buf[self.n_pix:].view((1,) + self.lat_shape)
        vae.native().decode_u8_into(x, pix.view((1,) + self.pix_shape))
        lat.copy_(latent_frames_u8(x))
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.copy_stream):
            self.copy_stream.wait_event(ev)
            self.host[s].copy_(buf, non_blocking=True)
            done = torch.cuda.Event()
            done.record(self.copy_stream)
        buf.record_stream(self.copy_stream)
        self.pending[s] = self.pool.submit(self._write, s, done, step)
        self.k += 1

    def _write(self, s: int, done: "torch.cuda.Event", step: int) -> None:
        done.synchronize()
        h = self.host[s].numpy()
        Image.fromarray(h[: self.n_pix].reshape(self.pix_shape)).save(os.path.join(self.pixel_dir, f"t{step}.png"))
        lat = h[self.n_pix:].reshape(self.lat_shape)
        for c in range(lat.shape[0]):
            Image.fromarray(lat[c], mode="L").save(os.path.join(self.latent_dir, f"ch{c:02d}", f"t{step}.png"))

    def drain(self) -> None:
        for i, f in enumerate(self.pending):
            if f is not None:
                f.result()
                self.pending[i] = None

    def close(self) -> None:
        self.drain()
        self.pool.shutdown(wait=True)


def _save_sync(x, vae, diffuser, step, pixel_dir, latent_dir):
    """The reference's synchronous per-step output (foreign / host models)."""
    img = vae.decode(x)
    img = img.clamp(0, 1)
    diffuser.reverse_to_img(img[0]).save(os.path.join(pixel_dir, f"t{step}.png"))
    save_latent_channels_by_dir(z=x, step=step, latent_root=latent_dir)


@torch.no_grad()
def save_reverse_steps_for_csv_row(
    *,
    csv_path: str,
    row_index: int,
    class_id: int,
    model: torch.nn.Module,
    vae: torch.nn.Module,
    device: str = "cuda",
    num_timesteps: int = 1000,
    z_shape: tuple = (1, 4, 28, 28),
    guidance_scale: float = 3.0,
    null_label: int = 0,
    save_steps: Optional[Sequence[int]] = None,
    save_every: Optional[int] = None,
    run_name: Optional[str] = None,
    out_root: str = "./step_images",
    base_wh: tuple = (400, 400),
    progress: bool = True,
    noise_source: str = "host",
) -> str:
    """generate_steps.py:72-191.  `noise_source` (dmx extension): "host" draws x_T and every step's
    noise from the global CPU generator in the reference CPU path's order; "device" uses Philox
    noise and graph-replayed steps."""
    device_t = torch.device(device)
    B = z_shape[0]
    if B != 1:
        raise ValueError("このスクリプトは 'n番目の行だけ' 用なので z_shape[0] は 1 を推奨します。")
    if run_name is None:
        entity = ["line", "circle", "arc"]
        run_name = f"class_{entity[int(class_id) - 1]}_row{int(row_index):05d}"
    out_dir = os.path.join(out_root, run_name)
    pixel_dir = os.path.join(out_dir, "pixel")
    latent_dir = os.path.join(out_dir, "latent")
    Path(pixel_dir).mkdir(parents=True, exist_ok=True)
    Path(latent_dir).mkdir(parents=True, exist_ok=True)

    diffuser = Diffuser(num_timesteps=num_timesteps, device=device_t)
    diffuser.noise_source = noise_source
    sampler = EntityCsvSampler(diffuser=diffuser, model=model, vae=vae, class_id=class_id, base_wh=base_wh,
                               device=device_t)
    vals, mask = sampler.load_cond(csv_path, count=1, start=row_index)
    y = torch.tensor([int(class_id)], device=device_t, dtype=torch.long)
    model_noise = model.to(device_t)
    model_noise.eval()
    vae.eval()

    x = diffuser._randn(z_shape, device_t)  # x_T: the CPU generator, as the reference's CPU path

    if save_steps is not None:
        save_set = set(int(s) for s in save_steps)
    elif save_every is not None:
        step = max(int(save_every), 1)
        save_set = set(range(num_timesteps, 0, -step))
        save_set.add(1)
    else:
        save_set = set(range(1, num_timesteps + 1))

    native = device_t.type == "cuda" and _native_kind(vae) == 4 and _native_kind(model) in (1, 2)
    writer = None
    if native:
        H, W = z_shape[2], z_shape[3]
        writer = FrameWriter(device_t, (8 * H, 8 * W, 3), (z_shape[1], H, W), pixel_dir, latent_dir)
    bar = tqdm(total=num_timesteps, desc=f"Reverse diffusion (row={row_index})") if progress else None
    device_loop = native and noise_source == "device" and guidance_scale and guidance_scale > 0
    if device_loop:
        nm = model_noise.native()
        x_state = x.contiguous().clone()  # stepped in place: the captured graph keeps its pointer
        t_dev = torch.full((1,), num_timesteps, device=device_t, dtype=torch.long)
        tables = diffuser.coef_tables(device_t, clamp_prev=True)
        seed = diffuser._seed()
        v, m = vals.float().contiguous(), mask.float().contiguous()

    def run(i_from, i_to, x):
        if device_loop:
            if x is not x_state:
                x_state.copy_(x)
            x = x_state
        for i in range(i_from, i_to, -1):
            # save (before denoising = x_t), generate_steps.py:162-174
            if i in save_set:
                if writer is not None:
                    writer.submit(x, vae, i)
                else:
                    _save_sync(x, vae, diffuser, i, pixel_dir, latent_dir)
            if device_loop:  # one graph-replayed step, t decremented on the device
                t_dev.fill_(i)
                nm.sample_loop(x, t_dev, y, null_label, v, m, float(guidance_scale), tables, 1, seed=seed)
            else:  # generate_steps.py:179-189 (i in [1, T]: denoise_cond's range assert holds)
                t = torch.full((B,), i, device=device_t, dtype=torch.long)
                x = diffuser._denoise_cond(model_noise, x, t, y, guidance_scale, null_label, vals, mask)
            if bar is not None:
                bar.update(1)
        return x.clone() if device_loop else x  # the guard keeps the chunk's input for a replay

    try:
        x = diffuser._guarded_host_loop(model_noise, x, run, on_replay=writer.drain if writer else None)
    finally:
        if writer is not None:
            writer.close()
        if bar is not None:
            bar.close()
    save_reverse_steps_for_csv_row.last_latent = x
    return out_dir
