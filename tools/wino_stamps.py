"""Winograd conv phase timing from a DMX_DIAG diagnostic build (MI355X only).

  DMX_LIB=libwstamp.so python tools/wino_stamps.py [out.json]

Runs one eager 128-sample U-Net forward (the bench's CFG batch), then reads every Winograd launch's
per-block s_memtime stamps (igemm_wino.h WSTAMP: start, after the prologue barrier, after the chunk
loop, end) and prints per launch: blocks, wall span, and the median per-block prologue / loop /
epilogue cycles, with the number of blocks each CU ran.  Timing only (s_memtime ticks = shader
clock cycles)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "diffusion-model_amd"))
from dmx import _lib, engine, synth  # noqa: E402
from models.unet_cond_geom import UnetCondWithGeomHead  # noqa: E402

SLOTS, BLOCKS = 32, 2048


def main():
    dev = torch.device("cuda:0")
    m = UnetCondWithGeomHead()
    m.load_state_dict(synth.unet_cond_geom_weights(0))
    m = m.to(dev).eval()
    g = torch.Generator().manual_seed(1)
    N = 128
    x = torch.randn((N, 4, 32, 32), generator=g).to(dev)
    t = torch.randint(1, 1001, (N,), generator=g).to(dev)
    y = torch.randint(0, 4, (N,), generator=g).to(dev)
    vals = torch.rand((N, 12), generator=g).to(dev)
    mask = torch.ones((N, 12), device=dev)
    lib = _lib.load()
    with torch.no_grad():
        for _ in range(3):  # warm
            m(x, t, y, cond_vals=vals, cond_mask=mask)
        torch.cuda.synchronize()
        lib.dmx_diag_wino_stamps(None, 0)  # reset: the next forward's launches stamp slots 0..
        m(x, t, y, cond_vals=vals, cond_mask=mask)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (SLOTS * BLOCKS * 5))()
    n = lib.dmx_diag_wino_stamps(buf, len(buf))
    if n <= 0:
        print("no stamps (not a DMX_DIAG build?)", n)
        return
    a = np.frombuffer(buf, dtype=np.uint64).reshape(SLOTS, BLOCKS, 5).astype(np.int64)
    out = []
    for s in range(SLOTS):
        blk = a[s]
        used = blk[:, 0] > 0
        if not used.any():
            continue
        b = blk[used]
        pro, loop, epi = b[:, 1] - b[:, 0], b[:, 2] - b[:, 1], b[:, 3] - b[:, 2]
        span = int(b[:, 3].max() - b[:, 0].min())
        cu = b[:, 4] & 0xFFFFFFFF
        cuid = ((cu >> 8) & 0xF) | (((cu >> 13) & 0x7) << 4) | (((b[:, 4] >> 32) & 0xF) << 8)
        _, per_cu = np.unique(cuid, return_counts=True)
        r = {"slot": s, "blocks": int(used.sum()), "span_cyc": span,
             "prologue_med": int(np.median(pro)), "loop_med": int(np.median(loop)), "epilogue_med": int(np.median(epi)),
             "block_med": int(np.median(b[:, 3] - b[:, 0])), "cus": int(len(per_cu)), "max_blocks_per_cu": int(per_cu.max())}
        out.append(r)
        print(r)
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
