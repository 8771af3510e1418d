"""Drop-in ``eval_iou_noise`` (reference eval_iou_noise.py): generated-image quality metrics
with the per-pair work — binarisation, exact Euclidean distance transform, IoU / GT-IoU,
far-noise ratio, Gaussian-weighted recall — in one HIP kernel launch for a whole batch of
pairs (libdmx ``dmx_eval_metrics``, csrc/eval.h).

Same names, arguments, defaults, return values and exceptions as the reference functions
(eval_iou_noise.py:52-298) plus ``compute_metrics_batch`` and ``evaluate`` (the body of the
reference's ``main``, eval_iou_noise.py:303-482, callable without argparse).  The metric
functions run on a GPU and raise ``DmxUnavailable`` without one (no host fallback).
"""
from __future__ import annotations

import argparse
import re
import sys
from concurrent.futures import ThreadPoolExecutor
from datetime import datetime
from pathlib import Path
from typing import Dict, List, Sequence, Tuple

import numpy as np
import pandas as pd
import torch
from PIL import Image

from dmx import _lib

_DT_BACKEND = "dmx"  # exact EDT on the GPU (the reference's scipy backend, bit for bit)

METRIC_KEYS = ("iou", "gt_iou", "far_noise_ratio", "gauss_recall", "inter", "union", "gt_area", "pred_area", "fp")

P_GT = re.compile(r"^p(\d+)\.jpg$", re.IGNORECASE)
P_GEN = re.compile(r"^pic(\d+)\.png$", re.IGNORECASE)


def _extract_gt_index(name: str):
    m = P_GT.match(name)
    return int(m.group(1)) if m else None


def _extract_gen_index(name: str):
    m = P_GEN.match(name)
    return int(m.group(1)) if m else None


def list_gt_files(gt_dir: Path) -> List[Tuple[int, Path]]:
    files = [(i, p) for p in Path(gt_dir).iterdir() if p.is_file() and (i := _extract_gt_index(p.name)) is not None]
    return sorted(files, key=lambda x: x[0])


def list_gen_files(gen_dir: Path) -> List[Tuple[int, Path]]:
    files = [(i, p) for p in Path(gen_dir).iterdir() if p.is_file() and (i := _extract_gen_index(p.name)) is not None]
    return sorted(files, key=lambda x: x[0])


def load_gray(image_path: Path) -> np.ndarray:
    """PIL decode + convert("L") (eval_iou_noise.py:86-87)."""
    return np.array(Image.open(image_path).convert("L"), dtype=np.uint8)


def load_binary_mask(image_path: Path, threshold: int = 128, invert: bool = True) -> np.ndarray:
    """eval_iou_noise.py:77-94."""
    arr = load_gray(image_path)
    return (arr < threshold) if invert else (arr >= threshold)


def mask_to_pil(mask: np.ndarray) -> Image.Image:
    return Image.fromarray(mask.astype(np.uint8) * 255, mode="L")


def save_side_by_side(gt_mask: np.ndarray, gen_mask: np.ndarray, out_path: Path) -> None:
    """eval_iou_noise.py:103-119 (left = GT, right = GEN)."""
    gt_img, gen_img = mask_to_pil(gt_mask), mask_to_pil(gen_mask)
    w, h = gt_img.size
    if gen_img.size != (w, h):
        gen_img = gen_img.resize((w, h), resample=Image.NEAREST)
    canvas = Image.new("L", (w * 2, h), color=0)
    canvas.paste(gt_img, (0, 0))
    canvas.paste(gen_img, (w, 0))
    canvas.save(out_path)


def save_diff_visual(gt_mask: np.ndarray, gen_mask: np.ndarray, out_path: Path) -> None:
    """eval_iou_noise.py:122-156: white background, TP black, FN blue, FP red."""
    rgb = np.full(gt_mask.shape + (3,), 255, dtype=np.uint8)
    rgb[np.logical_and(gt_mask, gen_mask)] = (0, 0, 0)
    rgb[np.logical_and(gt_mask, ~gen_mask)] = (0, 0, 255)
    rgb[np.logical_and(gen_mask, ~gt_mask)] = (255, 0, 0)
    Image.fromarray(rgb, mode="RGB").save(out_path)


# ---- native metrics -------------------------------------------------------------------------
def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise _lib.DmxUnavailable("eval_iou_noise metrics run on an MI355X (HIP) device; none is available")
    return torch.device("cuda", torch.cuda.current_device())


def _metrics_native(gts: np.ndarray, preds: np.ndarray, sigma: float, gray: bool = False, threshold: int = 128,
                    invert: bool = True) -> np.ndarray:
    """(n, h, w) masks (or grayscale with gray=True) -> (n, 9) float64 via dmx_eval_metrics."""
    from dmx.engine import _stream
    lib = _lib.load()
    dev = _device()
    g = torch.from_numpy(np.ascontiguousarray(gts, dtype=np.uint8)).to(dev)
    p = torch.from_numpy(np.ascontiguousarray(preds, dtype=np.uint8)).to(dev)
    n, h, w = g.shape
    ws = torch.empty((n, h, w), dtype=torch.int32, device=dev)
    out = torch.empty((n, len(METRIC_KEYS)), dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        _lib.check(lib.dmx_eval_metrics(g.data_ptr(), p.data_ptr(), n, h, w, int(gray), int(threshold), int(invert),
                                        float(sigma), ws.data_ptr(), out.data_ptr(), _stream(dev)))
    return out.cpu().numpy()


def _check_pair(gt: np.ndarray, pred: np.ndarray) -> None:
    if gt.shape != pred.shape:
        raise ValueError(f"Shape mismatch: gt{gt.shape} vs pred{pred.shape}")


def compute_metrics_batch(gts: Sequence[np.ndarray], preds: Sequence[np.ndarray], sigma: float = 2.0
                          ) -> List[Dict[str, float]]:
    """compute_metrics for many same-shape pairs in one launch."""
    gts, preds = np.stack([np.asarray(a, bool) for a in gts]), np.stack([np.asarray(a, bool) for a in preds])
    _check_pair(gts, preds)
    if sigma <= 0 and (gts.any() or preds.any()):
        raise ValueError("sigma must be > 0")
    res = _metrics_native(gts, preds, sigma)
    return [dict(zip(METRIC_KEYS, map(float, r))) for r in res]


def compute_metrics(gt: np.ndarray, pred: np.ndarray, sigma: float = 2.0) -> Dict[str, float]:
    """eval_iou_noise.py:239-272."""
    _check_pair(np.asarray(gt), np.asarray(pred))
    return compute_metrics_batch([gt], [pred], sigma)[0]


def gaussian_weighted_recall(gt: np.ndarray, pred: np.ndarray, sigma: float = 2.0) -> float:
    """eval_iou_noise.py:185-208."""
    if int(np.asarray(gt).sum()) == 0:
        return 1.0
    if sigma <= 0:
        raise ValueError("sigma must be > 0")
    return compute_metrics(gt, pred, sigma)["gauss_recall"]


def far_noise_ratio(gt: np.ndarray, pred: np.ndarray, sigma: float = 2.0) -> float:
    """eval_iou_noise.py:211-232."""
    if int(np.asarray(pred).sum()) == 0:
        return 0.0
    if sigma <= 0:
        raise ValueError("sigma must be > 0")
    return compute_metrics(gt, pred, sigma)["far_noise_ratio"]


def mean_std(x: np.ndarray) -> Tuple[float, float]:
    if x.size == 0:
        return float("nan"), float("nan")
    return float(x.mean()), float(x.std(ddof=0))


def quantiles(x: np.ndarray, ps: List[float]) -> Dict[str, float]:
    if x.size == 0:
        return {f"p{int(p)}": float("nan") for p in ps}
    return {f"p{int(p)}": float(v) for p, v in zip(ps, np.percentile(x, ps))}


def overdraw_rate(x: np.ndarray, threshold: float = 1.0) -> float:
    if x.size == 0:
        return float("nan")
    return float((x > threshold).mean())


# ---- the reference's main (eval_iou_noise.py:303-482) as a function ---------------------------
def evaluate(gt_dir, gen_dir, out_dir, threshold: int = 128, invert: bool = False, sigma: float = 2.0,
             max_pairs: int = -1, save_diff: bool = False, workers: int = 8, chunk_pairs: int = 256) -> pd.DataFrame:
    """Pairs p{k}.jpg with pic{k+1}.png, writes the binarised / side-by-side (/ diff) PNGs, the
    per-pair and summary CSVs and config.txt under out_dir/run_<timestamp>, returns the summary.
    Pairs are processed in chunks of ``chunk_pairs`` (bounded host and device memory): decoding
    and PNG writes run on a thread pool, every same-shape group of a chunk is one kernel launch.
    ``distance_backend`` in the summary / config.txt reads ``dmx`` (the reference writes
    ``scipy``): the exact EDT runs in csrc/eval.h and reproduces scipy's float64 distances bit for
    bit, so every metric column is the reference's."""
    gt_dir, gen_dir, out_root = Path(gt_dir), Path(gen_dir), Path(out_dir)
    out_root.mkdir(parents=True, exist_ok=True)
    if not gt_dir.exists():
        raise FileNotFoundError(f"gt_dir not found: {gt_dir}")
    if not gen_dir.exists():
        raise FileNotFoundError(f"gen_dir not found: {gen_dir}")
    run_dir = out_root / ("run_" + datetime.now().strftime("%Y%m%d_%H%M%S"))
    bin_gt_dir, bin_gen_dir, bin_pair_dir = (run_dir / "binarized" / d for d in ("gt", "gen", "pair"))
    for d in (bin_gt_dir, bin_gen_dir, bin_pair_dir):
        d.mkdir(parents=True, exist_ok=True)
    diff_dir = run_dir / "diff"
    if save_diff:
        diff_dir.mkdir(parents=True, exist_ok=True)
    gen_map = dict(list_gen_files(gen_dir))
    pairs, missing = [], 0
    for gt_idx, gt_path in list_gt_files(gt_dir):
        gen_path = gen_map.get(gt_idx + 1)
        if gen_path is None:
            missing += 1
            continue
        pairs.append((gt_idx, gt_path, gen_path))
    if max_pairs is not None and max_pairs > 0:
        pairs = pairs[:max_pairs]
    if not pairs:
        raise RuntimeError("有効な比較ペアが見つかりません。\n正解: p00000.jpg, p00001.jpg...\n"
                           "生成: pic1.png, pic2.png...\n対応: p00000 <-> pic1, p00001 <-> pic2 ...\n")
    rows: List[dict] = []
    with ThreadPoolExecutor(max_workers=workers) as pool:
        # bounded chunks of pairs: host memory holds at most `chunk_pairs` decoded pairs (the
        # reference holds one); each same-shape group of a chunk is one kernel launch
        for c0 in range(0, len(pairs), max(1, int(chunk_pairs))):
            chunk = pairs[c0:c0 + max(1, int(chunk_pairs))]
            grays = list(pool.map(lambda pr: (load_gray(pr[1]), load_gray(pr[2])), chunk))
            masks = [((g < threshold) if invert else (g >= threshold), (q < threshold) if invert else (q >= threshold))
                     for g, q in grays]
            del grays
            metrics: List[Dict[str, float]] = [None] * len(chunk)  # type: ignore
            groups: Dict[tuple, List[int]] = {}
            for i, (g, q) in enumerate(masks):
                _check_pair(g, q)
                groups.setdefault(g.shape, []).append(i)
            for idx in groups.values():
                for i, m in zip(idx, compute_metrics_batch([masks[i][0] for i in idx], [masks[i][1] for i in idx],
                                                           sigma)):
                    metrics[i] = m
            jobs = []
            for (gt_idx, gt_path, gen_path), (gm, pm), m in zip(chunk, masks, metrics):
                gt_bin = bin_gt_dir / f"{gt_path.stem}_bin.png"
                gen_bin = bin_gen_dir / f"{gen_path.stem}_bin.png"
                pair_path = bin_pair_dir / f"pair_gt{gt_idx:05d}_vs_{gen_path.stem}.png"
                jobs.append(pool.submit(lambda a, b: mask_to_pil(a).save(b), gm, gt_bin))
                jobs.append(pool.submit(lambda a, b: mask_to_pil(a).save(b), pm, gen_bin))
                jobs.append(pool.submit(save_side_by_side, gm, pm, pair_path))
                diff_path = None
                if save_diff:
                    diff_path = diff_dir / f"diff_gt{gt_idx:05d}_vs_{gen_path.stem}.png"
                    jobs.append(pool.submit(save_diff_visual, gm, pm, diff_path))
                rows.append({"gt_index": gt_idx, "gt_file": gt_path.name, "gen_file": gen_path.name,
                             "gt_bin": str(gt_bin.relative_to(run_dir)), "gen_bin": str(gen_bin.relative_to(run_dir)),
                             "pair_bin": str(pair_path.relative_to(run_dir)),
                             "diff_bin": str(diff_path.relative_to(run_dir)) if diff_path is not None else "", **m})
            for j in jobs:
                j.result()
    df = pd.DataFrame(rows)
    iou_mean, iou_std = mean_std(df["iou"].to_numpy(dtype=np.float64))
    gt_iou_mean, gt_iou_std = mean_std(df["gt_iou"].to_numpy(dtype=np.float64))
    fnr = df["far_noise_ratio"].to_numpy(dtype=np.float64)
    fnr_mean, fnr_std = mean_std(fnr)
    fnr_q = quantiles(fnr, [50, 90, 95])
    gr = df["gauss_recall"].to_numpy(dtype=np.float64)
    gr_mean, gr_std = mean_std(gr)
    q = quantiles(gr, [50, 90, 95])
    summary = pd.DataFrame([{
        "n_pairs": int(len(df)), "missing_pairs_skipped": int(missing), "threshold": int(threshold),
        "invert": bool(invert), "sigma": float(sigma), "distance_backend": _DT_BACKEND,
        "iou_mean": iou_mean, "iou_std": iou_std, "gt_iou_mean": gt_iou_mean, "gt_iou_std": gt_iou_std,
        "far_noise_ratio_mean": fnr_mean, "far_noise_ratio_std": fnr_std, "far_noise_ratio_median": fnr_q["p50"],
        "far_noise_ratio_p90": fnr_q["p90"], "far_noise_ratio_p95": fnr_q["p95"],
        "gauss_recall_mean": gr_mean, "gauss_recall_std": gr_std, "gauss_recall_median": q["p50"],
        "gauss_recall_p90": q["p90"], "gauss_recall_p95": q["p95"],
        "gauss_overdraw_rate_gt1": overdraw_rate(gr, threshold=1.0), "run_dir": str(run_dir),
    }])
    df.to_csv(run_dir / "metrics_detail.csv", index=False, encoding="utf-8-sig")
    summary.to_csv(run_dir / "metrics_summary.csv", index=False, encoding="utf-8-sig")
    (run_dir / "config.txt").write_text("\n".join([
        f"gt_dir={gt_dir}", f"gen_dir={gen_dir}", f"threshold={threshold}", f"invert={bool(invert)}",
        f"sigma={sigma}", f"distance_backend={_DT_BACKEND}", f"max_pairs={max_pairs}", f"save_diff={bool(save_diff)}",
        f"missing_pairs_skipped={missing}"]) + "\n", encoding="utf-8")
    return summary


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gt_dir", type=str, required=True)
    ap.add_argument("--gen_dir", type=str, required=True)
    ap.add_argument("--out_dir", type=str, required=True)
    ap.add_argument("--threshold", type=int, default=128)
    ap.add_argument("--invert", action="store_true")
    ap.add_argument("--sigma", type=float, default=2.0)
    ap.add_argument("--max_pairs", type=int, default=-1)
    ap.add_argument("--save_diff", action="store_true")
    a = ap.parse_args(argv)
    summary = evaluate(a.gt_dir, a.gen_dir, a.out_dir, a.threshold, a.invert, a.sigma, a.max_pairs, a.save_diff)
    print(summary.to_string(index=False))


if __name__ == "__main__":
    main(sys.argv[1:])
