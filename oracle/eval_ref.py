"""CPU restatement of eval_iou_noise.py's metrics (TEST INFRASTRUCTURE — see oracle/__init__.py).

Follows reference eval_iou_noise.py:77-94 (binarisation), 162-182 (distance map: scipy
distance_transform_edt of ~gt — scipy 1.15.3 here, the reference's first backend), 185-208
(Gaussian-weighted recall), 211-232 (far-noise ratio) and 239-272 (compute_metrics).
Pinned by tests/golden/eval_metrics.npz (reference outputs, tests/golden/make_golden_r2.py).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
from scipy.ndimage import distance_transform_edt


def binarize(gray: np.ndarray, threshold: int = 128, invert: bool = True) -> np.ndarray:
    """eval_iou_noise.py:86-94 on an already-decoded uint8 grayscale array."""
    arr = np.asarray(gray, dtype=np.uint8)
    return (arr < threshold) if invert else (arr >= threshold)


def distance_map_to_gt(gt: np.ndarray) -> np.ndarray:
    """eval_iou_noise.py:169-171."""
    return distance_transform_edt(~gt).astype(np.float64)


def gaussian_weighted_recall(gt: np.ndarray, pred: np.ndarray, sigma: float = 2.0) -> float:
    """eval_iou_noise.py:185-208."""
    gt_area = int(gt.sum())
    if gt_area == 0:
        return 1.0
    if sigma <= 0:
        raise ValueError("sigma must be > 0")
    w = np.exp(-(distance_map_to_gt(gt) ** 2) / (2.0 * (sigma ** 2)))
    return float((pred.astype(np.float64) * w).sum(dtype=np.float64) / gt_area)


def far_noise_ratio(gt: np.ndarray, pred: np.ndarray, sigma: float = 2.0) -> float:
    """eval_iou_noise.py:211-232."""
    pred_area = int(pred.sum())
    if pred_area == 0:
        return 0.0
    if sigma <= 0:
        raise ValueError("sigma must be > 0")
    far = distance_map_to_gt(gt) > sigma
    return float(np.logical_and(pred, far).sum(dtype=np.int64) / pred_area)


def compute_metrics(gt: np.ndarray, pred: np.ndarray, sigma: float = 2.0) -> Dict[str, float]:
    """eval_iou_noise.py:239-272."""
    if gt.shape != pred.shape:
        raise ValueError(f"Shape mismatch: gt{gt.shape} vs pred{pred.shape}")
    inter = np.logical_and(gt, pred).sum(dtype=np.int64)
    union = np.logical_or(gt, pred).sum(dtype=np.int64)
    gt_area = gt.sum(dtype=np.int64)
    pred_area = pred.sum(dtype=np.int64)
    return {
        "iou": float(inter / union) if union > 0 else 1.0,
        "gt_iou": float(inter / gt_area) if gt_area > 0 else 1.0,
        "far_noise_ratio": far_noise_ratio(gt, pred, sigma=sigma),
        "gauss_recall": gaussian_weighted_recall(gt, pred, sigma=sigma),
        "inter": float(inter), "union": float(union), "gt_area": float(gt_area), "pred_area": float(pred_area),
        "fp": float(np.logical_and(pred, np.logical_not(gt)).sum(dtype=np.int64)),
    }
