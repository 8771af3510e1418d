"""Drop-in ``entityCsvSampler`` (reference entityCsvSampler.py:9-199).

Host-side conditioning only: a headerless 13-column entity CSV becomes (B,12)
``cond_vals`` / ``cond_mask`` (drawing -> unit coordinates, Y flipped, radius
/ W, angles in degrees -> /360) and ``Diffuser.sample_latent_cond`` does the
device work.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np
import pandas as pd
import torch

from diff import Diffuser

# entity columns of the CSV per class: (key, column, normaliser)
_LAYOUT = {
    1: (("x1", 1, "x"), ("y1", 2, "y"), ("x2", 3, "x"), ("y2", 4, "y")),
    2: (("cx", 5, "x"), ("cy", 6, "y"), ("cr", 7, "r")),
    3: (("ax", 8, "x"), ("ay", 9, "y"), ("ar", 10, "r"), ("theta1", 11, "a"), ("theta2", 12, "a")),
}
# columns used to infer the drawing size per class (entityCsvSampler.py:174-190)
_WH_COLS = {1: ([1, 3], [2, 4]), 2: ([5], [6]), 3: ([8], [9])}


class EntityCsvSampler:
    KEY_ORDER = ["x1", "y1", "x2", "y2", "cx", "cy", "cr", "ax", "ay", "ar", "theta1", "theta2"]
    IDX: Dict[str, int] = {k: i for i, k in enumerate(KEY_ORDER)}

    def __init__(self, diffuser: Diffuser, model, vae, class_id: int = 1,
                 base_wh: Optional[Tuple[float, float]] = (400, 400), device: Optional[torch.device] = None):
        self.diffuser = diffuser
        self.model = model
        self.vae = vae
        self.class_id = int(class_id)
        self.base_wh = base_wh
        self.device = device or getattr(diffuser, "device",
                                        torch.device("cuda" if torch.cuda.is_available() else "cpu"))

    def set_class_id(self, class_id: int) -> None:
        self.class_id = int(class_id)

    def _rows(self, csv_path: str, count: Optional[int], start: int):
        df = pd.read_csv(csv_path, header=None)
        vals, mask = self._build_vals_mask_for(df, self.class_id, self.base_wh)
        end = len(vals) if count is None else min(start + count, len(vals))
        if start >= end:
            raise ValueError("選択範囲にデータがありません。（start/countを確認）")
        return (torch.from_numpy(vals[start:end]).float().to(self.device),
                torch.from_numpy(mask[start:end]).float().to(self.device))

    def sample(self, csv_path: str, count: Optional[int] = None, start: int = 0, guidance_scale: float = 3.0):
        """entityCsvSampler.py:50-80."""
        vals, mask = self._rows(csv_path, count, start)
        return self.diffuser.sample_latent_cond(model=self.model, class_counts=(self.class_id, vals.shape[0]),
                                                vae=self.vae, guidance_scale=guidance_scale, cond=vals,
                                                cond_mask=mask)

    def load_cond(self, csv_path: str, count: Optional[int] = None, start: int = 0):
        """entityCsvSampler.py:82-98."""
        return self._rows(csv_path, count, start)

    def _build_vals_mask_for(self, df: pd.DataFrame, class_id: int, base_wh):
        """entityCsvSampler.py:101-163."""
        W, H = base_wh if base_wh is not None else self._infer_base_wh(df, class_id)
        if class_id not in _LAYOUT:
            raise ValueError("class_id must be 1(line), 2(circle), or 3(arc).")
        n, k = len(df), len(self.KEY_ORDER)
        vals = np.zeros((n, k), dtype=np.float32)
        mask = np.zeros((n, k), dtype=np.float32)
        for key, col, how in _LAYOUT[class_id]:
            v = df[col].to_numpy(dtype=np.float32).astype(np.float32)
            if how == "x" or how == "r":
                v = v / np.float32(W)
            elif how == "y":
                v = 1.0 - (v / np.float32(H))
            else:
                v = self._norm_angle_vec(v)
            vals[:, self.IDX[key]] = v
            mask[:, self.IDX[key]] = 1.0
        return vals, mask

    @staticmethod
    def _snap(v: float, choices=(224, 256, 280, 300, 320, 384, 400, 448), tol=1.5) -> float:
        for c in choices:
            if abs(v - c) <= tol:
                return float(c)
        return float(v)

    def _infer_base_wh(self, df: pd.DataFrame, class_id: int) -> Tuple[float, float]:
        if class_id not in _WH_COLS:
            raise ValueError("class_id must be 1(line), 2(circle), or 3(arc).")
        xc, yc = _WH_COLS[class_id]
        x_max = float(np.max(np.abs(df[xc].to_numpy())))
        y_max = float(np.max(np.abs(df[yc].to_numpy())))
        return self._snap(x_max), self._snap(y_max)

    @staticmethod
    def _norm_angle_vec(v: np.ndarray) -> np.ndarray:
        out = v.astype(np.float32).copy()
        deg = np.abs(out) > 1.0
        out[deg] = (out[deg] % 360.0) / 360.0
        return out
