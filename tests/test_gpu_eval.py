"""eval_iou_noise metrics on the GPU (dmx_eval_metrics) vs the reference's own outputs
(tests/golden/eval_metrics.npz, make_golden_eval.py) and the oracle (oracle/eval_ref.py).

Tolerances: counts and the ratios of counts (iou, gt_iou, far_noise_ratio, inter, union,
gt_area, pred_area, fp) bit-exact — the EDT is exact and the far-noise test compares the
same float64 distances; gauss_recall (a float64 sum of exp() over the predicted pixels, in a
different order and with the device's exp) within 1e-12 relative."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEYS = ("iou", "gt_iou", "far_noise_ratio", "gauss_recall", "inter", "union", "gt_area", "pred_area", "fp")


def _check(got, exp):
    got, exp = np.asarray(got, np.float64), np.asarray(exp, np.float64)
    exact = [i for i, k in enumerate(KEYS) if k != "gauss_recall"]
    assert np.array_equal(got[..., exact], exp[..., exact]), (got, exp)
    gi = KEYS.index("gauss_recall")
    assert np.allclose(got[..., gi], exp[..., gi], rtol=1e-12, atol=0), (got[..., gi], exp[..., gi])


def test_compute_metrics_batch_vs_reference(golden, cuda):
    import eval_iou_noise as ev
    g = golden("eval_metrics.npz")
    res = ev.compute_metrics_batch(list(g["mask_gt"]), list(g["mask_gen"]), sigma=2.0)
    _check([[r[k] for k in KEYS] for r in res], g["metrics"])
    one = ev.compute_metrics(g["ns_gt"], g["ns_gen"], sigma=3.5)
    _check([one[k] for k in KEYS], g["ns_metrics"])
    assert ev.gaussian_weighted_recall(g["mask_gt"][0], g["mask_gen"][0]) == res[0]["gauss_recall"]
    assert ev.far_noise_ratio(g["mask_gt"][0], g["mask_gen"][0]) == res[0]["far_noise_ratio"]


def test_device_binarisation_matches_reference(golden, cuda):
    import eval_iou_noise as ev
    g = golden("eval_metrics.npz")
    got = ev._metrics_native(g["gray_gt"], g["gray_gen"], 2.0, gray=True, threshold=128, invert=True)
    _check(got, g["metrics"])


def test_random_masks_vs_oracle(cuda):
    import eval_iou_noise as ev
    from oracle import eval_ref
    rng = np.random.default_rng(5)
    gts = rng.random((4, 40, 72)) < 0.03
    preds = rng.random((4, 40, 72)) < 0.05
    got = ev.compute_metrics_batch(list(gts), list(preds), sigma=1.5)
    for r, gm, pm in zip(got, gts, preds):
        e = eval_ref.compute_metrics(gm, pm, 1.5)
        _check([r[k] for k in KEYS], [e[k] for k in KEYS])


def test_wide_masks_vs_oracle(cuda):
    """w > 1024: pass 2 reads the row from the workspace instead of LDS (same exact EDT)."""
    import eval_iou_noise as ev
    from oracle import eval_ref
    rng = np.random.default_rng(9)
    gts = rng.random((2, 12, 1500)) < 0.01
    preds = rng.random((2, 12, 1500)) < 0.02
    gts[1] = False  # no GT pixel: scipy's virtual-feature distances
    got = ev.compute_metrics_batch(list(gts), list(preds), sigma=2.0)
    for r, gm, pm in zip(got, gts, preds):
        e = eval_ref.compute_metrics(gm, pm, 2.0)
        _check([r[k] for k in KEYS], [e[k] for k in KEYS])


def test_errors_like_reference(cuda):
    import eval_iou_noise as ev
    a = np.zeros((8, 8), bool)
    a[2, 3] = True
    with pytest.raises(ValueError):
        ev.compute_metrics(a, np.zeros((8, 9), bool))
    with pytest.raises(ValueError):
        ev.gaussian_weighted_recall(a, a, sigma=0.0)
    assert ev.gaussian_weighted_recall(np.zeros_like(a), a) == 1.0
    assert ev.far_noise_ratio(a, np.zeros_like(a)) == 0.0


def test_evaluate_directories_end_to_end(golden, cuda, tmp_path):
    """The reference main()'s pairing (p{k}.jpg <-> pic{k+1}.png), CSVs and images from evaluate()."""
    import pandas as pd
    import eval_iou_noise as ev
    g = golden("eval_metrics.npz")
    gt_dir, gen_dir = tmp_path / "gt", tmp_path / "gen"
    gt_dir.mkdir()
    gen_dir.mkdir()
    o1 = o2 = 0
    for k, (l1, l2) in enumerate(zip(g["gt_lens"], g["gen_lens"])):
        g["gt_files"][o1:o1 + l1].tofile(gt_dir / f"p{k:05d}.jpg")
        g["gen_files"][o2:o2 + l2].tofile(gen_dir / f"pic{k + 1}.png")
        o1 += l1
        o2 += l2
    summary = ev.evaluate(gt_dir, gen_dir, tmp_path / "out", threshold=128, invert=True, sigma=2.0, save_diff=True)
    run_dir = summary["run_dir"][0]
    df = pd.read_csv(os.path.join(run_dir, "metrics_detail.csv"))
    assert np.allclose(df[list(KEYS)].to_numpy(), g["metrics"], rtol=1e-12, atol=0)  # through CSV text
    assert int(summary["n_pairs"][0]) == len(g["gt_lens"])
    assert len(os.listdir(os.path.join(run_dir, "diff"))) == len(g["gt_lens"])
    # bounded chunks (one pair per chunk): the same per-pair rows
    s1 = ev.evaluate(gt_dir, gen_dir, tmp_path / "out1", threshold=128, invert=True, sigma=2.0, chunk_pairs=1)
    d1 = pd.read_csv(os.path.join(s1["run_dir"][0], "metrics_detail.csv"))
    assert d1[list(KEYS)].equals(df[list(KEYS)])
