"""CPU-only: the C-ABI library loads and exports every symbol include/dmx.h declares;
the native weight-key contract equals the reference state_dicts; host-side logic of the
drop-in surface (schedule tables, arg normalisation, CSV conditioning) matches the
reference goldens."""
import json
import os
import re

import numpy as np
import pytest
import torch

from conftest import GOLDEN, REPO


def header_symbols():
    src = open(os.path.join(REPO, "include", "dmx.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(dmx_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    from dmx import _lib
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert set(syms) == bound, set(syms) ^ bound
    assert lib.dmx_abi_version() == 1


def test_native_key_contract_matches_reference():
    from dmx import _lib, spec
    ref = json.load(open(os.path.join(GOLDEN, "keys.json")))
    def as_list(keys):
        return [(k, tuple(s)) for k, s in keys]
    assert as_list(ref["unet_cond_geom"]) == _lib.model_keys(_lib.DMX_UNET_COND_GEOM)
    assert as_list(ref["vae"]) == _lib.model_keys(_lib.DMX_VAE)
    assert as_list(ref["unet_in4"]) == _lib.model_keys(_lib.DMX_UNET, in_ch=4)
    assert list(spec.unet_cond_geom_spec().shapes().items()) == _lib.model_keys(_lib.DMX_UNET_COND_GEOM)
    # remove_deep_conv variant and UnetCond (no geom head) agree with dmx.spec
    assert list(spec.unet_cond_spec(remove_deep_conv=True).shapes().items()) == \
        _lib.model_keys(_lib.DMX_UNET_COND, remove_deep_conv=True)
    assert list(spec.unet_spec(in_ch=3).shapes().items()) == _lib.model_keys(_lib.DMX_UNET, in_ch=3)


def test_dropin_modules_state_dict_and_loadmodel(tmp_path, unet_sd):
    from models.unet_cond_geom import UnetCondWithGeomHead
    from models.vae import VAE
    from utils import Utils
    ref = json.load(open(os.path.join(GOLDEN, "keys.json")))
    m = UnetCondWithGeomHead()
    assert [[k, list(v.shape)] for k, v in m.state_dict().items()] == [list(x) for x in ref["unet_cond_geom"]]
    path = tmp_path / "trained_para.pth"
    torch.save(unet_sd, path)
    m2 = Utils.loadModel(str(path), UnetCondWithGeomHead(), device="cpu")
    assert not m2.training
    assert torch.equal(m2.state_dict()["sa6.mha.in_proj_weight"], unet_sd["sa6.mha.in_proj_weight"])
    assert [[k, list(v.shape)] for k, v in VAE().state_dict().items()] == [list(x) for x in ref["vae"]]


def test_no_cpu_fallback(unet_sd):
    """The product path fails loudly off-GPU instead of computing on the host."""
    from dmx import DmxUnavailable
    from models.unet_cond_geom import UnetCondWithGeomHead
    m = UnetCondWithGeomHead().eval()
    x = torch.zeros((1, 4, 32, 32))
    with pytest.raises(DmxUnavailable):
        m(x, torch.ones(1, dtype=torch.long), torch.ones(1, dtype=torch.long))


def test_schedule_tables_bit_exact(golden):
    import diff
    g = golden("schedule.npz")
    d = diff.Diffuser(1000, device="cpu")
    assert np.array_equal(d.betas.numpy(), g["betas"])
    assert np.array_equal(d.alpha_bars.numpy(), g["alpha_bars"])
    c1, c2, sd = d.coef_tables("cpu", True)
    a, ab = torch.from_numpy(g["alphas"]), torch.from_numpy(g["alpha_bars"])
    for tv in (1, 2, 500, 1000):  # the reference's per-step expressions, diff.py:141-144,160-161
        ti = torch.tensor([tv - 1])
        al, abv, abp = a[ti], ab[ti], ab[torch.clamp(ti - 1, min=0)]
        assert torch.equal(c1[ti], (1 - al) / torch.sqrt(1 - abv))
        assert torch.equal(c2[ti], torch.sqrt(al))
        assert torch.equal(sd[ti], torch.sqrt((1 - al) * (1 - abp) / (1 - abv)))
    _, _, sdu = d.coef_tables("cpu", False)
    ti = torch.tensor([0])
    assert torch.equal(sdu[ti], torch.sqrt((1 - a[ti]) * (1 - ab[ti - 1]) / (1 - ab[ti])))


def test_time_table_bit_exact_vs_reference_formula():
    from dmx.engine import pos_table
    from oracle import ref
    t = torch.arange(1, 1001)
    assert torch.equal(pos_table(1000), ref.pos_encoding(t.unsqueeze(-1).float() * 0 + t.unsqueeze(-1)))


def test_sampler_csv_dropin_matches_reference(golden):
    import diff
    from entityCsvSampler import EntityCsvSampler
    import pandas as pd
    g = golden("sampler_csv.npz")
    df = pd.read_csv(os.path.join(GOLDEN, "entities.csv"), header=None)
    s = EntityCsvSampler(diff.Diffuser(10), None, None, class_id=1, device="cpu")
    for cid in (1, 2, 3):
        v, m = s._build_vals_mask_for(df, cid, (400, 400))
        assert np.array_equal(v, g[f"vals_{cid}"]) and np.array_equal(m, g[f"mask_{cid}"])
        v, m = s._build_vals_mask_for(df, cid, (320.0, 280.0))
        assert np.array_equal(v, g[f"vals_{cid}_320x280"])
        assert np.array_equal(np.array(s._infer_base_wh(df, cid)), g[f"infer_wh_{cid}"])
    with pytest.raises(ValueError):
        s._build_vals_mask_for(df, 4, (400, 400))
    vals, mask = s.load_cond(os.path.join(GOLDEN, "entities.csv"), count=2, start=3)
    assert vals.shape == (2, 12) and torch.equal(vals, torch.from_numpy(g["vals_1"][3:5]))
    with pytest.raises(ValueError):
        s.load_cond(os.path.join(GOLDEN, "entities.csv"), count=2, start=7)


def test_sample_latent_cond_argument_normalisation():
    """diff.py:206-312 host logic: class_counts forms, cond dict/list/tensor, masks, errors."""
    import diff
    d = diff.Diffuser(10)
    assert d._norm_counts({1: 2, 3: 0, 2: 1}) == [(1, 2), (2, 1)]
    assert d._norm_counts((3, 4)) == [(3, 4)]
    assert d._norm_counts([(1, 1), (2, 2)]) == [(1, 1), (2, 2)]
    for bad in ({1: 0}, "x", (1, 2, 3)):
        with pytest.raises(ValueError):
            d._norm_counts(bad)
    y = [1, 1, 3]
    v, m = d._build_cond(y, None, None, None, None, "cpu")
    assert v.abs().sum() == 0 and m[0, :4].sum() == 4 and m[2, 7:].sum() == 5 and m.sum() == 13
    v, m = d._build_cond(y, {1: {"x1": 0.5, "zz": 9}, 3: {"ar": 0.25}}, {3: {"ar": 0.0, "theta1": 1.0}},
                         None, None, "cpu")
    assert v[0, 0] == 0.5 and m[0, 0] == 1 and v[2, 9] == 0.25 and m[2, 9] == 0.0 and m[2, 10] == 1.0
    v, m = d._build_cond(y, [{"cx": 0.1}, {}, {"cy": 0.2}], [{"cx": 0.0}, {}, {}], None, None, "cpu")
    assert v[0, 4] == np.float32(0.1) and m[0, 4] == 0 and m[2, 5] == 1
    with pytest.raises(ValueError):
        d._build_cond(y, [{}], None, None, None, "cpu")
    t = torch.tensor([[0.0, 1.0] + [0.0] * 10] * 3)
    v, m = d._build_cond(y, t, None, None, None, "cpu")
    assert torch.equal(m, (t != 0).float())
    with pytest.raises(ValueError):
        d._build_cond(y, torch.zeros(2, 12), None, None, None, "cpu")
    with pytest.raises(ValueError):
        d._build_cond(y, torch.zeros(3, 12), torch.zeros(3, 11), None, None, "cpu")
    with pytest.raises(ValueError):  # z_shape None needs a vae (diff.py:316-317)
        d.sample_latent_cond(None, (1, 1), z_shape=None, vae=None)


def test_latent_shape_inference_matches_encoder_arithmetic():
    from models.vae import latent_hw
    assert latent_hw(224, 224) == (28, 28) and latent_hw(256, 256) == (32, 32) and latent_hw(225, 230) == (28, 28)
