"""CPU tests of the C-ABI library: it loads, exports every symbol include/*.h declares,
and its model plans name exactly the reference state-dict keys (no GPU compute here)."""
import ctypes
import glob
import os
import re

import pytest
import torch

from helpers import HIFI_CFG, ISTFT_CFG
from stts2_mi355x import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    out = set()
    for h in sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))):
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        out |= set(re.findall(r"\b(stts_[a-z0-9_]+)\s*\(", src))
    return sorted(out)


def test_library_exports_all_declared_symbols():
    L = E.lib()
    syms = declared_symbols()
    assert len(syms) >= 14 + 20  # stts2.h + stts2_train.h
    for s in syms:
        assert hasattr(L, s), f"libstts2.so does not export {s}"


def _plan(kind, cfg):
    L = E.lib()
    arr = (ctypes.c_int * len(cfg))(*cfg)
    h = ctypes.c_void_p()
    rc = L.stts_model_create(kind, arr, len(cfg), ctypes.byref(h))
    return rc, h


def _dec_cfg(module, ist):
    g = module.generator
    cfg = [module.dim_in, module.style_dim, g.upsample_initial_channel, len(g.upsample_rates), *g.upsample_rates,
           *g.upsample_kernel_sizes, len(g.resblock_kernel_sizes), *g.resblock_kernel_sizes,
           *[d for ds in g.resblock_dilation_sizes for d in ds]]
    return cfg + ([g.gen_istft_n_fft, g.gen_istft_hop_size] if ist else [])


@pytest.mark.parametrize("kind", ["hifigan", "istftnet"])
def test_decoder_plan_names_match_state_dict(kind):
    from stts2_mi355x.hifigan import Decoder as H
    from stts2_mi355x.istftnet import Decoder as I
    ist = kind == "istftnet"
    mod = (I if ist else H)(dim_in=512, style_dim=128, dim_out=80, **(ISTFT_CFG if ist else HIFI_CFG))
    rc, h = _plan(1 if ist else 0, _dec_cfg(mod, ist))
    assert rc == 0
    L = E.lib()
    sd = mod.state_dict()
    names = [L.stts_param_name(h, i).decode() for i in range(L.stts_param_count(h))]
    assert sorted(names) == sorted(sd.keys())
    for i, n in enumerate(names):
        assert L.stts_param_numel(h, i) == sd[n].numel(), n
    assert L.stts_packed_bytes(h, 1) > 0 and L.stts_packed_bytes(h, 0) > L.stts_packed_bytes(h, 1)
    ws = L.stts_workspace_bytes(h, 1, 32, 400)
    assert 0 < ws < 8 << 30  # B=32 x 10 s in bf16 fits a few GB of the 288 GB HBM
    # forward without packed weights / params must fail loudly, not compute
    rc = L.stts_decoder_fwd(h, 0, None, None, None, None, None, 0, 0, 1, 4, None, None, 0, None)
    assert rc < 0
    L.stts_model_destroy(h)


def test_f0n_plan_names_match_state_dict():
    from stts2_mi355x.models import ProsodyPredictor
    pp = ProsodyPredictor(style_dim=128, d_hid=512, nlayers=3, max_dur=50, dropout=0.2)
    rc, h = _plan(2, [512, 128])
    assert rc == 0
    L = E.lib()
    sd = pp.state_dict()
    names = [L.stts_param_name(h, i).decode() for i in range(L.stts_param_count(h))]
    assert set(names) <= set(sd.keys())
    assert {n for n in sd if n.startswith(("F0.", "N.", "F0_proj", "N_proj"))} == set(names)
    L.stts_model_destroy(h)


def test_bad_configs_rejected():
    assert _plan(0, [512, 128, 512, 4, 10, 5, 3])[0] < 0       # truncated
    assert _plan(0, [512, 128, 256, 1, 2, 4, 1, 3, 1, 3, 5])[0] < 0  # init channel must be 512
    assert _plan(7, [1])[0] < 0                                 # unknown kind
    assert _plan(2, [511, 128])[0] < 0                          # odd d_hid


def test_error_strings():
    L = E.lib()
    for code in (0, -1, -2, -3, -4, -5):
        assert L.stts_error_string(code)


def test_product_path_refuses_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from helpers import make_decoder
    dec, _ = make_decoder("hifigan")
    with pytest.raises(RuntimeError):
        dec(torch.zeros(1, 512, 4), torch.zeros(1, 8), torch.zeros(1, 8), torch.zeros(1, 128))


def test_style_plan_names_match_state_dict():
    from stts2_mi355x.models import StyleEncoder
    se = StyleEncoder(dim_in=64, style_dim=128, max_conv_dim=512)
    rc, h = _plan(3, [64, 128, 512])
    assert rc == 0
    L = E.lib()
    sd = se.state_dict()
    names = [L.stts_param_name(h, i).decode() for i in range(L.stts_param_count(h))]
    assert sorted(names) == sorted(sd.keys())
    for i, n in enumerate(names):
        assert L.stts_param_numel(h, i) == sd[n].numel(), n
    assert L.stts_workspace_bytes(h, 0, 1, 241) > 0
    assert L.stts_workspace_bytes(h, 0, 1, 48) < 0  # 5x5 valid conv needs T >= 65 (reference raises too)
    L.stts_model_destroy(h)


def test_duration_path_argument_checks():
    """The duration-path entry points validate shapes before touching the device (include/stts2.h)."""
    from stts2_mi355x import prosody
    L = prosody._L()
    assert L.stts_bilstm_workspace_bytes(2, 10, 256) == ((2 * 2 * 10 * 1024 + 2 * 256 * 1024) * 4 + 2 * 2 * 2 * 256 * 8 + 8
                                                          + 16 * 2 * 10 * 1024 * 4)  # split-K scratch (B T <= 256)
    assert L.stts_bilstm_workspace_bytes(32, 400, 256) == (2 * 32 * 400 * 1024 + 2 * 256 * 1024) * 4 + 2 * 32 * 2 * 256 * 8 + 8
    params = (ctypes.c_void_p * 8)(*([1] * 8))
    # H must be a multiple of 32 and <= 256
    assert L.stts_bilstm_fwd(1, 0, 0, 0, 1, 4, 8, None, params, 300, 1, None, None, 1, 1 << 30, None) == -1
    assert L.stts_bilstm_fwd(1, 0, 0, 0, 1, 4, 8, None, params, 24, 1, None, None, 1, 1 << 30, None) == -1
    # workspace too small
    assert L.stts_bilstm_fwd(1, 0, 0, 0, 1, 4, 8, None, params, 32, 1, None, None, 1, 16, None) == -4
    assert L.stts_row_norm(1, 0, 0, 0, 1, 1, 8, 3, 1, 1, 0, 1e-5, 0, 0.0, None, None, 0, 1, 0, 0, None) == -1
    assert L.stts_frames_gemm(1, 0, 0, 0, 1, 1, 1, 1, 0, 0, 0, 0, 1, 0, 0, None, None, 1, 0, 0, 0, 1, None) == -1


def test_duration_modules_keep_reference_keys():
    """TextEncoder / ProsodyPredictor expose the reference's state-dict names (models.py:241-466)."""
    from stts2_mi355x.models import ProsodyPredictor, TextEncoder
    te = TextEncoder(channels=512, kernel_size=5, depth=3, n_symbols=178)
    keys = set(te.state_dict())
    for k in ("embedding.weight", "cnn.2.0.weight_g", "cnn.2.0.weight_v", "cnn.2.0.bias", "cnn.2.1.gamma",
              "cnn.2.1.beta", "lstm.weight_hh_l0_reverse", "lstm.bias_ih_l0"):
        assert k in keys, k
    assert len(keys) == 1 + 3 * 5 + 8
    pp = ProsodyPredictor(style_dim=128, d_hid=512, nlayers=3, max_dur=50, dropout=0.2)
    pk = set(pp.state_dict())
    for k in ("text_encoder.lstms.0.weight_ih_l0", "text_encoder.lstms.5.fc.weight", "lstm.bias_hh_l0_reverse",
              "duration_proj.linear_layer.weight", "shared.weight_hh_l0"):
        assert k in pk, k
    with pytest.raises(RuntimeError):
        te(torch.zeros(1, 4, dtype=torch.long), torch.tensor([4]))


def test_option_defaults_are_the_documented_ones():
    """engine.OPT_DEFAULTS (what tests restore) equals the library's own production defaults."""
    from stts2_mi355x import engine
    engine.reset_options()
    for k, v in engine.OPT_DEFAULTS.items():
        assert engine.get_option(k) == v, (k, engine.get_option(k), v)
    assert engine.lib().stts_get_option(999) < 0


def test_bilstm_error_word_offset():
    """The BiLSTM error word lies inside the workspace, 8-byte aligned, before the exchange words."""
    from stts2_mi355x import prosody
    L = prosody._L()
    for B, T, H in ((1, 5, 256), (4, 37, 256), (32, 400, 256), (3, 7, 64)):
        off = L.stts_bilstm_error_offset(B, T, H)
        assert 0 < off and off % 8 == 0 and off + 8 <= L.stts_bilstm_workspace_bytes(B, T, H)
    assert L.stts_bilstm_error_offset(-1, 1, 1) < 0
