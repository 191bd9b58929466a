"""Vocos decoder (Modules/vocos.py) on the CPU: the oracle restatement against
the reference's golden outputs, the drop-in module's state-dict contract against the reference's
(recorded by tests/golden/make_golden_vocos.py), and the native plan's parameter names."""
import ctypes

import numpy as np
import pytest
import torch

from helpers import fill_module, golden, meta
from oracle import stts_oracle as orc
from stts2_mi355x import engine as E
from stts2_mi355x import synth
from stts2_mi355x.vocos import Decoder

CASES = [(1200, 300, 4, 2), (1024, 256, 16, 1), (1200, 300, 40, 1)]


def make_vocos(n_fft=1200, hop=300, num_layers=8):
    return fill_module(Decoder(dim_in=512, style_dim=128, dim_out=80, intermediate_dim=1536, num_layers=num_layers,
                               gen_istft_n_fft=n_fft, gen_istft_hop_size=hop)).eval()


def test_state_dict_matches_reference():
    ref = meta()["vocos_state_dict"]
    sd = make_vocos().state_dict()
    assert sorted(sd) == sorted(ref)
    for k, shp in ref.items():
        assert list(sd[k].shape) == shp, k
    # the ISTFT window buffer is torch.hann_window(n_fft) (periodic), as vocos.py:187
    assert torch.equal(sd["generator.stft.istft.window"], torch.hann_window(1200))


@pytest.mark.parametrize("n_fft,hop,T,B", CASES)
def test_oracle_matches_reference_golden(n_fft, hop, T, B):
    g = golden(f"vocos_n{n_fft}_T{T}_B{B}")
    dec = make_vocos(n_fft, hop)
    asr, f0, n, s = [torch.from_numpy(a) for a in synth.decoder_inputs(B, T, tag="vocos")]
    taps = {}
    with torch.no_grad():
        out = orc.decoder_vocos(asr, f0, n, s, dec.state_dict(), dict(num_layers=8, n_fft=n_fft, hop=hop), taps)
    assert out.shape == (B, 1, 2 * T * hop)
    assert np.abs(out.numpy() - g["out"]).max() < 1e-5
    assert np.abs(taps["frontend"].numpy() - g["tap_frontend"]).max() < 1e-5


def test_plan_names_match_state_dict():
    dec = make_vocos(num_layers=3)
    L = E.lib()
    cfg = [512, 128, 1536, 3, 1200, 300]
    arr = (ctypes.c_int * 6)(*cfg)
    h = ctypes.c_void_p()
    assert L.stts_model_create(E.KIND_VOCOS, arr, 6, ctypes.byref(h)) == 0
    sd = dec.state_dict()
    names = [L.stts_param_name(h, i).decode() for i in range(L.stts_param_count(h))]
    assert sorted(names) == sorted(sd)
    for i, n in enumerate(names):
        assert L.stts_param_numel(h, i) == sd[n].numel(), n
    assert 0 < L.stts_workspace_bytes(h, 1, 32, 400) < 4 << 30
    assert L.stts_decoder_fwd(h, 0, None, None, None, None, None, 0, 0, 1, 4, None, None, 0, None) < 0
    L.stts_model_destroy(h)
    for bad in ([256, 128, 1536, 3, 1200, 300],   # generator dim must be decode.3's 512
                [512, 128, 1536, 3, 1200, 1200],  # hop == n_fft: no 'same' padding
                [512, 128, 1536, 3, 4099, 300]):  # n_fft without a two-factor split <= 64
        arr = (ctypes.c_int * 6)(*bad)
        assert L.stts_model_create(E.KIND_VOCOS, arr, 6, ctypes.byref(h)) < 0


def test_build_models_vocos():
    from stts2_mi355x.inference import build_models
    cfg = {"model_params": {"hidden_dim": 512, "style_dim": 128, "n_mels": 80, "n_layer": 3, "max_dur": 50,
                            "dropout": 0.2, "dim_in": 64,
                            "decoder": {"type": "vocos", "intermediate_dim": 1536, "num_layers": 8,
                                        "gen_istft_n_fft": 1200, "gen_istft_hop_size": 300}},
           "symbol": {"pad": "$", "punctuation": ";:,.!?", "letters": "abc", "letters_ipa": "ɑ", "extend": ""}}
    m = build_models(cfg)
    assert m["decoder"].decoder_type == "vocos"
    assert sorted(m["decoder"].state_dict()) == sorted(meta()["vocos_state_dict"])
