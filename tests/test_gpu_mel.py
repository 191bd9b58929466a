"""GPU parity of the style front-end: the HIP log-mel (stts_wave_preprocess, mel.hip) and the
chunked style averaging (stts2_mi355x.inference.get_style) against the CPU oracle
(oracle/stts_oracle.py wave_preprocess / get_style, a restatement of torchaudio's MelSpectrogram
as inference.py:43-49 instantiates it).  Parity with the reference itself is unpinned (torchaudio
is absent, and the reference holds no mel fixture); tests/test_mel_oracle.py pins the oracle to
float64 formulas and known answers.

Tolerances: log-mel max-abs 2e-4 (fp32 direct DFT vs torch.stft's FFT; the log compresses the
relative error of loud bins and the 1e-5 floor bounds quiet ones); style fp32 max-abs 1e-4."""
import numpy as np
import pytest
import torch

from helpers import fill_module, speech_like
from oracle import stts_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("L", [1025, 1200, 72000, 72137, 240000])
def test_wave_preprocess_matches_oracle(L):
    from stts2_mi355x.inference import Preprocess
    x = speech_like(f"mel:{L}", L)
    ref = orc.wave_preprocess(x).numpy()
    out = Preprocess().wave_preprocess(x).cpu().numpy()
    assert out.shape == ref.shape == (1, 80, 1 + L // 300)
    err = np.abs(out - ref).max()
    print(f"L={L}: log-mel max-abs {err:.2e}")
    assert err < 2e-4


def test_batch_rows_are_independent():
    from stts2_mi355x.engine import wave_preprocess_batch
    xs = np.stack([speech_like(f"melb:{b}", 30000) for b in range(3)])
    out = wave_preprocess_batch(torch.from_numpy(xs)).cpu().numpy()
    for b in range(3):
        assert np.abs(out[b] - orc.wave_preprocess(xs[b]).numpy()[0]).max() < 2e-4


def test_short_wave_raises():
    from stts2_mi355x.inference import Preprocess
    with pytest.raises(ValueError):
        Preprocess().wave_preprocess(np.zeros(1024, np.float32))  # reflect pad 1024 needs L > 1024


@pytest.mark.parametrize("dur", [2.5, 9.5, 10.5])
def test_get_style_matches_oracle(dur):
    """2.5 s: one chunk; 9.5 s: three 3-s chunks, the 0.5-s tail dropped; 10.5 s: three chunks and
    a 1.5-s tail (inference.py:195-217)."""
    from stts2_mi355x.inference import get_style
    from stts2_mi355x.models import StyleEncoder
    se = fill_module(StyleEncoder(dim_in=64, style_dim=128, max_conv_dim=512)).eval()
    sd = {k: v.detach().clone() for k, v in se.state_dict().items()}
    audio = speech_like(f"style:{dur}", int(24000 * dur))
    with torch.no_grad():
        ref = orc.get_style(audio, sd).numpy()
        out = get_style(se.cuda(), audio).cpu().numpy()
    assert out.shape == ref.shape == (1, 128)
    err = np.abs(out - ref).max()
    print(f"get_style {dur}s: max-abs {err:.2e} (ref absmax {np.abs(ref).max():.3f})")
    assert err < 1e-4
