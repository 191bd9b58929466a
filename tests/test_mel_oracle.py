"""CPU checks of the style front-end oracle (oracle/stts_oracle.py mel_spectrogram /
wave_preprocess / melscale_fbanks).  Parity with the reference is UNPINNED upstream: the reference
builds its mel with torchaudio, which is absent here, and holds no mel fixture.  These tests pin
the restatement to independent float64 formulas and to known answers of the reference's own
configuration (sample_rate left at torchaudio's 16000 default while the audio is 24 kHz)."""
import math

import numpy as np
import torch

from helpers import speech_like
from oracle import stts_oracle as orc


def test_filterbank_matches_float64_htk_formula():
    fb = orc.melscale_fbanks().numpy().astype(np.float64)
    freqs = np.linspace(0, 8000, 1025)
    mel = lambda f: 2595 * np.log10(1 + f / 700)  # noqa: E731
    f_pts = 700 * (10 ** (np.linspace(mel(0), mel(8000), 82) / 2595) - 1)
    ref = np.zeros((1025, 80))
    for m in range(80):
        lo, c, hi = f_pts[m], f_pts[m + 1], f_pts[m + 2]
        ref[:, m] = np.clip(np.minimum((freqs - lo) / (c - lo), (hi - freqs) / (hi - c)), 0, None)
    assert fb.shape == (1025, 80)
    assert np.abs(fb - ref).max() < 1e-4
    assert fb.max() <= 1.0 + 1e-6 and (fb.sum(0) > 0).all()


def test_frames_and_shape():
    for L in (1025, 72000, 72137):
        out = orc.wave_preprocess(speech_like(f"orc:{L}", L))
        assert tuple(out.shape) == (1, 80, 1 + L // 300)


def test_tone_lands_in_the_16k_filterbank_band():
    """A 1500 Hz tone at 24 kHz peaks at DFT bin 1500*2048/24000 = 128; the reference's filterbank
    (built for 16 kHz) reads that bin as 128 * 8000/1024 = 1000 Hz, so the loudest mel band is the
    one whose triangle covers 1000 Hz, not 1500 Hz."""
    sr, L = 24000, 24000
    x = (0.5 * np.sin(2 * np.pi * 1500 * np.arange(L) / sr)).astype(np.float32)
    mel = orc.wave_preprocess(x)[0]
    band = int(mel[:, 10:-10].mean(1).argmax())
    fb = orc.melscale_fbanks().numpy()
    assert fb[128, band] > 0.5, (band, fb[128, band])
    assert fb[int(round(1500 * 1024 / 8000)), band] == 0.0


def test_log_floor_and_normalisation():
    """Silence gives log(1e-5) -> (log(1e-5) + 4) / 4 in every bin."""
    out = orc.wave_preprocess(np.zeros(4000, np.float32))
    assert torch.allclose(out, torch.full_like(out, (math.log(1e-5) + 4) / 4))
