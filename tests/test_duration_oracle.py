"""CPU: the oracle's duration / text path (TextEncoder, DurationEncoder, ProsodyPredictor.forward)
against the reference's own outputs (tests/golden/duration_*.npz, make_golden_duration.py)."""
import numpy as np
import pytest
import torch

from helpers import DURATION_CASES, duration_inputs, golden, make_duration_modules
from oracle import stts_oracle as orc


@pytest.fixture(scope="module")
def sds():
    te, pp = make_duration_modules()
    return te.state_dict(), pp.state_dict()


@pytest.mark.parametrize("T,lengths", DURATION_CASES)
def test_duration_oracle_vs_reference(T, lengths, sds):
    te_sd, pp_sd = sds
    g = golden(f"duration_T{T}_B{len(lengths)}")
    tok, ln, s, aln = duration_inputs(T, lengths)
    assert np.array_equal(g["lengths"], ln)
    s_t, aln_t = torch.from_numpy(s), torch.from_numpy(aln)
    t_en = orc.text_encoder(tok, ln, te_sd)
    assert np.abs(t_en.numpy() - g["t_en"]).max() < 1e-5
    d = orc.duration_encoder(torch.from_numpy(g["t_en"]), s_t, ln, pp_sd, "text_encoder.")
    assert np.abs(d.numpy() - g["d"]).max() < 1e-5
    duration, en = orc.predictor_forward(torch.from_numpy(g["t_en"]), s_t, ln, aln_t, pp_sd)
    assert np.abs(duration.numpy() - g["duration"]).max() < 1e-5
    assert np.abs(en.numpy() - g["en"]).max() < 1e-5
    x = orc.bilstm(torch.from_numpy(g["d"]), pp_sd, "lstm.")  # inference.py:246, unpacked
    dur_inf = torch.sigmoid(torch.nn.functional.linear(x, pp_sd["duration_proj.linear_layer.weight"],
                                                       pp_sd["duration_proj.linear_layer.bias"])).sum(-1)
    assert np.abs(dur_inf.numpy() - g["dur_inference"]).max() < 1e-4
    assert np.abs((torch.from_numpy(g["t_en"]) @ aln_t).numpy() - g["asr"]).max() < 1e-5


def test_padding_rows_are_zero():
    g = golden("duration_T24_B3")
    for b, n in enumerate(g["lengths"]):
        assert np.all(g["t_en"][b, :, n:] == 0) and np.all(g["d"][b, n:] == 0)


def test_oracle_durations_known_answers():
    """inference.py:134-148, 247-258 restated; known answers (inference.py cannot be imported here: it
    downloads nltk data at import, SURVEY §8(c), so this step is pinned by hand-computed cases)."""
    x = torch.tensor([[1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 40.0, 1.0]])
    out = orc.replace_outliers_zscore(x)
    mean, std = x.mean(), x.std()
    assert abs(float(out[0, 12]) - float(mean + 3 * std * 0.95)) < 1e-5
    assert torch.equal(out[0, :12], x[0, :12])
    # logits of +-inf-like magnitude: sigmoid sums are exact integers
    logits = torch.full((1, 6, 50), -30.0)
    logits[0, :, :3] = 30.0  # 3 frames per token
    dur, pred = orc.durations(logits, torch.zeros(1, 6), mix=0.0, speed=1.0)
    assert torch.equal(pred, torch.full((6,), 3.0))
    dur, pred = orc.durations(logits, torch.zeros(1, 6), mix=0.0, speed=2.0)  # 1.5 rounds half to even
    assert torch.equal(pred, torch.full((6,), 2.0))
    dur, pred = orc.durations(torch.full((1, 6, 50), -30.0), torch.zeros(1, 6), mix=0.0)
    assert torch.equal(pred, torch.ones(6))  # clamp(min=1)
    aln = orc.alignment_matrix(torch.tensor([2.0, 1.0, 3.0]))
    assert aln.shape == (1, 3, 6) and aln.sum() == 6 and aln[0, 2, 3:].sum() == 3
