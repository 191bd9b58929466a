"""GPU parity: the duration / text path through the HIP kernels (csrc/prosody.hip) vs the reference's
golden outputs and the oracle.  fp32 throughout; tolerance 1e-4 max-abs on every output."""
import numpy as np
import pytest
import torch

from helpers import DURATION_CASES, duration_inputs, golden, make_duration_modules
from oracle import stts_oracle as orc
from stts2_mi355x import synth
from stts2_mi355x.prosody import LSTM, matmul

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope="module")
def mods():
    te, pp = make_duration_modules()
    return te.cuda(), pp.cuda()


def _err(a, b):
    return float(np.abs(a.detach().cpu().numpy() - b).max())


@pytest.mark.parametrize("T,lengths", DURATION_CASES)
def test_text_encoder(T, lengths, mods):
    te, pp = mods
    g = golden(f"duration_T{T}_B{len(lengths)}")
    tok, ln, s, aln = duration_inputs(T, lengths)
    m = orc.length_to_mask(ln, T)
    t_en = te(torch.from_numpy(tok).cuda(), torch.from_numpy(ln).cuda(), m.cuda())
    assert tuple(t_en.shape) == g["t_en"].shape
    assert _err(t_en, g["t_en"]) < TOL


@pytest.mark.parametrize("T,lengths", DURATION_CASES)
def test_duration_encoder_and_predictor(T, lengths, mods):
    te, pp = mods
    g = golden(f"duration_T{T}_B{len(lengths)}")
    tok, ln, s, aln = duration_inputs(T, lengths)
    t_en = torch.from_numpy(g["t_en"]).cuda()
    s_t, ln_t, aln_t = torch.from_numpy(s).cuda(), torch.from_numpy(ln).cuda(), torch.from_numpy(aln).cuda()
    d = pp.text_encoder(t_en, s_t, ln_t)
    assert _err(d, g["d"]) < TOL
    duration, en = pp(t_en, s_t, ln_t, aln_t)
    assert _err(duration, g["duration"]) < TOL
    assert _err(en, g["en"]) < TOL
    x, _ = pp.lstm(torch.from_numpy(g["d"]).cuda())  # inference.py:246 (no packing)
    lin = pp.duration_proj.linear_layer
    from stts2_mi355x.prosody import linear_frames
    dur_inf = torch.sigmoid(linear_frames(x, lin.weight, lin.bias)).sum(-1)
    assert _err(dur_inf, g["dur_inference"]) < 1e-3
    assert _err(matmul(t_en, aln_t), g["asr"]) < TOL


def test_shared_lstm_vs_reference_tap():
    from helpers import fill_module
    from stts2_mi355x.models import ProsodyPredictor
    pp = fill_module(ProsodyPredictor(style_dim=128, d_hid=512, nlayers=3, max_dur=50, dropout=0.2)).eval().cuda()
    T, B = 40, 1  # the f0n fixtures use unprefixed formula weights
    g = golden(f"f0n_T{T}_B{B}")
    en = torch.from_numpy(np.stack([synth.normal(f"f0n:en:{b}:{T}", (640, T)) for b in range(B)])).cuda()
    h, _ = pp.shared(en.transpose(-1, -2))
    assert _err(h.transpose(1, 2), g["tap_lstm"]) < TOL


@pytest.mark.parametrize("H,Cin,T,lengths", [(16, 8, 5, (5, 1, 3)), (64, 40, 33, (33, 17)), (256, 640, 130, None),
                                             (128, 96, 7, (0, 7))])
def test_lstm_vs_torch(H, Cin, T, lengths):
    torch.manual_seed(H + T)
    lstm = LSTM(Cin, H, 1, batch_first=True, bidirectional=True)
    B = 2 if lengths is None else len(lengths)
    x = torch.randn(B, T, Cin)
    ref = torch.nn.LSTM(Cin, H, 1, batch_first=True, bidirectional=True)
    ref.load_state_dict(lstm.state_dict())
    with torch.no_grad():
        if lengths is None:
            want, (hn, cn) = ref(x)
        else:
            ln = torch.tensor(lengths)
            if min(lengths) == 0:  # torch refuses empty sequences in a pack: compare the non-empty rows
                want = torch.zeros(B, T, 2 * H)
                keep = ln > 0
                pk = torch.nn.utils.rnn.pack_padded_sequence(x[keep], ln[keep], batch_first=True,
                                                             enforce_sorted=False)
                y, _ = ref(pk)
                y, _ = torch.nn.utils.rnn.pad_packed_sequence(y, batch_first=True, total_length=T)
                want[keep] = y
            else:
                pk = torch.nn.utils.rnn.pack_padded_sequence(x, ln, batch_first=True, enforce_sorted=False)
                y, (hn, cn) = ref(pk)
                want, _ = torch.nn.utils.rnn.pad_packed_sequence(y, batch_first=True, total_length=T)
    lstm = lstm.cuda()
    got, (ghn, gcn) = lstm(x.cuda(), lengths=None if lengths is None else torch.tensor(lengths))
    assert _err(got, want.numpy()) < TOL
    if lengths is None or min(lengths) > 0:
        assert _err(ghn, hn.numpy()) < TOL and _err(gcn, cn.numpy()) < TOL


def test_lstm_strided_input_and_packed_sequence():
    torch.manual_seed(3)
    lstm = LSTM(24, 32, 1, batch_first=True, bidirectional=True)
    ref = torch.nn.LSTM(24, 32, 1, batch_first=True, bidirectional=True)
    ref.load_state_dict(lstm.state_dict())
    x_cm = torch.randn(2, 24, 11)  # channel-major; the LSTM reads the transposed view
    with torch.no_grad():
        want, _ = ref(x_cm.transpose(1, 2))
    lstm = lstm.cuda()
    got, _ = lstm(x_cm.cuda().transpose(1, 2))
    assert _err(got, want.numpy()) < TOL
    ln = torch.tensor([11, 6])
    pk = torch.nn.utils.rnn.pack_padded_sequence(x_cm.transpose(1, 2), ln, batch_first=True, enforce_sorted=False)
    with torch.no_grad():
        wy, _ = ref(pk)
    wy, _ = torch.nn.utils.rnn.pad_packed_sequence(wy, batch_first=True)
    gpk = torch.nn.utils.rnn.pack_padded_sequence(x_cm.cuda().transpose(1, 2), ln, batch_first=True,
                                                  enforce_sorted=False)
    gy, _ = lstm(gpk)
    gy, _ = torch.nn.utils.rnn.pad_packed_sequence(gy, batch_first=True)
    assert _err(gy, wy.numpy()) < TOL


def test_matmul_and_conv_shapes():
    torch.manual_seed(5)
    a, b = torch.randn(3, 70, 33), torch.randn(3, 33, 129)
    got = matmul(a.cuda(), b.cuda())
    assert _err(got, (a @ b).numpy()) < 1e-4
    got = matmul(a.transpose(1, 2).contiguous().cuda().transpose(1, 2), b.cuda())  # strided operand
    assert _err(got, (a @ b).numpy()) < 1e-4


def test_bad_token_raises(mods):
    te, _ = mods
    tok = torch.tensor([[1, 2, 500]]).cuda()
    with pytest.raises(IndexError):
        te(tok, torch.tensor([3]).cuda())


def test_cpu_tensors_refused(mods):
    _, pp = mods
    with pytest.raises(RuntimeError):
        pp.lstm.cpu()(torch.randn(1, 4, 640))
    pp.lstm.cuda()
