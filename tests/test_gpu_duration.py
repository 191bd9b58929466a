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


@pytest.fixture(autouse=True)
def _inference():
    """These modules' HIP paths are forward-only (engine.forward_only): run as inference.py does."""
    with torch.no_grad():
        yield
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


@pytest.mark.parametrize("H,Cin,T,lengths", [(32, 8, 5, (5, 1, 3)), (64, 40, 33, (33, 17)), (256, 640, 130, None),
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


@pytest.mark.parametrize("B,T,Cin,N,K", [(1, 16, 512, 512, 5), (2, 7, 640, 50, 1), (1, 3, 300, 70, 3)])
def test_frames_gemm_split_k(B, T, Cin, N, K):
    """Few-tile launches split K (deterministic fixed-order reduction): conv1d vs torch, and the
    result does not depend on the workspace size (fewer splits)."""
    from stts2_mi355x import prosody as P
    torch.manual_seed(B * T + N)
    x, w, bias = torch.randn(B, T, Cin), torch.randn(N, Cin, K) * 0.05, torch.randn(N)
    want = torch.nn.functional.conv1d(x.transpose(1, 2), w, bias, padding=(K - 1) // 2).transpose(1, 2)
    xd, wd, bd = x.cuda(), w.cuda(), bias.cuda()
    outs = []
    for elems in (16 * B * T * N, 2 * B * T * N, 0):
        y = torch.empty(B, T, N, device="cuda")
        ws = torch.empty(max(elems, 1), device="cuda")
        P.check(P._L().stts_frames_gemm_ws(P._ptr(xd), *xd.stride(), B, T, Cin, P._ptr(wd), 0, wd.stride(0),
                                           wd.stride(1), wd.stride(2), N, K, (K - 1) // 2, P._ptr(bd), None,
                                           P._ptr(y), *y.stride(), T, P._ptr(ws) if elems else None, elems * 4,
                                           P._stream()))
        outs.append(y.cpu())
    for o in outs:
        assert _err(o, want.numpy()) < 1e-4


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
        te(tok, torch.tensor([3]).cuda())  # device tokens: the kernel's range flag
    with pytest.raises(IndexError):
        te(tok.cpu(), torch.tensor([3]))  # host tokens: checked before the upload
    te(torch.tensor([[1, 2, 177]]), torch.tensor([3]))


def test_text_encoder_fold_cache_follows_weights(mods):
    """The cached weight-norm fold is recomputed after load_state_dict (parameter versions change)."""
    te, _ = mods
    tok = torch.tensor([[3, 4, 5, 6]])
    a = te(tok, None).clone()
    sd = {k: v.clone() for k, v in te.state_dict().items()}
    g = sd["cnn.0.0.weight_g"]
    te.load_state_dict({**sd, "cnn.0.0.weight_g": g * 1.5})
    b = te(tok, None).clone()
    te.load_state_dict(sd)
    c = te(tok, None)
    assert (a - b).abs().max().item() > 1e-3 and torch.equal(a, c)


def test_cpu_tensors_refused(mods):
    _, pp = mods
    with pytest.raises(RuntimeError):
        pp.lstm.cpu()(torch.randn(1, 4, 640))
    pp.lstm.cuda()


@pytest.mark.parametrize("mix,prev,speed", [(0.0, 0.0, 1.0), (0.1, 0.0, 1.0), (0.3, 2.5, 0.8), (0.1, 0.0, 1.7)])
def test_durations_vs_oracle(mix, prev, speed):
    from stts2_mi355x.prosody import durations
    torch.manual_seed(int(mix * 100 + speed * 10))
    T = 57
    logits = torch.randn(1, T, 50) * 2.0
    logits[0, 20] += 25.0  # a long token -> exercises the z-score outlier clamp
    z = torch.randn(1, T)
    want_dur, want_pred = orc.durations(logits.clone(), z, mix, prev, speed)
    dur, pred, total, dmean = durations(logits.cuda(), None, z.cuda(), mix, prev, speed)
    assert _err(dur, want_dur.numpy()) < 1e-4
    assert torch.equal(pred.cpu().reshape(-1).float(), want_pred)
    assert int(total[0]) == int(want_pred.sum())
    assert abs(float(dmean[0]) - float(want_dur.mean())) < 1e-4


def test_expand_frames_is_the_alignment_product():
    from stts2_mi355x.prosody import expand_frames
    torch.manual_seed(9)
    pred = torch.tensor([[2, 1, 4, 1, 3], [1, 1, 2, 0, 0]], dtype=torch.int32)
    F = 11
    src = torch.randn(2, 5, 7)  # (b, t, c)
    aln = torch.zeros(2, 5, F)
    for b in range(2):
        c = 0
        for t in range(5):
            aln[b, t, c:c + int(pred[b, t])] = 1
            c += int(pred[b, t])
    want = src.transpose(1, 2) @ aln
    got = expand_frames(src.cuda(), pred.cuda(), F)
    assert torch.equal(got.cpu(), want)
    got = expand_frames(src.transpose(1, 2).contiguous().cuda().transpose(1, 2), pred.cuda(), F)  # strided
    assert torch.equal(got.cpu(), want)


def test_synthesizer_chain_vs_oracle(mods):
    """inference.py:225-272 from the token ids to the waveform: HIP chain vs the oracle chain, fp32."""
    from helpers import make_decoder
    from stts2_mi355x.inference import Synthesizer
    te, pp = mods
    dec, cfg = make_decoder("hifigan")
    tokens = [int(v) for v in (synth.hash_u01("chain:tok", 22) * 177 + 1)]
    s = torch.from_numpy(synth.normal("chain:s", (1, 128)))
    z = torch.from_numpy(synth.normal("chain:z", (1, len(tokens) + 2)))
    noise_fn = lambda F: torch.from_numpy(synth.source_noise(1, 600 * F, tag="chain"))  # noqa: E731
    cpu = lambda m: {k: v.cpu() for k, v in m.state_dict().items()}  # noqa: E731
    want, want_mean, want_pred = orc.inference_chain(tokens, s, cpu(te), cpu(pp),
                                                     {k: v.cpu() for k, v in dec.state_dict().items()}, cfg, z,
                                                     noise_fn, mix=0.1)
    syn = Synthesizer(te, pp, dec.cuda())
    a = syn.alignment(tokens, s.cuda(), t=0.1, z=z.cuda())
    assert torch.equal(a["pred"].cpu().reshape(-1).float(), want_pred)
    F = a["frames"]
    out, dmean = syn.inference(tokens, s.cuda(), t=0.1, z=z.cuda(), noise=noise_fn(F).cuda())
    assert out.shape[-1] == 600 * F == want.shape[-1]
    assert _err(out, want.numpy()) < 1e-3  # north-star waveform tolerance
    assert abs(float(dmean) - float(want_mean)) < 1e-4


def test_lstm_groupings_bit_identical():
    """The recurrence's utterances-per-workgroup choice (1 / 2 / 4) changes no bit of the output."""
    from stts2_mi355x.prosody import set_lstm_group
    torch.manual_seed(11)
    lstm = LSTM(64, 256, 1, batch_first=True, bidirectional=True).cuda()
    x = torch.randn(7, 29, 64).cuda()
    ln = torch.tensor([29, 3, 17, 29, 1, 8, 22])
    outs = []
    try:
        for bg in (1, 2, 4):
            set_lstm_group(bg)
            outs.append(lstm(x, lengths=ln)[0])
    finally:
        set_lstm_group(0)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    ref = torch.nn.LSTM(64, 256, 1, batch_first=True, bidirectional=True)
    ref.load_state_dict({k: v.cpu() for k, v in lstm.state_dict().items()})
    with torch.no_grad():
        y, _ = ref(torch.nn.utils.rnn.pack_padded_sequence(x.cpu(), ln, batch_first=True, enforce_sorted=False))
    y, _ = torch.nn.utils.rnn.pad_packed_sequence(y, batch_first=True, total_length=29)
    assert _err(outs[2], y.numpy()) < TOL


def test_lstm_cooperative_many_utterances():
    """H = 256 runs the cooperative recurrence (W_hh split over 8 workgroups, persistent over the
    utterances): ragged batch larger than the co-resident group count, zero-length rows included."""
    from stts2_mi355x.prosody import set_lstm_group
    torch.manual_seed(12)
    lstm = LSTM(40, 256, 1, batch_first=True, bidirectional=True)
    ref = torch.nn.LSTM(40, 256, 1, batch_first=True, bidirectional=True)
    ref.load_state_dict(lstm.state_dict())
    lstm = lstm.cuda()
    B, T = 40, 23
    ln = torch.randint(1, T + 1, (B,))
    ln[5], ln[0] = 0, T
    x = torch.randn(B, T, 40)
    set_lstm_group(-1)
    try:
        got, (hn, cn) = lstm(x.cuda(), lengths=ln)
    finally:
        set_lstm_group(0)
    keep = ln > 0
    with torch.no_grad():
        y, (rh, rc) = ref(torch.nn.utils.rnn.pack_padded_sequence(x[keep], ln[keep], batch_first=True,
                                                                   enforce_sorted=False))
    y, _ = torch.nn.utils.rnn.pad_packed_sequence(y, batch_first=True, total_length=T)
    want = torch.zeros(B, T, 512)
    want[keep] = y
    assert _err(got, want.numpy()) < TOL
    assert _err(hn[:, keep], rh.numpy()) < TOL and _err(cn[:, keep], rc.numpy()) < TOL
    set_lstm_group(1)
    try:
        alt, _ = lstm(x.cuda(), lengths=ln)
    finally:
        set_lstm_group(0)
    assert _err(got, alt.cpu().numpy()) < 1e-5


def test_generate_vs_oracle(mods):
    """StyleTTS2.generate (inference.py:303-319) on the drop-ins: three sentences with prev_d_mean
    chained from one to the next, each trimmed by 4000 samples at both ends, concatenated and padded,
    against the oracle's restatement of the same loop (fp32, waveform tolerance 1e-3)."""
    from helpers import make_decoder
    from stts2_mi355x.inference import Synthesizer
    te, pp = mods
    dec, cfg = make_decoder("hifigan")
    sents = [[int(v) for v in (synth.hash_u01(f"gen:tok:{i}", n) * 177 + 1)] for i, n in enumerate((18, 9, 26))]
    s = torch.from_numpy(synth.normal("gen:s", (1, 128)))
    zs = [torch.from_numpy(synth.normal(f"gen:z:{i}", (1, len(t) + 2))) for i, t in enumerate(sents)]
    nfs = [(lambda F, i=i: torch.from_numpy(synth.source_noise(1, 600 * F, tag=f"gen{i}"))) for i in range(3)]
    cpu = lambda m: {k: v.cpu() for k, v in m.state_dict().items()}  # noqa: E731
    want = orc.generate(sents, s, cpu(te), cpu(pp), cpu(dec), cfg, zs, nfs, stabilize=True)
    syn = Synthesizer(te, pp, dec.cuda())
    got = syn.generate(sents, {"style": s.cuda(), "speed": 1}, stabilize=True, z=[z.cuda() for z in zs],
                       noise=[(lambda F, f=f: f(F).cuda()) for f in nfs])
    assert got.shape == want.shape
    assert np.all(got[:4000] == 0) and np.all(got[-4000:] == 0)
    err = float(np.abs(got - want).max())
    print(f"generate: {len(sents)} sentences, {got.shape[0]} samples, max-abs vs oracle {err:.3e}")
    assert err < 1e-3


def test_generate_text_path_and_rng(mods):
    """generate(text) splits and merges sentences as Preprocess.text_preprocess does, tokenizes each,
    and draws its noise from torch's generator: reproducible under torch.manual_seed."""
    from helpers import make_decoder
    from stts2_mi355x.inference import Synthesizer, TextCleaner
    te, pp = mods
    dec, _ = make_decoder("hifigan")
    table = {ch: i + 1 for i, ch in enumerate("abcdefghijklmnopqrstuvwxyz ,.")}
    syn = Synthesizer(te, pp, dec.cuda(), tokenize=TextCleaner(table))
    text = "one two three four. five six seven eight nine ten eleven twelve thirteen; fourteen"
    style = {"style": torch.from_numpy(synth.normal("gen:s2", (1, 128))).cuda(), "speed": 1.0}
    torch.manual_seed(5)
    a = syn.generate(text, style, n_merge=4)
    torch.manual_seed(5)
    b = syn.generate(text, style, n_merge=4)
    assert np.array_equal(a, b) and a.shape[0] > 8000 and np.isfinite(a).all()


def test_lstm_cooperative_timeout_raises():
    """A peer workgroup that never publishes its h (debug hook) makes every wait of the cooperative
    recurrence time out: the kernel terminates, poisons y / h_n / c_n with NaN from that step on, and
    the host raises at its next check instead of returning NaN audio silently."""
    from stts2_mi355x import prosody
    torch.manual_seed(13)
    lstm = LSTM(40, 256, 1, batch_first=True, bidirectional=True).cuda()
    x = torch.randn(1, 6, 40).cuda()
    prosody.check_pending()
    prosody.set_lstm_group(-1)
    prosody.set_bilstm_debug(spin_limit=4000, drop=True)
    y, (hn, cn) = lstm(x)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="timed out"):
        prosody.check_pending()
    # step 0 of each direction (t = 0 forward, t = T-1 reverse) ran before the failed wait
    assert torch.isnan(y[:, 1:, :256]).all() and torch.isnan(y[:, :-1, 256:]).all()
    assert torch.isnan(hn).all() and torch.isnan(cn).all()
    prosody.set_bilstm_debug(0, False)
    y2, _ = lstm(x)  # healthy again, and the check passes
    prosody.check_pending()
    assert torch.isfinite(y2).all()


def test_generate_vs_reference_fixture():
    """StyleTTS2.generate on the drop-ins against the REFERENCE's own generate() output
    (tests/golden/generate_ref.npz: same weights, token ids, dur_stats draws and SineGen noise), fp32,
    north-star waveform tolerance 1e-3."""
    from stts2_mi355x.inference import Synthesizer
    from test_generate_ref_cpu import case, modules
    g, sents, zs, nfs = case()
    te, pp, dec = modules(int(g["n_symbols"]))
    syn = Synthesizer(te.cuda(), pp.cuda(), dec.cuda())
    got = syn.generate(sents, {"style": torch.from_numpy(g["s"]).cuda(), "speed": 1}, stabilize=True,
                       z=[z.cuda() for z in zs], noise=[(lambda F, f=f: f(F).cuda()) for f in nfs])
    assert got.shape == g["wav"].shape
    err = float(np.abs(got - g["wav"]).max())
    print(f"generate vs reference fixture: {got.shape[0]} samples, max-abs {err:.3e}")
    assert err < 1e-3
