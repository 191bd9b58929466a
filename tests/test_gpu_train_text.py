"""GPU parity of the text / duration path under train.py's G step (train.py:217, 220-223, 230-233, 286-299, 318,
323, 327) through the C-ABI: the drop-in TextEncoder / ProsodyPredictor.forward (DurationEncoder, packed BiLSTMs,
AdaLayerNorm, duration_proj, en = d^T @ aln) and the duration losses, against the REFERENCE modules' own autograd
(tests/golden/train_text_T24_B3.npz from tests/golden/make_golden_train_text.py: fp64 = the truth, fp32 = the
reference as it runs), in eval mode (dropout off) and in train mode as train.py runs the modules (dropout on, with the
same injected keep masks on both sides: train_text_drop_T24_B3.npz, training.set_dropout_masks), on a ragged batch
(lengths 24 / 19 / 13); and each new backward kernel separately against torch's fp64 autograd on the CPU.

Bound: every parameter / input gradient per tensor within max(2 x the fp32 reference's own error
vs fp64, 1e-4 of the tensor's scale), and within 1e-4 of the module's largest |g| (normwise)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import DURATION_CASES, duration_inputs, golden, make_duration_modules
from stts2_mi355x import synth
from test_gpu_train_pred import _check_fixture, _rel

pytestmark = pytest.mark.gpu


def _dur_losses_ref(d, d_gt, input_lengths):
    """train.py:286-299 (the test's CPU checker)."""
    loss_ce = 0
    loss_dur = 0
    for _s2s_pred, _text_input, _text_length in zip(d, d_gt, input_lengths):
        _s2s_pred = _s2s_pred[:_text_length, :]
        _text_input = _text_input[:_text_length].long()
        _s2s_trg = torch.zeros_like(_s2s_pred)
        for p in range(_s2s_trg.shape[0]):
            _s2s_trg[p, :_text_input[p]] = 1
        _dur_pred = torch.sigmoid(_s2s_pred).sum(axis=1)
        loss_dur += F.l1_loss(_dur_pred[1:_text_length - 1], _text_input[1:_text_length - 1])
        loss_ce += F.binary_cross_entropy_with_logits(_s2s_pred.flatten(), _s2s_trg.flatten())
    return loss_dur / d.size(0), loss_ce / d.size(0)


@pytest.mark.parametrize("mode", ["eval", "train"])
def test_text_chain_grads_vs_reference(mode):
    """t_en = text_encoder(tokens); asr = t_en @ attn; d, p = predictor(t_en, s, lengths, attn); the probe losses +
    loss_dur + loss_ce, backward: every TextEncoder and ProsodyPredictor parameter gradient and the style gradient vs
    the reference's autograd.  train: the modules in train mode with the fixture's injected dropout masks (the seven
    dropout calls of the chain, in the reference's order and layouts)."""
    from stts2_mi355x import texttrain, training
    from stts2_mi355x.prosody import matmul
    fx = golden("train_text_T24_B3" if mode == "eval" else "train_text_drop_T24_B3")
    T, lengths = DURATION_CASES[0]
    tok, ln, s, aln = duration_inputs(T, lengths)
    B, F_ = len(lengths), aln.shape[2]
    te, pp = make_duration_modules()
    te, pp = te.cuda().train(mode == "train"), pp.cuda().train(mode == "train")
    calls = []
    if mode == "train":
        def masks(k, shape, p):
            calls.append((k, shape, p))
            return torch.from_numpy(synth.dropout_mask(k, shape, p))
        training.set_dropout_masks(masks)
    probes = {k: torch.from_numpy(synth.normal(f"tt:probe:{k}:{T}", shp)).float().cuda() for k, shp in
              (("asr", (B, 512, F_)), ("d", (B, T, 50)), ("p", (B, 640, F_)))}
    tok_t, ln_t = torch.from_numpy(tok).cuda(), torch.from_numpy(ln)
    sd = torch.from_numpy(s).cuda().requires_grad_(True)
    attn = torch.from_numpy(aln).cuda()
    m = torch.arange(T)[None, :] + 1 > ln_t[:, None]  # length_to_mask (models.py:463-466)
    try:
        t_en = te(tok_t, ln_t, m)
        asr = matmul(t_en, attn)
        d, p = pp(t_en, sd, ln_t, attn, m)
    finally:
        training.set_dropout_masks(None)
    if mode == "train":  # 3 CNN blocks (p 0.2), 3 DurationEncoder LSTMs (0.2), the duration projection (0.5)
        assert [c[2] for c in calls] == [0.2] * 6 + [0.5], calls
    loss_dur, loss_ce = texttrain.duration_losses(d, attn.sum(-1), ln_t)
    loss = ((asr * probes["asr"]).sum() + (d * probes["d"]).sum() + (p * probes["p"]).sum()
            + float(fx["lambda_dur"]) * loss_dur + float(fx["lambda_ce"]) * loss_ce)
    loss.backward()
    for k, ours in (("t_en", t_en), ("d", d), ("p", p)):
        e = _rel(ours.detach(), fx[f"f64.{k}"])
        print(f"output {k}: {e:.2e}")
        assert e < 1e-4, k
    for k, ours in (("loss_dur", loss_dur), ("loss_ce", loss_ce)):
        e = abs(float(ours) - float(fx[f"f64.{k}"])) / abs(float(fx[f"f64.{k}"]))
        print(f"{k}: ours {float(ours):.6f} reference {float(fx[f'f64.{k}']):.6f} rel {e:.2e}")
        assert e < 1e-5, k
    grads = {**{"te." + k: q.grad for k, q in te.named_parameters()},
             **{"pp." + k: q.grad for k, q in pp.named_parameters()}}
    _check_fixture(grads, fx, "text encoder + predictor")
    eo, er = _rel(sd.grad, fx["f64.grad_s"]), _rel(fx["f32.grad_s"], fx["f64.grad_s"])
    print(f"style input grad: ours {eo:.2e}, fp32 reference {er:.2e}")
    assert eo <= max(2 * er, 1e-4)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_row_norm_bwd_vs_torch(mode):
    """stts_row_norm_bwd (LayerNorm + LeakyReLU, AdaLayerNorm + style concat, the plain concat; all with the row
    mask) vs torch's fp64 autograd of the same ops."""
    from stts2_mi355x import texttrain as TT
    torch.manual_seed(5 + mode)
    B, T, C, E = 3, 17, 96, 24
    lens = [17, 11, 4]
    x = torch.randn(B, T, C, dtype=torch.float64) * 2 + 0.3
    gamma, beta = torch.randn(C, dtype=torch.float64), torch.randn(C, dtype=torch.float64)
    gb = torch.randn(B, 2 * C, dtype=torch.float64) * 0.5
    ex = torch.randn(B, E, dtype=torch.float64)
    mask = (torch.arange(T)[None, :] < torch.tensor(lens)[:, None]).double()[..., None]
    Eu = 0 if mode == 0 else E
    gy = torch.randn(B, T, C + Eu, dtype=torch.float64)
    leaves = [t.clone().requires_grad_(True) for t in (x, gamma, beta, gb, ex)]
    xr, gr, br, gbr, exr = leaves
    if mode == 0:
        yr = F.leaky_relu(F.layer_norm(xr, (C,), gr, br, 1e-5), 0.2) * mask
    elif mode == 1:
        yr = torch.cat([(1 + gbr[:, None, :C]) * F.layer_norm(xr, (C,), eps=1e-5) + gbr[:, None, C:],
                        exr[:, None, :].expand(B, T, E)], -1) * mask
    else:
        yr = torch.cat([xr, exr[:, None, :].expand(B, T, E)], -1) * mask
    yr.backward(gy)
    dev = [t.float().cuda().requires_grad_(True) for t in (x, gamma, beta, gb, ex)]
    xd, gd, bd, gbd, exd = dev
    ln = torch.tensor(lens, dtype=torch.int32, device="cuda")
    if mode == 0:
        y = TT.layer_norm_act(xd, gd, bd, 1e-5, 0.2, ln)
    elif mode == 1:
        y = TT.ada_layer_norm(xd, gbd, 1e-5, ln, extra=exd)
    else:
        y = TT.concat_mask(xd, exd, ln)
    y.backward(gy.float().cuda())
    assert _rel(y.detach(), yr.detach()) < 1e-5
    pairs = [("x", xd, xr)] + ([("gamma", gd, gr), ("beta", bd, br)] if mode == 0 else []) + \
            ([("gb", gbd, gbr)] if mode == 1 else []) + ([("extra", exd, exr)] if mode else [])
    for k, a, b in pairs:
        e = _rel(a.grad, b.grad)
        print(f"row_norm mode {mode} d{k}: {e:.2e}")
        assert e < 1e-5, k


def test_embedding_bwd_vs_torch():
    """stts_embedding_bwd: repeated tokens, masked positions, deterministic order: dW equals torch's fp64 autograd of
    embedding + masked_fill, and two runs are bitwise equal."""
    from stts2_mi355x import texttrain as TT
    torch.manual_seed(7)
    B, T, C, n_sym = 4, 30, 320, 50
    lens = [30, 22, 9, 1]
    tok = torch.randint(0, n_sym, (B, T))
    W = torch.randn(n_sym, C, dtype=torch.float64)
    gy = torch.randn(B, T, C, dtype=torch.float64)
    mask = (torch.arange(T)[None, :] < torch.tensor(lens)[:, None]).double()[..., None]
    Wr = W.clone().requires_grad_(True)
    (F.embedding(tok, Wr) * mask).backward(gy)
    ln = torch.tensor(lens, dtype=torch.int32, device="cuda")
    outs = []
    for _ in range(2):
        Wd = W.float().cuda().requires_grad_(True)
        y = TT._EmbeddingFn.apply(Wd, tok.cuda(), ln)
        y.backward(gy.float().cuda())
        outs.append(Wd.grad.clone())
    assert _rel(y.detach(), (F.embedding(tok, W) * mask)) < 1e-6
    e = _rel(outs[0], Wr.grad)
    print(f"embedding dW: {e:.2e}")
    assert e < 1e-6 and torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("lens", [[24, 19, 13], [9, 2, 30]])
def test_duration_losses_vs_train_py(lens):
    """stts_dur_losses vs train.py:286-299 run by torch in fp64 on the CPU (values and the logits gradient), incl. an
    utterance of length 2 (F.l1_loss over no elements: NaN, as torch)."""
    from stts2_mi355x import texttrain as TT
    torch.manual_seed(9)
    B, T, K = len(lens), max(lens), 50
    d = torch.randn(B, T, K, dtype=torch.float64) * 3
    dgt = torch.zeros(B, T, dtype=torch.float64)
    for b, n in enumerate(lens):
        dgt[b, :n] = torch.randint(1, 12, (n,)).double()
    ln = torch.tensor(lens)
    dr = d.clone().requires_grad_(True)
    ld, lc = _dur_losses_ref(dr, dgt, ln)
    gd, gc = 0.7, 1.3
    dd = d.float().cuda().requires_grad_(True)
    od, oc = TT.duration_losses(dd, dgt.float().cuda(), ln)
    has_nan = min(lens) <= 2
    if has_nan:
        assert torch.isnan(od) and torch.isnan(ld)
        (gc * lc).backward()
        (gc * oc).backward()
    else:
        assert abs(float(od) - float(ld)) / abs(float(ld)) < 1e-5
        (gd * ld + gc * lc).backward()
        (gd * od + gc * oc).backward()
    assert abs(float(oc) - float(lc)) / abs(float(lc)) < 1e-5
    e = _rel(dd.grad, dr.grad)
    print(f"dur losses lens {lens}: loss_dur {float(od):.5f} ({float(ld):.5f}), loss_ce {float(oc):.5f} "
          f"({float(lc):.5f}), dlogits {e:.2e}")
    assert e < 1e-5


def test_packed_bilstm_grads_vs_torch():
    """The packed-sequence BiLSTM under autograd (stts_bilstm_fwd_train / _bwd with lengths) vs torch's nn.LSTM over
    pack_padded_sequence in fp64: outputs, input and all 8 parameter gradients; padded rows get no gradient."""
    from stts2_mi355x import texttrain as TT
    from torch.nn.utils.rnn import pack_padded_sequence, pad_packed_sequence
    torch.manual_seed(4)
    B, T, Cin, H = 3, 21, 72, 64
    lens = [21, 14, 3]
    ref = torch.nn.LSTM(Cin, H, 1, batch_first=True, bidirectional=True).double()
    x = torch.randn(B, T, Cin, dtype=torch.float64)
    gy = torch.randn(B, T, 2 * H, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    yp, _ = ref(pack_padded_sequence(xr, torch.tensor(lens), batch_first=True, enforce_sorted=False))
    yr, _ = pad_packed_sequence(yp, batch_first=True, total_length=T)
    yr.backward(gy)
    ours = torch.nn.LSTM(Cin, H, 1, batch_first=True, bidirectional=True)
    ours.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    ours = ours.cuda()
    xd = x.float().cuda().requires_grad_(True)
    y = TT.bilstm(ours, xd, torch.tensor(lens, dtype=torch.int32, device="cuda"))
    y.backward(gy.float().cuda())
    assert _rel(y.detach(), yr.detach()) < 1e-5
    assert _rel(xd.grad, xr.grad) < 1e-5
    for b, n in enumerate(lens):
        assert float(xd.grad[b, n:].abs().max() if n < T else 0.0) == 0.0
    for (k, q), (_, qr) in zip(ours.named_parameters(), ref.named_parameters()):
        e = _rel(q.grad, qr.grad)
        print(f"packed lstm {k}: {e:.2e}")
        assert e < 1e-5, k


def test_text_modules_no_grad_match_inference():
    """The trainable path and the fused inference kernels agree (same modules, same inputs)."""
    T, lengths = DURATION_CASES[0]
    tok, ln, s, aln = duration_inputs(T, lengths)
    te, pp = make_duration_modules()
    te, pp = te.cuda().eval(), pp.cuda().eval()
    tok_t, ln_t, sd, attn = torch.from_numpy(tok).cuda(), torch.from_numpy(ln), torch.from_numpy(s).cuda(), \
        torch.from_numpy(aln).cuda()
    with torch.no_grad():
        a_t = te(tok_t, ln_t)
        a_d, a_p = pp(a_t, sd, ln_t, attn)
    b_t = te(tok_t, ln_t)
    b_d, b_p = pp(b_t, sd.clone().requires_grad_(True), ln_t, attn)
    assert _rel(b_t.detach(), a_t) < 1e-5 and _rel(b_d.detach(), a_d) < 1e-5 and _rel(b_p.detach(), a_p) < 1e-5


def test_trainstep_text_mode():
    """TrainStep(text_encoder=, predictor=, style_encoder=) from the tokens (train.py:217-262, 286-307, 318, 323-327):
    the duration losses equal texttrain.duration_losses over a hand-run predictor forward, g_loss carries
    lambda_ce loss_ce + lambda_dur loss_dur, the text encoder collects gradients through both consumers of t_en (asr and
    the predictor) and its AdamW step moves it by at most lr."""
    from test_gpu_train_step import _discs, _train_inputs
    from helpers import fill_module, make_decoder
    from stts2_mi355x import texttrain
    from stts2_mi355x.models import StyleEncoder
    from stts2_mi355x.trainstep import TrainStep
    T, lengths = 24, (24, 20)
    tok, ln, s, aln = duration_inputs(T, lengths)
    B, Fm = len(lengths), aln.shape[2]
    ml = 40
    Fb = aln.sum((1, 2)).astype(int)
    starts = [int(min(3, f - ml)) for f in Fb]
    assert min(starts) >= 0
    _, _, _, _, wav, noise = _train_inputs(B, ml)
    mels = torch.from_numpy(np.stack([synth.normal(f"tt:mel:{b}:{Fm}", (80, 2 * Fm)) for b in range(B)])).cuda()
    F0_real = torch.from_numpy(synth.normal(f"tt:f0real:{ml}", (B, 2 * ml))).float().abs().cuda() * 200
    N_real = torch.from_numpy(synth.normal(f"tt:nreal:{ml}", (B, 2 * ml))).float().cuda()
    te, pp = make_duration_modules()
    te, pp = te.cuda().eval(), pp.cuda().eval()
    dec, _ = make_decoder("hifigan")
    mpd, msd = _discs()
    se = fill_module(StyleEncoder(dim_in=64, style_dim=128, max_conv_dim=512)).cuda().eval()
    te0 = {k: v.detach().clone() for k, v in te.named_parameters()}
    step = TrainStep(dec.cuda().eval(), mpd.cuda().train(), msd.cuda().train(), predictor=pp, style_encoder=se,
                     text_encoder=te, capture=True)
    attn = torch.from_numpy(aln).cuda()
    text = dict(texts=torch.from_numpy(tok).cuda(), input_lengths=torch.from_numpy(ln), attn=attn, attn_mono=attn,
                mels=mels, starts=starts, mel_len=ml)
    # the predictor's duration logits of the same (pre-step) weights, by hand, for the loss check
    with torch.no_grad():
        t_en0 = te(torch.from_numpy(tok).cuda(), torch.from_numpy(ln))
        d0, _ = pp(t_en0, se(mels.unsqueeze(1)), torch.from_numpy(ln), attn)
        ld0, lc0 = texttrain.duration_losses(d0, attn.sum(-1), torch.from_numpy(ln))
    out = step(None, None, None, None, wav.cuda(), noise=noise.cuda(), F0_real=F0_real, N_real=N_real, text=text)
    for k, ref in (("loss_dur", ld0), ("loss_ce", lc0)):
        assert abs(float(out[k]) - float(ref)) <= 1e-5 * abs(float(ref)), k
    parts = (5.0 * out["loss_mel"] + out["loss_gen_all"] + out["loss_F0_rec"] + out["loss_norm_rec"]
             + out["loss_ce"] + out["loss_dur"])
    assert abs(float(out["g_loss"]) - float(parts)) <= 1e-5 * abs(float(parts))
    got = step.captured["text_encoder"]
    assert set(got) == {k for k, _ in te.named_parameters()}
    assert all(torch.isfinite(g).all() for g in got.values())
    assert float(got["embedding.weight"].abs().max()) > 0 and float(got["lstm.weight_hh_l0"].abs().max()) > 0
    moved = [float((p.detach() - te0[k]).abs().max()) for k, p in te.named_parameters()]
    assert max(moved) <= 1.5e-4 and sorted(moved)[len(moved) // 2] > 0
    print(f"TrainStep text mode: loss_dur {float(out['loss_dur']):.4f}, loss_ce {float(out['loss_ce']):.4f}, "
          f"g_loss {float(out['g_loss']):.4f}; text encoder max step {max(moved):.2e}")
