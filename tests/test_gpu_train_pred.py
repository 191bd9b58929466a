"""GPU parity of the trainable ProsodyPredictor.F0Ntrain and StyleEncoder (train.py's G step differentiates both:
train.py:258, 265, 318, 323-324) through the C-ABI, against the REFERENCE modules' own autograd
(tests/golden/train_f0n_*.npz, train_style_*.npz from tests/golden/make_golden_train_pred.py: fp64 = the truth,
fp32 = the reference as it runs), eval mode (dropout off); the train-mode dropout separately.

Bound: every parameter / input gradient within 1e-4 of the module's largest |g| (normwise), and
per tensor no worse than max(2 x the fp32 reference's own error vs fp64, 1e-4 of the tensor's scale)."""
import numpy as np
import pytest
import torch

from helpers import fill_module, golden
from stts2_mi355x import synth

pytestmark = pytest.mark.gpu


def _check_fixture(grads, fx, what, norm_tol=1e-4):
    names = [str(k) for k in fx["names"]]
    gm = float(fx["f64.maxabs"].max())
    worst, worst_ref, worst_n = (0.0, ""), (0.0, ""), (0.0, "")
    for i, k in enumerate(names):
        assert grads.get(k) is not None, f"{what}: no gradient for {k}"
        g = grads[k].detach().double().cpu().reshape(-1)[torch.from_numpy(fx["f64.idx"][i])].numpy()
        scale = max(float(fx["f64.maxabs"][i]), 1e-3 * gm)
        eo = np.abs(g - fx["f64.val"][i]).max() / scale
        er = np.abs(fx["f32.val"][i] - fx["f64.val"][i]).max() / scale
        en = np.abs(g - fx["f64.val"][i]).max() / gm
        worst, worst_ref, worst_n = max(worst, (eo, k)), max(worst_ref, (er, k)), max(worst_n, (en, k))
        assert eo <= max(2.0 * er, 1e-4), (what, k, eo, er)
        assert en <= norm_tol, (what, k, "normwise", en)
    print(f"{what}: vs fp64 worst {worst[0]:.2e} ({worst[1]}), fp32 reference worst {worst_ref[0]:.2e} "
          f"({worst_ref[1]}), module-normwise {worst_n[0]:.2e} ({worst_n[1]}), {len(names)} tensors")


def _rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max() / b.abs().max())


def _predictor():
    from stts2_mi355x.models import ProsodyPredictor
    return fill_module(ProsodyPredictor(style_dim=128, d_hid=512, nlayers=3, max_dur=50, dropout=0.2)).cuda()


def test_bilstm_grads_vs_torch():
    """The trainable BiLSTM (stts_bilstm_fwd_train / stts_bilstm_bwd) against torch's nn.LSTM autograd in fp64."""
    from stts2_mi355x import training as Tr
    torch.manual_seed(3)
    B, T, Cin, H = 3, 23, 80, 64
    ref = torch.nn.LSTM(Cin, H, 1, batch_first=True, bidirectional=True).double()
    x = torch.randn(B, T, Cin, dtype=torch.float64)
    gy = torch.randn(B, T, 2 * H, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    yr, _ = ref(xr)
    yr.backward(gy)
    ours = torch.nn.LSTM(Cin, H, 1, batch_first=True, bidirectional=True)
    ours.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    ours = ours.cuda()
    xd = x.float().cuda().requires_grad_(True)
    y = Tr.bilstm_frames(ours, xd)
    y.backward(gy.float().cuda())
    assert _rel(y.detach(), yr.detach()) < 1e-5
    assert _rel(xd.grad, xr.grad) < 1e-5
    for (k, p), (_, pr) in zip(ours.named_parameters(), ref.named_parameters()):
        e = _rel(p.grad, pr.grad)
        print(f"lstm {k}: {e:.2e}")
        assert e < 1e-5, k


def test_f0ntrain_grads_vs_reference():
    """F0Ntrain under autograd (eval: dropout off) vs the reference module's autograd: outputs, every shared /
    F0 / N / projection parameter gradient and the input gradients (en, s)."""
    fx = golden("train_f0n_T12_B2")
    B, T = int(fx["B"]), int(fx["T"])
    pp = _predictor().eval()
    en = torch.from_numpy(np.stack([synth.normal(f"tp:en:{b}:{T}", (640, T)) for b in range(B)])).cuda()
    s = torch.from_numpy(np.stack([synth.normal(f"tp:s:{b}", (128,)) for b in range(B)])).cuda()
    rF, rN = (torch.from_numpy(synth.normal(f"tp:probe:{k}:{T}", (B, 2 * T))).float().cuda() for k in ("F0", "N"))
    en.requires_grad_(True)
    s.requires_grad_(True)
    F0, N = pp.F0Ntrain(en, s)
    ((F0 * rF).sum() + (N * rN).sum()).backward()
    assert _rel(F0.detach(), fx["f64.F0"]) < 1e-4 and _rel(N.detach(), fx["f64.N"]) < 1e-4
    _check_fixture({k: p.grad for k, p in pp.named_parameters()}, fx, "F0Ntrain params")
    for k, t in (("en", en), ("s", s)):
        eo, er = _rel(t.grad, fx[f"f64.grad_{k}"]), _rel(fx[f"f32.grad_{k}"], fx[f"f64.grad_{k}"])
        print(f"F0Ntrain input {k}: ours {eo:.2e}, fp32 reference {er:.2e}")
        assert eo <= max(2 * er, 1e-4), k


@pytest.mark.parametrize("Fr,B", [(80, 2), (97, 1)])
def test_style_encoder_grads_vs_reference(Fr, B):
    """StyleEncoder under autograd vs the reference module's autograd (97 frames: odd widths at every
    DownSample, the repeated last column)."""
    from stts2_mi355x.models import StyleEncoder
    fx = golden(f"train_style_F{Fr}_B{B}")
    se = fill_module(StyleEncoder(dim_in=64, style_dim=128, max_conv_dim=512)).cuda().eval()
    mel = torch.from_numpy(np.stack([synth.normal(f"tp:mel:{b}:{Fr}", (1, 80, Fr)) for b in range(B)])).cuda()
    r = torch.from_numpy(synth.normal(f"tp:probe:style:{Fr}", (B, 128))).float().cuda()
    mel.requires_grad_(True)
    out = se(mel)
    (out * r).sum().backward()
    assert _rel(out.detach(), fx["f64.out"]) < 1e-4
    _check_fixture({k: p.grad for k, p in se.named_parameters()}, fx, f"StyleEncoder F={Fr}")
    eo, er = _rel(mel.grad, fx["f64.grad_mel"]), _rel(fx["f32.grad_mel"], fx["f64.grad_mel"])
    print(f"StyleEncoder input grad: ours {eo:.2e}, fp32 reference {er:.2e}")
    assert eo <= max(2 * er, 1e-4)


def test_style_encoder_no_grad_matches_engine():
    """The trainable path and the fused inference engine agree (same module, same input)."""
    from stts2_mi355x.models import StyleEncoder
    se = fill_module(StyleEncoder(dim_in=64, style_dim=128, max_conv_dim=512)).cuda().eval()
    mel = torch.from_numpy(synth.normal("tp:mel:x", (2, 1, 80, 96))).cuda()  # >= 80 frames: the 5x5 valid conv
    with torch.no_grad():
        a = se(mel)
    b = se(mel.clone().requires_grad_(True))
    assert _rel(b.detach(), a) < 1e-4


def test_dropout_train_mode():
    """Train-mode dropout (stts_dropout): keep rate ~ 1 - p, kept values scaled by 1 / (1 - p), the gradient
    through the same mask, torch.manual_seed reproduces the draw; F0Ntrain in train mode differs from eval and
    is reproducible under the same seed."""
    from stts2_mi355x import training as Tr
    x = torch.randn(1 << 20, device="cuda").abs() + 0.5
    xd = x.clone().requires_grad_(True)
    torch.manual_seed(11)
    y = Tr.dropout(xd, 0.2)
    keep = y != 0
    rate = float(keep.float().mean())
    assert abs(rate - 0.8) < 5e-3, rate
    assert torch.allclose(y[keep], x[keep] / 0.8)
    g = torch.randn_like(x)
    y.backward(g)
    assert torch.allclose(xd.grad, torch.where(keep, g / 0.8, torch.zeros_like(g)))
    assert torch.equal(xd.grad != 0, keep)
    torch.manual_seed(11)
    assert torch.equal(Tr.dropout(x, 0.2), y.detach())
    pp = _predictor().train()
    T, B = 12, 2
    en = torch.from_numpy(np.stack([synth.normal(f"tp:en:{b}:{T}", (640, T)) for b in range(B)])).cuda()
    s = torch.from_numpy(np.stack([synth.normal(f"tp:s:{b}", (128,)) for b in range(B)])).cuda()
    torch.manual_seed(5)
    F0a, _ = pp.F0Ntrain(en, s)
    torch.manual_seed(5)
    F0b, _ = pp.F0Ntrain(en, s)
    F0e, _ = pp.eval().F0Ntrain(en, s)
    assert torch.equal(F0a, F0b)
    assert _rel(F0a.detach(), F0e.detach()) > 1e-3


def test_train_step_with_predictor_and_style_encoder():
    """TrainStep(predictor=, style_encoder=) (train.py:258-270, 300-307, 323-324) against the same step composed by
    hand: s / F0 / N from the two modules, the plain step on detached leaves, then the modules' backward with the
    leaves' gradients plus torch's smooth-L1 gradients.  Checks the wiring: the loss terms (vs torch
    F.smooth_l1_loss), that s collects the gradients of both its consumers, every predictor / style-encoder
    gradient the optimizers consumed, and that the AdamW steps moved those modules."""
    import torch.nn.functional as F
    from test_gpu_train_step import _discs, _train_inputs
    from helpers import make_decoder
    from stts2_mi355x.models import StyleEncoder
    from stts2_mi355x.trainstep import TrainStep
    B, T = 2, 48  # gt = 96 mel frames (the style encoder's valid 5x5 conv needs >= 80)
    asr, _, _, _, wav, noise = _train_inputs(B, T)
    p_en = torch.from_numpy(np.stack([synth.normal(f"tp:en:{b}:{T}", (640, T)) for b in range(B)]))
    gt = torch.from_numpy(np.stack([synth.normal(f"tp:mel:{b}:{2 * T}", (80, 2 * T)) for b in range(B)]))
    F0_real = torch.from_numpy(synth.normal(f"tp:f0real:{T}", (B, 2 * T))).float().abs() * 200
    N_real = torch.from_numpy(synth.normal(f"tp:nreal:{T}", (B, 2 * T))).float()
    mods = []
    for _ in range(2):
        dec, _ = make_decoder("hifigan")
        mpd, msd = _discs()
        se = fill_module(StyleEncoder(dim_in=64, style_dim=128, max_conv_dim=512))
        mods.append((dec.cuda().eval(), mpd.cuda().train(), msd.cuda().train(), _predictor().eval(), se.cuda().eval()))
    cu = lambda t: t.cuda()  # noqa: E731
    # the step under test
    dec, mpd, msd, pp, se = mods[0]
    pp0 = {k: v.detach().clone() for k, v in pp.named_parameters()}
    se0 = {k: v.detach().clone() for k, v in se.named_parameters()}
    step = TrainStep(dec, mpd, msd, predictor=pp, style_encoder=se, capture=True)
    out = step(cu(asr), None, None, None, cu(wav), noise=cu(noise), p_en=cu(p_en), gt=cu(gt), F0_real=cu(F0_real),
               N_real=cu(N_real))
    # composed by hand
    dec2, mpd2, msd2, pp2, se2 = mods[1]
    s = se2(cu(gt).unsqueeze(1))
    F0, N = pp2.F0Ntrain(cu(p_en), s)
    leaves = [t.detach().clone().requires_grad_(True) for t in (F0, N, s)]
    ref = TrainStep(dec2, mpd2, msd2, capture=True)(cu(asr), leaves[0], leaves[1], leaves[2], cu(wav), noise=cu(noise))
    F0c, Nc = F0.detach().clone().requires_grad_(True), N.detach().clone().requires_grad_(True)
    lF0 = F.smooth_l1_loss(cu(F0_real), F0c) / 10
    lN = F.smooth_l1_loss(cu(N_real), Nc)
    (lF0 + lN).backward()
    torch.autograd.backward([F0, N, s], [leaves[0].grad + F0c.grad, leaves[1].grad + Nc.grad, leaves[2].grad])
    assert abs(float(out["loss_F0_rec"]) - float(lF0)) <= 1e-6 * abs(float(lF0))
    assert abs(float(out["loss_norm_rec"]) - float(lN)) <= 1e-6 * abs(float(lN))
    for k in ("d_loss", "loss_mel", "loss_gen_all"):
        assert abs(float(out[k]) - float(ref[k])) <= 1e-5 * abs(float(ref[k])), k
    assert abs(float(out["g_loss"]) - float(ref["g_loss"] + lF0 + lN)) <= 1e-5 * abs(float(out["g_loss"]))
    for tag, m in (("predictor", pp2), ("style_encoder", se2)):
        got = step.captured[tag]
        gm = max(float(p.grad.abs().max()) for p in m.parameters() if p.grad is not None)
        worst = max((_rel(got[k], p.grad) * float(p.grad.abs().max()) / gm, k) for k, p in m.named_parameters()
                    if p.grad is not None)
        print(f"{tag}: {len(got)} gradients, worst module-normwise difference {worst[0]:.2e} ({worst[1]})")
        assert worst[0] < 1e-4, (tag, worst)
    moved = [float((p.detach() - pp0[k]).abs().max()) for k, p in pp.named_parameters() if k in step.captured["predictor"]]
    assert min(moved) > 0 and max(moved) <= 1.5e-4  # one AdamW step at lr 1e-4
    moved = [float((p.detach() - se0[k]).abs().max()) for k, p in se.named_parameters()]
    assert min(moved) > 0 and max(moved) <= 1.5e-5  # lr 1e-5
