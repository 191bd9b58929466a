"""ORACLE — test infrastructure only.  CPU restatement of the StyleTTS2-lite synthesis path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / CPU baseline; the product path (the HIP library
behind include/stts2.h) never calls it.

Each function restates one reference function op for op with stock PyTorch-CPU ops
on a plain state dict (the reference modules themselves never leave the survey
container).  Pinning: tests/golden/*.npz were produced by importing the reference
modules (tests/golden/make_golden.py) on formula weights/inputs/noise
(stts2_mi355x/synth.py); tests/test_oracle_golden.py checks this file against them.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

SQRT2 = math.sqrt(2)


def _t(sd, k):
    v = sd[k]
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))


def wn(sd, p):
    """torch.nn.utils.weight_norm(dim=0) fold, as the reference's forward pre-hook computes it."""
    return torch._weight_norm(_t(sd, p + ".weight_v"), _t(sd, p + ".weight_g"), 0)


def _bias(sd, p):
    k = p + ".bias"
    return _t(sd, k) if k in sd else None


def snake(x, a):
    """Snake1D, reference hifigan.py:68 / :329: x + (1/a) * sin(a*x)**2."""
    return x + (1 / a) * (torch.sin(a * x) ** 2)


def adain1d(x, s, sd, p):
    """reference hifigan.py:14-24 (AdaIN1d): (1+gamma)*InstanceNorm(x)+beta, h = fc(s)."""
    h = F.linear(s, _t(sd, p + ".fc.weight"), _t(sd, p + ".fc.bias"))
    h = h.view(h.size(0), h.size(1), 1)
    gamma, beta = torch.chunk(h, chunks=2, dim=1)
    return (1 + gamma) * F.instance_norm(x, eps=1e-5) + beta


def adain_resblock1(x, s, sd, p, kernel_size, dilation):
    """reference hifigan.py:65-74 (AdaINResBlock1.forward)."""
    for j, d in enumerate(dilation):
        a1 = _t(sd, f"{p}.alpha1.{j}")
        a2 = _t(sd, f"{p}.alpha2.{j}")
        xt = adain1d(x, s, sd, f"{p}.adain1.{j}")
        xt = xt + (1 / a1) * (torch.sin(a1 * xt) ** 2)
        xt = F.conv1d(xt, wn(sd, f"{p}.convs1.{j}"), _bias(sd, f"{p}.convs1.{j}"), 1,
                      (kernel_size * d - d) // 2, d)
        xt = adain1d(xt, s, sd, f"{p}.adain2.{j}")
        xt = xt + (1 / a2) * (torch.sin(a2 * xt) ** 2)
        xt = F.conv1d(xt, wn(sd, f"{p}.convs2.{j}"), _bias(sd, f"{p}.convs2.{j}"), 1, (kernel_size - 1) // 2, 1)
        x = xt + x
    return x


def adain_resblk1d(x, s, sd, p, upsample: bool, learned_sc: bool):
    """reference hifigan.py:359-403 == models.py:326-370 (AdainResBlk1d, eval: dropout = identity)."""
    r = adain1d(x, s, sd, p + ".norm1")
    r = F.leaky_relu(r, 0.2)
    if upsample:
        C = r.shape[1]
        r = F.conv_transpose1d(r, wn(sd, p + ".pool"), _bias(sd, p + ".pool"), stride=2, padding=1,
                               output_padding=1, groups=C)
    r = F.conv1d(r, wn(sd, p + ".conv1"), _bias(sd, p + ".conv1"), 1, 1)
    r = adain1d(r, s, sd, p + ".norm2")
    r = F.leaky_relu(r, 0.2)
    r = F.conv1d(r, wn(sd, p + ".conv2"), _bias(sd, p + ".conv2"), 1, 1)
    sc = F.interpolate(x, scale_factor=2, mode="nearest") if upsample else x
    if learned_sc:
        sc = F.conv1d(sc, wn(sd, p + ".conv1x1"), None)
    return (r + sc) / SQRT2


# ----------------------------------------------------------------------------------
# harmonic-plus-noise source
# ----------------------------------------------------------------------------------

def sine_source(f0_curve, sd, p, upsample_scale: int, noise):
    """reference hifigan.py:189-218 (SineGen.forward) + :254-268 (SourceModuleHnNSF) + :323.

    f0_curve [B, 2T]; noise [B, L, 9] = the randn_like(sine_waves) draw (hifigan.py:213).
    rand_ini (hifigan.py:126-129) is added to sample 0 only and the ÷upsample_scale linear
    downsample reads samples 300j+149/150 only, so it never reaches the output (measured
    diff 0.0); it is omitted.  Returns har [B, L, 1] (pre-transpose)."""
    with torch.no_grad():  # SourceModuleHnNSF.forward runs l_sin_gen under no_grad (hifigan.py:262-263)
        # (always in fp32, the reference's dtype: an fp64 run of the oracle, the training tests' truth,
        # keeps the reference's fp32 phase quantisation)
        f0_curve, noise = f0_curve.float(), noise.float()
        f0 = F.interpolate(f0_curve[:, None], scale_factor=upsample_scale).transpose(1, 2)  # nearest, [B,L,1]
        fn = torch.multiply(f0, torch.FloatTensor([[range(1, 10)]]))
        rad_values = (fn / 24000) % 1
        rad_values = F.interpolate(rad_values.transpose(1, 2), scale_factor=1 / upsample_scale,
                                   mode="linear").transpose(1, 2)
        phase = torch.cumsum(rad_values, dim=1) * 2 * np.pi
        phase = F.interpolate(phase.transpose(1, 2) * upsample_scale, scale_factor=upsample_scale,
                              mode="linear").transpose(1, 2)
        sine_waves = torch.sin(phase) * 0.1
        uv = (f0 > 10).type(torch.float32)
        noise_amp = uv * 0.003 + (1 - uv) * 0.1 / 3
        sine_waves = sine_waves * uv + noise_amp * noise
    w = _t(sd, p + ".l_linear.weight")
    return torch.tanh(F.linear(sine_waves.to(w.dtype), w, _t(sd, p + ".l_linear.bias")))


# ----------------------------------------------------------------------------------
# HiFi-GAN decoder
# ----------------------------------------------------------------------------------

def generator_hifigan(x, s, f0_curve, sd, cfg, noise, taps=None):
    """reference hifigan.py:321-347 (Generator.forward)."""
    rates, kernels = cfg["upsample_rates"], cfg["upsample_kernel_sizes"]
    rks, rds = cfg["resblock_kernel_sizes"], cfg["resblock_dilation_sizes"]
    nk = len(rks)
    scale = int(np.prod(rates))
    src = sine_source(f0_curve, sd, "generator.m_source", scale, noise)
    har = src.transpose(1, 2)
    if taps is not None:
        taps["source"] = src
    for i, (u, k) in enumerate(zip(rates, kernels)):
        a = _t(sd, f"generator.alphas.{i}")
        x = x + (1 / a) * (torch.sin(a * x) ** 2)
        if i + 1 < len(rates):
            sf = int(np.prod(rates[i + 1:]))
            xs_src = F.conv1d(har, _t(sd, f"generator.noise_convs.{i}.weight"),
                              _t(sd, f"generator.noise_convs.{i}.bias"), sf, (sf + 1) // 2)
            xs_src = adain_resblock1(xs_src, s, sd, f"generator.noise_res.{i}", 7, [1, 3, 5])
        else:
            xs_src = F.conv1d(har, _t(sd, f"generator.noise_convs.{i}.weight"),
                              _t(sd, f"generator.noise_convs.{i}.bias"))
            xs_src = adain_resblock1(xs_src, s, sd, f"generator.noise_res.{i}", 11, [1, 3, 5])
        x = F.conv_transpose1d(x, wn(sd, f"generator.ups.{i}"), _bias(sd, f"generator.ups.{i}"), u,
                               u // 2 + u % 2, u % 2)
        x = x + xs_src
        xs = None
        for j in range(nk):
            r = adain_resblock1(x, s, sd, f"generator.resblocks.{i * nk + j}", rks[j], rds[j])
            xs = r if xs is None else xs + r
        x = xs / nk
        if taps is not None:
            taps[f"stage{i}"] = x
    a = _t(sd, f"generator.alphas.{len(rates)}")
    x = x + (1 / a) * (torch.sin(a * x) ** 2)
    x = F.conv1d(x, wn(sd, "generator.conv_post"), _bias(sd, "generator.conv_post"), 1, 3)
    if taps is not None:
        taps["pre_tanh"] = x
    return torch.tanh(x)


def decoder_frontend(asr, F0_curve, N, s, sd):
    """reference hifigan.py:458-472 == istftnet.py:704-718 (eval branch)."""
    F0 = F.conv1d(F0_curve.unsqueeze(1), wn(sd, "F0_conv"), _bias(sd, "F0_conv"), 2, 1)
    Nc = F.conv1d(N.unsqueeze(1), wn(sd, "N_conv"), _bias(sd, "N_conv"), 2, 1)
    x = torch.cat([asr, F0, Nc], axis=1)
    x = adain_resblk1d(x, s, sd, "encode", False, True)
    asr_res = F.conv1d(asr, wn(sd, "asr_res.0"), _bias(sd, "asr_res.0"))
    res = True
    for i in range(4):
        if res:
            x = torch.cat([x, asr_res, F0, Nc], axis=1)
        up = i == 3
        x = adain_resblk1d(x, s, sd, f"decode.{i}", up, True)  # dim_in 1090 != dim_out
        if up:
            res = False
    return x


def train_smooth(F0_curve, N, F0_down, N_down):
    """Decoder.forward's train-mode branch (hifigan.py:447-455): box-smooth F0_curve over F0_down frames
    and N over N_down frames (0 = off); the reference draws F0_down from [0, 3, 7] and N_down from
    [0, 3, 7, 15] with random.randint."""
    if F0_down:
        F0_curve = F.conv1d(F0_curve.unsqueeze(1), torch.ones(1, 1, F0_down, dtype=F0_curve.dtype),
                            padding=F0_down // 2).squeeze(1) / F0_down
    if N_down:
        N = F.conv1d(N.unsqueeze(1), torch.ones(1, 1, N_down, dtype=N.dtype), padding=N_down // 2).squeeze(1) / N_down
    return F0_curve, N


def decoder_hifigan(asr, F0_curve, N, s, sd, cfg, noise, taps=None, smooth=None):
    """reference hifigan.py:446-475 (Decoder.forward; eval, or the train-mode smoothing with
    smooth = (F0_down, N_down))."""
    if smooth is not None:
        F0_curve, N = train_smooth(F0_curve, N, *smooth)
    x = decoder_frontend(asr, F0_curve, N, s, sd)
    if taps is not None:
        taps["frontend"] = x
    return generator_hifigan(x, s, F0_curve, sd, cfg, noise, taps)


# ----------------------------------------------------------------------------------
# iSTFTNet decoder
# ----------------------------------------------------------------------------------

def stft_transform(wave, sd, n_fft, hop):
    """reference istftnet.py:207-243 (CustomSTFT.transform, center=True, replicate pad)."""
    pad = n_fft // 2
    wave = F.pad(wave, (pad, pad), mode="replicate")
    x = wave.unsqueeze(1)
    re = F.conv1d(x, _t(sd, "generator.stft.weight_forward_real"), None, stride=hop, padding=0)
    im = F.conv1d(x, _t(sd, "generator.stft.weight_forward_imag"), None, stride=hop, padding=0)
    mag = torch.sqrt(re ** 2 + im ** 2 + 1e-14)
    phase = torch.atan2(im, re)
    phase[(im == 0) & (re < 0)] = torch.pi
    return mag, phase


def stft_inverse(mag, phase, sd, n_fft, hop):
    """reference istftnet.py:246-293 (CustomSTFT.inverse; no window-sum normalisation)."""
    re = mag * torch.cos(phase)
    im = mag * torch.sin(phase)
    rr = F.conv_transpose1d(re, _t(sd, "generator.stft.weight_backward_real"), None, stride=hop, padding=0)
    ii = F.conv_transpose1d(im, _t(sd, "generator.stft.weight_backward_imag"), None, stride=hop, padding=0)
    w = rr - ii
    pad = n_fft // 2
    return w[..., pad:-pad]


def generator_istft(x, s, f0_curve, sd, cfg, noise, taps=None):
    """reference istftnet.py:543-573 (Generator.forward)."""
    rates, kernels = cfg["upsample_rates"], cfg["upsample_kernel_sizes"]
    rks, rds = cfg["resblock_kernel_sizes"], cfg["resblock_dilation_sizes"]
    n_fft, hop = cfg["gen_istft_n_fft"], cfg["gen_istft_hop_size"]
    nk = len(rks)
    scale = int(np.prod(rates)) * hop
    src = sine_source(f0_curve, sd, "generator.m_source", scale, noise)
    if taps is not None:
        taps["source"] = src
    har_source = src.transpose(1, 2).squeeze(1)
    spec, ph = stft_transform(har_source, sd, n_fft, hop)
    har = torch.cat([spec, ph], dim=1)
    if taps is not None:
        taps["har"] = har
    for i, (u, k) in enumerate(zip(rates, kernels)):
        x = F.leaky_relu(x, 0.1)
        if i + 1 < len(rates):
            sf = int(np.prod(rates[i + 1:]))
            xs_src = F.conv1d(har, _t(sd, f"generator.noise_convs.{i}.weight"),
                              _t(sd, f"generator.noise_convs.{i}.bias"), sf, (sf + 1) // 2)
            xs_src = adain_resblock1(xs_src, s, sd, f"generator.noise_res.{i}", 7, [1, 3, 5])
        else:
            xs_src = F.conv1d(har, _t(sd, f"generator.noise_convs.{i}.weight"),
                              _t(sd, f"generator.noise_convs.{i}.bias"))
            xs_src = adain_resblock1(xs_src, s, sd, f"generator.noise_res.{i}", 11, [1, 3, 5])
        x = F.conv_transpose1d(x, wn(sd, f"generator.ups.{i}"), _bias(sd, f"generator.ups.{i}"), u, (k - u) // 2)
        if i == len(rates) - 1:
            x = F.pad(x, (1, 0), mode="reflect")
        x = x + xs_src
        xs = None
        for j in range(nk):
            r = adain_resblock1(x, s, sd, f"generator.resblocks.{i * nk + j}", rks[j], rds[j])
            xs = r if xs is None else xs + r
        x = xs / nk
        if taps is not None:
            taps[f"stage{i}"] = x
    x = F.leaky_relu(x)
    x = F.conv1d(x, wn(sd, "generator.conv_post"), _bias(sd, "generator.conv_post"), 1, 3)
    if taps is not None:
        taps["post"] = x
    nb = n_fft // 2 + 1
    spec = torch.exp(x[:, :nb, :])
    phase = torch.sin(x[:, nb:, :])
    return stft_inverse(spec, phase, sd, n_fft, hop)


def decoder_istft(asr, F0_curve, N, s, sd, cfg, noise, taps=None):
    """reference istftnet.py:692-721 (Decoder.forward, eval)."""
    x = decoder_frontend(asr, F0_curve, N, s, sd)
    if taps is not None:
        taps["frontend"] = x
    return generator_istft(x, s, F0_curve, sd, cfg, noise, taps)


# ----------------------------------------------------------------------------------
# ProsodyPredictor.F0Ntrain and StyleEncoder
# ----------------------------------------------------------------------------------

def f0n_convstacks(xl, s, sd, prefix="", taps=None):
    """reference models.py:451-461: F0 / N AdainResBlk1d stacks + 1x1 projections.
    xl = shared-LSTM output, [B, d_hid, T] (models.py:449-451)."""
    out = []
    for br in ("F0", "N"):
        h = xl
        for i in range(3):
            p = f"{prefix}{br}.{i}"
            ls = (p + ".conv1x1.weight_v") in sd
            h = adain_resblk1d(h, s, sd, p, upsample=(i == 1), learned_sc=ls)
        h = F.conv1d(h, _t(sd, f"{prefix}{br}_proj.weight"), _t(sd, f"{prefix}{br}_proj.bias"))
        out.append(h.squeeze(1))
    return tuple(out)


def shared_lstm(en, sd, prefix="", d_hid=512, style_dim=128):
    """reference models.py:449: nn.LSTM(d_hid+style_dim, d_hid//2, bidirectional, batch_first)."""
    lstm = torch.nn.LSTM(d_hid + style_dim, d_hid // 2, 1, batch_first=True, bidirectional=True)
    lsd = {k[len(prefix) + 7:]: _t(sd, k) for k in sd if k.startswith(prefix + "shared.")}
    lstm.load_state_dict(lsd)
    with torch.no_grad():
        x, _ = lstm(en.transpose(-1, -2))
    return x.transpose(-1, -2)


def f0ntrain(en, s, sd, prefix=""):
    """reference models.py:448-461 (ProsodyPredictor.F0Ntrain)."""
    xl = shared_lstm(en, sd, prefix)
    return f0n_convstacks(xl, s, sd, prefix)


def _down_half(x):
    """reference models.py:58-61 (DownSample 'half')."""
    if x.shape[-1] % 2 != 0:
        x = torch.cat([x, x[..., -1].unsqueeze(-1)], dim=-1)
    return F.avg_pool2d(x, 2)


def resblk2d(x, sd, p, learned_sc):
    """reference models.py:82-123 (ResBlk, normalize=False, downsample='half')."""
    sc = x
    if learned_sc:
        sc = F.conv2d(sc, _t(sd, p + ".conv1x1.weight"), None)
    sc = _down_half(sc)
    r = F.leaky_relu(x, 0.2)
    r = F.conv2d(r, _t(sd, p + ".conv1.weight"), _t(sd, p + ".conv1.bias"), 1, 1)
    C = r.shape[1]
    r = F.conv2d(r, _t(sd, p + ".downsample_res.conv.weight"), _t(sd, p + ".downsample_res.conv.bias"),
                 2, 1, 1, C)
    r = F.leaky_relu(r, 0.2)
    r = F.conv2d(r, _t(sd, p + ".conv2.weight"), _t(sd, p + ".conv2.bias"), 1, 1)
    return (sc + r) / SQRT2


def style_encoder(mel, sd, prefix="", taps=None):
    """reference models.py:125-150 (StyleEncoder.forward). mel [B,1,80,F] -> [B,style_dim]."""
    h = F.conv2d(mel, _t(sd, prefix + "shared.0.weight"), _t(sd, prefix + "shared.0.bias"), 1, 1)
    for i in range(1, 5):
        p = f"{prefix}shared.{i}"
        h = resblk2d(h, sd, p, (p + ".conv1x1.weight") in sd)
        if taps is not None:
            taps[f"blk{i}"] = h
    h = F.leaky_relu(h, 0.2)
    h = F.conv2d(h, _t(sd, prefix + "shared.6.weight"), _t(sd, prefix + "shared.6.bias"))
    h = F.adaptive_avg_pool2d(h, 1)
    h = F.leaky_relu(h, 0.2)
    h = h.view(h.size(0), -1)
    return F.linear(h, _t(sd, prefix + "unshared.weight"), _t(sd, prefix + "unshared.bias"))


# ---------------------------------------------------------------- style front-end
# Parity unpinned upstream: the reference builds its mel with torchaudio (absent from this image and
# from the reference tree), so these restate torchaudio's published MelSpectrogram defaults as the
# reference instantiates them (inference.py:43-49): MelSpectrogram(n_mels=80, n_fft=2048,
# win_length=1200, hop_length=300) with every other argument at its default -- sample_rate 16000
# (the reference never passes 24000), f_min 0, f_max sample_rate/2, hann_window(periodic), power 2,
# center=True with reflect padding, onesided, norm None, HTK mel scale.
MEL = dict(n_mels=80, n_fft=2048, win_length=1200, hop_length=300, sample_rate=16000, mean=-4.0, std=4.0)


def _hz_to_mel_htk(f):
    return 2595.0 * math.log10(1.0 + f / 700.0)


def melscale_fbanks(n_freqs=1025, f_min=0.0, f_max=8000.0, n_mels=80, sample_rate=16000):
    """torchaudio.functional.melscale_fbanks(norm=None, mel_scale="htk"): [n_freqs, n_mels] fp32."""
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_pts = torch.linspace(_hz_to_mel_htk(f_min), _hz_to_mel_htk(f_max), n_mels + 2)
    f_pts = 700.0 * (10 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.clamp(torch.min(down, up), min=0.0)


def mel_spectrogram(wave):
    """torchaudio.transforms.MelSpectrogram(**reference args)(wave): [..., L] -> [..., 80, 1 + L // 300]."""
    m = MEL
    spec = torch.stft(wave, m["n_fft"], m["hop_length"], m["win_length"], torch.hann_window(m["win_length"]),
                      center=True, pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    power = spec.abs().pow(2.0)
    fb = melscale_fbanks(m["n_fft"] // 2 + 1, 0.0, m["sample_rate"] / 2, m["n_mels"], m["sample_rate"])
    return torch.matmul(power.transpose(-1, -2), fb).transpose(-1, -2)


def wave_preprocess(wave):
    """reference inference.py:43-49 (Preprocess.wave_preprocess): np [L] -> [1, 80, F] log-mel."""
    x = torch.from_numpy(np.asarray(wave)).float()
    mel = mel_spectrogram(x)
    return (torch.log(1e-5 + mel.unsqueeze(0)) - MEL["mean"]) / MEL["std"]


def get_style(audio, sd, sr=24000, split_dur=3, prefix=""):
    """reference inference.py:195-217 (StyleTTS2.get_styles, after the optional denoise): the style
    vector of a reference clip, averaged over split_dur-second chunks when the clip is >= 4 s."""
    audio = np.asarray(audio, dtype=np.float32)
    enc = lambda a: style_encoder(wave_preprocess(a).unsqueeze(1), sd, prefix)  # noqa: E731
    if split_dur > 0 and len(audio) / sr >= 4:
        jump = sr * split_dur
        total = len(audio)
        ref = enc(audio[0:jump])
        count = 1
        for i in range(jump, total, jump):
            if i + jump >= total:
                if (total - i) / sr >= 1:
                    ref = ref + enc(audio[i:total])
                    count += 1
                continue
            ref = ref + enc(audio[i:i + jump])
            count += 1
        return ref / count
    return enc(audio)


# ----------------------------------------------------------------------------------
# Duration / text path: TextEncoder, DurationEncoder,
# ProsodyPredictor.forward.  Stock torch-CPU ops in the reference's op order.
# ----------------------------------------------------------------------------------

def bilstm(x, sd, p, lengths=None):
    """nn.LSTM(bidirectional, batch_first) `p` on x [B, T, C]; with `lengths`, the reference's
    pack_padded_sequence -> LSTM -> pad_packed_sequence -> zero pad to T (models.py:267-285,
    510-523, 420-430)."""
    H = _t(sd, p + "weight_hh_l0").shape[1]
    C = _t(sd, p + "weight_ih_l0").shape[1]
    lstm = torch.nn.LSTM(C, H, 1, batch_first=True, bidirectional=True)
    lstm.load_state_dict({k[len(p):]: _t(sd, k) for k in sd if k.startswith(p) and "_l0" in k})
    with torch.no_grad():
        if lengths is None:
            y, _ = lstm(x)
            return y
        ln = torch.as_tensor(lengths).cpu()
        pk = torch.nn.utils.rnn.pack_padded_sequence(x, ln, batch_first=True, enforce_sorted=False)
        y, _ = lstm(pk)
        y, _ = torch.nn.utils.rnn.pad_packed_sequence(y, batch_first=True)
    out = torch.zeros(x.shape[0], x.shape[1], y.shape[-1])
    out[:, :y.shape[1]] = y
    return out


def length_to_mask(lengths, T=None):
    """reference models.py:463-466 / inference.py:58-62: True where t >= length."""
    ln = torch.as_tensor(lengths)
    T = int(ln.max()) if T is None else T
    return torch.arange(T).unsqueeze(0).expand(ln.shape[0], -1) + 1 > ln.unsqueeze(1)


def text_encoder(tokens, lengths, sd, prefix="", depth=3, slope=0.2):
    """reference models.py:256-285 (TextEncoder.forward, eval): -> [B, C, T]."""
    tokens = torch.as_tensor(tokens)
    m = length_to_mask(lengths, tokens.shape[1]).unsqueeze(1)
    x = F.embedding(tokens, _t(sd, prefix + "embedding.weight")).transpose(1, 2)
    x = x.masked_fill(m, 0.0)
    for i in range(depth):
        p = f"{prefix}cnn.{i}."
        w = wn(sd, p + "0")
        x = F.conv1d(x, w, _t(sd, p + "0.bias"), padding=(w.shape[-1] - 1) // 2)
        C = x.shape[1]
        x = F.layer_norm(x.transpose(1, -1), (C,), _t(sd, p + "1.gamma"), _t(sd, p + "1.beta"), 1e-5).transpose(1, -1)
        x = F.leaky_relu(x, slope)
        x = x.masked_fill(m, 0.0)
    x = bilstm(x.transpose(1, 2), sd, prefix + "lstm.", lengths).transpose(1, 2)
    return x.masked_fill(m, 0.0)


def ada_layer_norm(x, s, sd, p, eps=1e-5):
    """reference models.py:383-392 on x [B, T, C]."""
    h = F.linear(s, _t(sd, p + "fc.weight"), _t(sd, p + "fc.bias"))
    C = x.shape[-1]
    gamma, beta = h[:, :C].unsqueeze(1), h[:, C:].unsqueeze(1)
    return (1 + gamma) * F.layer_norm(x, (C,), eps=eps) + beta


def duration_encoder(x, style, lengths, sd, prefix="", nlayers=3):
    """reference models.py:497-523 (DurationEncoder.forward, eval): x [B, C, T] -> [B, T, C + sty]."""
    B, C, T = x.shape
    m = length_to_mask(lengths, T).unsqueeze(-1)  # [B, T, 1]
    s = style.unsqueeze(1).expand(B, T, style.shape[-1])
    h = torch.cat([x.transpose(1, 2), s], -1).masked_fill(m, 0.0)
    for i in range(nlayers):
        h = bilstm(h, sd, f"{prefix}lstms.{2 * i}.", lengths)
        h = ada_layer_norm(h, style, sd, f"{prefix}lstms.{2 * i + 1}.")
        h = torch.cat([h, s], -1).masked_fill(m, 0.0)
    return h


def predictor_forward(texts, style, lengths, alignment, sd, prefix=""):
    """reference models.py:417-446 (ProsodyPredictor.forward, eval) -> (duration, en)."""
    d = duration_encoder(texts, style, lengths, sd, prefix + "text_encoder.")
    x = bilstm(d, sd, prefix + "lstm.", lengths)
    duration = F.linear(x, _t(sd, prefix + "duration_proj.linear_layer.weight"),
                        _t(sd, prefix + "duration_proj.linear_layer.bias"))
    en = d.transpose(-1, -2) @ alignment
    return duration.squeeze(-1), en


def replace_outliers_zscore(x, threshold=3.0, factor=0.95):
    """reference inference.py:134-148."""
    mean, std = x.mean(), x.std()
    z = (x - mean) / std
    mask = torch.abs(z) > threshold
    rep = mean + torch.sign(x - mean) * (threshold * std * factor)
    out = x.clone()
    out[mask] = rep[mask]
    return out


def durations(logits, z, mix=0.1, prev_mean=0.0, speed=1.0):
    """reference inference.py:247-258 for one utterance: logits [1, T, max_dur], z [1, T] = the
    standard-normal draw of dur_stats (normal_(mean, std) = mean + std * z) -> (duration, pred_dur)."""
    speed = min(max(speed, 0.0001), 2)
    duration = torch.sigmoid(logits).sum(axis=-1)
    mu = prev_mean if prev_mean != 0 else duration.mean()
    dur_stats = mu + duration.std() * z
    duration = duration * (1 - mix) + dur_stats * mix
    duration[:, 1:-2] = replace_outliers_zscore(duration[:, 1:-2])
    duration = duration / speed
    pred_dur = torch.round(duration.squeeze()).clamp(min=1)
    return duration, pred_dur


def alignment_matrix(pred_dur):
    """reference inference.py:259-263."""
    aln = torch.zeros(pred_dur.shape[0], int(pred_dur.sum()))
    c = 0
    for i in range(aln.shape[0]):
        aln[i, c:c + int(pred_dur[i])] = 1
        c += int(pred_dur[i])
    return aln.unsqueeze(0)


def inference_chain(tokens, s, te_sd, pp_sd, dec_sd, dec_cfg, z, noise_fn, mix=0.1, prev_mean=0.0, speed=1.0):
    """reference inference.py:225-272 (StyleTTS2.__inference) from the cleaner's token ids on, with the
    HiFi-GAN decoder: -> (audio [600 F], duration.mean(), pred_dur).  noise_fn(F) -> [1, 600F, 9]."""
    ids = [0] + [int(i) for i in tokens] + [0]
    tok = torch.tensor(ids).unsqueeze(0)
    ln = torch.tensor([len(ids)])
    t_en = text_encoder(tok, ln, te_sd)
    d = duration_encoder(t_en, s, ln, pp_sd, "text_encoder.")
    x = bilstm(d, pp_sd, "lstm.")
    logits = F.linear(x, _t(pp_sd, "duration_proj.linear_layer.weight"), _t(pp_sd, "duration_proj.linear_layer.bias"))
    duration, pred = durations(logits, z, mix, prev_mean, speed)
    aln = alignment_matrix(pred)
    en = d.transpose(-1, -2) @ aln
    F0, N = f0ntrain(en, s, pp_sd)
    asr = t_en @ aln
    out = decoder_hifigan(asr, F0, N, s, dec_sd, dec_cfg, noise_fn(aln.shape[-1]))
    return out.squeeze(), duration.mean(), pred


def generate(sentences, s, te_sd, pp_sd, dec_sd, dec_cfg, zs, noise_fns, stabilize=True, speed=1.0):
    """reference inference.py:303-319 (StyleTTS2.generate) over per-sentence token-id lists: each
    sentence through inference_chain with t = 0.2 (stabilize) or 0 and prev_d_mean chained, its
    audio trimmed by 4000 samples at both ends, concatenated, padded with 4000 zeros at both ends."""
    smooth = 0.2 if stabilize else 0.0
    prev = 0.0
    wavs = []
    for toks, z, nf in zip(sentences, zs, noise_fns):
        wav, prev, _ = inference_chain(toks, s, te_sd, pp_sd, dec_sd, dec_cfg, z, nf, mix=smooth,
                                       prev_mean=float(prev), speed=speed)
        wavs.append(wav.numpy()[4000:-4000])
    out = np.concatenate(wavs)
    return np.concatenate([np.zeros([4000]), out, np.zeros([4000])], axis=0)


# ----------------------------------------------------------------------- training step (§8(f) rank 3)
MPD_PERIODS = (2, 3, 5, 7, 11)


def discriminator_p(x, sd, prefix, period):
    """DiscriminatorP.forward (Modules/discriminators.py:108-129): x [B, 1, T] -> (score, fmap)."""
    b, c, t = x.shape
    if t % period != 0:  # :112-115 reflect pad on the right
        n_pad = period - (t % period)
        x = F.pad(x, (0, n_pad), "reflect")
        t = t + n_pad
    x = x.view(b, c, t // period, period)
    fmap = []
    for j in range(5):  # :117-120
        p = f"{prefix}.convs.{j}"
        x = F.conv2d(x, wn(sd, p), _t(sd, p + ".bias"), (3 if j < 4 else 1, 1), (2, 0))
        x = F.leaky_relu(x, 0.1)
        fmap.append(x)
    p = f"{prefix}.conv_post"
    x = F.conv2d(x, wn(sd, p), _t(sd, p + ".bias"), 1, (1, 0))  # :121-122
    fmap.append(x)
    return torch.flatten(x, 1, -1), fmap


def mpd(y, y_hat, sd, periods=MPD_PERIODS):
    """MultiPeriodDiscriminator.forward (discriminators.py:143-156)."""
    y_d_rs, y_d_gs, fmap_rs, fmap_gs = [], [], [], []
    for i, p in enumerate(periods):
        r, fr = discriminator_p(y, sd, f"discriminators.{i}", p)
        g, fg = discriminator_p(y_hat, sd, f"discriminators.{i}", p)
        y_d_rs.append(r)
        y_d_gs.append(g)
        fmap_rs.append(fr)
        fmap_gs.append(fg)
    return y_d_rs, y_d_gs, fmap_rs, fmap_gs


# ----------------------------------------------------------------------- Vocos decoder (§8(f) rank 4)
def vocos_alias(sd):
    """Modules/vocos.py builds its weight-norm layers with torch.nn.utils.parametrizations.weight_norm
    (:10): state-dict keys `<p>.parametrizations.weight.original0` (g) / `original1` (v) instead of
    `<p>.weight_g` / `<p>.weight_v`.  Same fold (dim 0), so alias them for wn()."""
    out = dict(sd)
    for k in list(sd):
        for suf, new in ((".parametrizations.weight.original0", ".weight_g"),
                         (".parametrizations.weight.original1", ".weight_v")):
            if k.endswith(suf):
                out[k[: -len(suf)] + new] = sd[k]
    return out


def convnext_block(x, s, sd, p):
    """ConvNeXtBlock.forward (Modules/vocos.py:56-69): depthwise k7 conv, AdaIN1d, Linear ->
    GELU (erf) -> Linear, layer scale gamma, residual."""
    C = x.shape[1]
    r = x
    x = F.conv1d(x, _t(sd, p + ".dwconv.weight"), _t(sd, p + ".dwconv.bias"), 1, 3, 1, C)
    x = adain1d(x, s, sd, p + ".norm")
    x = x.transpose(1, 2)
    x = F.linear(x, _t(sd, p + ".pwconv1.weight"), _t(sd, p + ".pwconv1.bias"))
    x = F.gelu(x)
    x = F.linear(x, _t(sd, p + ".pwconv2.weight"), _t(sd, p + ".pwconv2.bias"))
    x = _t(sd, p + ".gamma") * x
    return r + x.transpose(1, 2)


def vocos_istft(spec, window, n_fft, hop):
    """ISTFT.forward, padding 'same' (Modules/vocos.py:190-232): irfft, window, overlap-add by
    fold, divide by the folded squared-window envelope, trim (win - hop) / 2 each side."""
    pad = (n_fft - hop) // 2
    B, N, T = spec.shape
    ifft = torch.fft.irfft(spec, n_fft, dim=1, norm="backward") * window[None, :, None]
    out_size = (T - 1) * hop + n_fft
    y = F.fold(ifft, output_size=(1, out_size), kernel_size=(1, n_fft), stride=(1, hop))[:, 0, 0, pad:-pad]
    wsq = window.square().expand(1, T, -1).transpose(1, 2)
    env = F.fold(wsq, output_size=(1, out_size), kernel_size=(1, n_fft), stride=(1, hop)).squeeze()[pad:-pad]
    return y / env


def generator_vocos(x, s, sd, cfg, taps=None):
    """Generator.forward (Modules/vocos.py:157-162) + ISTFTHead.forward (:271-296)."""
    for i in range(cfg["num_layers"]):
        x = convnext_block(x, s, sd, f"generator.convnext.{i}")
    x = F.layer_norm(x.transpose(1, 2), (x.shape[1],), _t(sd, "generator.final_layer_norm.weight"),
                     _t(sd, "generator.final_layer_norm.bias"), 1e-6)
    if taps is not None:
        taps["ln"] = x
    x = F.linear(x, _t(sd, "generator.stft.out.weight"), _t(sd, "generator.stft.out.bias")).transpose(1, 2)
    mag, p = x.chunk(2, dim=1)
    mag = torch.clip(torch.exp(mag), max=1e2)
    S = mag * (torch.cos(p) + 1j * torch.sin(p))
    return vocos_istft(S, _t(sd, "generator.stft.istft.window"), cfg["n_fft"], cfg["hop"])


def decoder_vocos(asr, F0_curve, N, s, sd, cfg, taps=None):
    """Decoder.forward (Modules/vocos.py:392-421, eval): the hifigan front-end, the ConvNeXt
    generator, unsqueeze(1)."""
    sd = vocos_alias(sd)
    x = decoder_frontend(asr, F0_curve, N, s, sd)
    if taps is not None:
        taps["frontend"] = x
    return generator_vocos(x, s, sd, cfg, taps).unsqueeze(1)


# ----------------------------------------------------------------------- multi-resolution mel loss (§8(f) rank 3)
MRSTFT = dict(fft_sizes=(1024, 2048, 512), hop_sizes=(120, 240, 50), win_lengths=(600, 1200, 240))


def mel_spectrogram_sr(wave, sample_rate, n_fft, win_length, hop_length, n_mels=128):
    """torchaudio.transforms.MelSpectrogram(sample_rate, n_fft, win_length, hop_length, window_fn=hann)
    at its other defaults (losses.py:43): f_min 0, f_max sr // 2, power 2, center/reflect, HTK, no norm."""
    lead = wave.shape[:-1]  # torchaudio packs the leading dims into one batch dim around torch.stft
    spec = torch.stft(wave.reshape(-1, wave.shape[-1]), n_fft, hop_length, win_length,
                      torch.hann_window(win_length, dtype=wave.dtype),
                      center=True, pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    spec = spec.reshape(lead + spec.shape[-2:])
    power = spec.abs().pow(2.0)
    fb = melscale_fbanks(n_fft // 2 + 1, 0.0, float(sample_rate // 2), n_mels, sample_rate).to(power.dtype)
    return torch.matmul(power.transpose(-1, -2), fb).transpose(-1, -2)


def stft_loss(x, y, fft_size, shift_size, win_length, sample_rate=24000):
    """STFTLoss.forward (losses.py:46-63) + SpectralConvergengeLoss (:18-21)."""
    x_mag = (torch.log(1e-5 + mel_spectrogram_sr(x, sample_rate, fft_size, win_length, shift_size)) + 4) / 4
    y_mag = (torch.log(1e-5 + mel_spectrogram_sr(y, sample_rate, fft_size, win_length, shift_size)) + 4) / 4
    return torch.norm(y_mag - x_mag, p=1) / torch.norm(y_mag, p=1)


def mrstft_loss(x, y, fft_sizes=MRSTFT["fft_sizes"], hop_sizes=MRSTFT["hop_sizes"],
                win_lengths=MRSTFT["win_lengths"]):
    """MultiResolutionSTFTLoss.forward (losses.py:79-94): the mean spectral-convergence loss."""
    sc = 0.0
    for fs, ss, wl in zip(fft_sizes, hop_sizes, win_lengths):
        sc = sc + stft_loss(x, y, fs, ss, wl)
    return sc / len(fft_sizes)


# ----------------------------------------------------------------------- MultiResSpecDiscriminator (§8(f) rank 3)
MSD_RES = ((1024, 120, 600), (2048, 240, 1200), (512, 50, 240))


def spec_discriminator(y, sd, prefix, fft_size, hop, win):
    """SpecDiscriminator.forward (Modules/discriminators.py:47-63): |torch.stft| image [B, 1, frames,
    bins] -> 4 Conv2d (3, 9) [strides (1,1), (1,2) x 3] + LReLU(0.1) -> Conv2d (3, 3) + LReLU -> out."""
    y = y.squeeze(1)
    y = torch.stft(y, fft_size, hop, win, torch.hann_window(win, dtype=y.dtype), return_complex=True)  # stft() :11-27
    y = torch.abs(y).transpose(2, 1).unsqueeze(1)
    fmap = []
    for j in range(5):
        p = f"{prefix}.discriminators.{j}"
        stride, pad = ((1, 2) if 1 <= j <= 3 else (1, 1)), ((1, 4) if j < 4 else (1, 1))
        y = F.leaky_relu(F.conv2d(y, wn(sd, p), _t(sd, p + ".bias"), stride, pad), 0.1)
        fmap.append(y)
    y = F.conv2d(y, wn(sd, f"{prefix}.out"), _t(sd, f"{prefix}.out.bias"), 1, 1)
    fmap.append(y)
    return torch.flatten(y, 1, -1), fmap


def msd(y, y_hat, sd, res=MSD_RES):
    """MultiResSpecDiscriminator.forward (discriminators.py:80-94)."""
    y_d_rs, y_d_gs, fmap_rs, fmap_gs = [], [], [], []
    for i, (f, h, w) in enumerate(res):
        r, fr = spec_discriminator(y, sd, f"discriminators.{i}", f, h, w)
        g, fg = spec_discriminator(y_hat, sd, f"discriminators.{i}", f, h, w)
        y_d_rs.append(r)
        y_d_gs.append(g)
        fmap_rs.append(fr)
        fmap_gs.append(fg)
    return y_d_rs, y_d_gs, fmap_rs, fmap_gs


def gan_losses(y_d_rs, y_d_gs, fmap_rs, fmap_gs):
    """losses.py:97-128: feature_loss, generator_loss(.)[0], discriminator_loss(.)[0]."""
    fm = sum(torch.mean(torch.abs(rl - gl)) for dr, dg in zip(fmap_rs, fmap_gs) for rl, gl in zip(dr, dg)) * 2
    gen = sum(torch.mean((1 - dg) ** 2) for dg in y_d_gs)
    disc = sum(torch.mean((1 - dr) ** 2) + torch.mean(dg ** 2) for dr, dg in zip(y_d_rs, y_d_gs))
    return fm, gen, disc


# ----------------------------------------------------------------------- the assembled training step (config 5)
TAU = 0.04


def discriminator_tprls_loss(disc_real_outputs, disc_generated_outputs):
    """losses.py:131-138 discriminator_TPRLS_loss."""
    loss = 0
    for dr, dg in zip(disc_real_outputs, disc_generated_outputs):
        m_DG = torch.median((dr - dg))
        L_rel = torch.mean((((dr - dg) - m_DG) ** 2)[dr < dg + m_DG])
        loss += TAU - F.relu(TAU - L_rel)
    return loss


def generator_tprls_loss(disc_real_outputs, disc_generated_outputs):
    """losses.py:140-147 generator_TPRLS_loss (its loop names the real outputs dg and the generated dr)."""
    loss = 0
    for dg, dr in zip(disc_real_outputs, disc_generated_outputs):
        m_DG = torch.median((dr - dg))
        L_rel = torch.mean((((dr - dg) - m_DG) ** 2)[dr < dg + m_DG])
        loss += TAU - F.relu(TAU - L_rel)
    return loss


def feature_loss(fmap_r, fmap_g):
    """losses.py:97-103."""
    loss = 0
    for dr, dg in zip(fmap_r, fmap_g):
        for rl, gl in zip(dr, dg):
            loss += torch.mean(torch.abs(rl - gl))
    return loss * 2


def generator_loss(disc_outputs):
    """losses.py:120-128 (the loss only)."""
    loss = 0
    for dg in disc_outputs:
        loss += torch.mean((1 - dg) ** 2)
    return loss


def discriminator_loss(disc_real_outputs, disc_generated_outputs):
    """losses.py:106-117 (the loss only)."""
    loss = 0
    for dr, dg in zip(disc_real_outputs, disc_generated_outputs):
        loss += torch.mean((1 - dr) ** 2) + torch.mean(dg ** 2)
    return loss


def generator_loss_all(y, y_hat, mpd_sd, msd_sd):
    """GeneratorLoss.forward (losses.py:156-168)."""
    y_df_hat_r, y_df_hat_g, fmap_f_r, fmap_f_g = mpd(y, y_hat, mpd_sd)
    y_ds_hat_r, y_ds_hat_g, fmap_s_r, fmap_s_g = msd(y, y_hat, msd_sd)
    loss_fm_f = feature_loss(fmap_f_r, fmap_f_g)
    loss_fm_s = feature_loss(fmap_s_r, fmap_s_g)
    loss_gen_f = generator_loss(y_df_hat_g)
    loss_gen_s = generator_loss(y_ds_hat_g)
    loss_rel = generator_tprls_loss(y_df_hat_r, y_df_hat_g) + generator_tprls_loss(y_ds_hat_r, y_ds_hat_g)
    return (loss_gen_s + loss_gen_f + loss_fm_s + loss_fm_f + loss_rel).mean()


def discriminator_loss_all(y, y_hat, mpd_sd, msd_sd):
    """DiscriminatorLoss.forward (losses.py:177-190)."""
    y_df_hat_r, y_df_hat_g, _, _ = mpd(y, y_hat, mpd_sd)
    loss_disc_f = discriminator_loss(y_df_hat_r, y_df_hat_g)
    y_ds_hat_r, y_ds_hat_g, _, _ = msd(y, y_hat, msd_sd)
    loss_disc_s = discriminator_loss(y_ds_hat_r, y_ds_hat_g)
    loss_rel = discriminator_tprls_loss(y_df_hat_r, y_df_hat_g) + discriminator_tprls_loss(y_ds_hat_r, y_ds_hat_g)
    return (loss_disc_s + loss_disc_f + loss_rel).mean()


def adamw_update(p, g, m, v, step, lr, betas=(0.0, 0.99), eps=1e-9, weight_decay=1e-4):
    """torch.optim.AdamW's single-tensor update (torch/optim/adam.py _single_tensor_adam with decoupled
    weight decay, amsgrad off), as optimizers.py:65-73 builds it; in place on p, m, v (fp32 tensors);
    `step` counts this update (1 first)."""
    beta1, beta2 = betas
    p.mul_(1 - lr * weight_decay)
    m.lerp_(g, 1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bias_correction1 = 1 - beta1 ** step
    bias_correction2 = 1 - beta2 ** step
    denom = (v.sqrt() / (bias_correction2 ** 0.5)).add_(eps)
    p.addcdiv_(m, denom, value=-(lr / bias_correction1))


def train_step(dec_sd, mpd_sd, msd_sd, cfg, asr, F0_curve, N, s, wav, noise, lr_dec=1e-5, lr_disc=1e-4,
               lambda_mel=5.0, lambda_gen=1.0, smooth=None):
    """train.py:267-327 restricted to the decoder and the discriminators (BASELINE config 5): the decoder
    forward (eval, as train.py:190 leaves it, or the train-mode smoothing), then
      d_loss = DiscriminatorLoss(wav, y_rec.detach()); backward; AdamW on the MPD and MSD   (:272-276)
      g_loss = lambda_mel MultiResolutionSTFTLoss(y_rec, wav) + lambda_gen GeneratorLoss(wav, y_rec);
      backward; AdamW on the decoder                                                        (:278-325)
    Every state dict is a {name: fp32 tensor}; parameters are updated in place (new leaves), so the
    caller passes copies.  Returns (y_rec, losses dict, grads dict {"dec" / "mpd" / "msd" / "inputs": {...}})."""
    leaf = lambda sd: {k: v.detach().clone().requires_grad_(True) for k, v in sd.items()}  # noqa: E731
    dsd, psd, ssd = leaf(dec_sd), leaf(mpd_sd), leaf(msd_sd)
    ins = {k: v.detach().clone().requires_grad_(True) for k, v in
           (("asr", asr), ("F0_curve", F0_curve), ("N", N), ("s", s))}
    y_rec = decoder_hifigan(ins["asr"], ins["F0_curve"], ins["N"], ins["s"], dsd, cfg, noise, smooth=smooth)
    d_loss = discriminator_loss_all(wav, y_rec.detach(), psd, ssd)
    d_loss.backward()
    grads = {"mpd": {k: v.grad for k, v in psd.items()}, "msd": {k: v.grad for k, v in ssd.items()}}
    with torch.no_grad():
        for sd_ in (psd, ssd):
            for k, v in sd_.items():
                adamw_update(v, v.grad, torch.zeros_like(v), torch.zeros_like(v), 1, lr_disc)
                v.grad = None
    loss_mel = mrstft_loss(y_rec, wav)
    loss_gen_all = generator_loss_all(wav, y_rec, psd, ssd)
    g_loss = lambda_mel * loss_mel + lambda_gen * loss_gen_all
    g_loss.backward()
    grads["dec"] = {k: v.grad for k, v in dsd.items()}
    grads["inputs"] = {k: v.grad for k, v in ins.items()}
    with torch.no_grad():
        for k, v in dsd.items():
            if v.grad is not None:
                adamw_update(v, v.grad, torch.zeros_like(v), torch.zeros_like(v), 1, lr_dec)
    losses = {"d_loss": d_loss.item(), "loss_mel": loss_mel.item(), "loss_gen_all": loss_gen_all.item(),
              "g_loss": g_loss.item()}
    params = {"dec": {k: v.detach() for k, v in dsd.items()}, "mpd": {k: v.detach() for k, v in psd.items()},
              "msd": {k: v.detach() for k, v in ssd.items()}}
    return y_rec.detach(), losses, grads, params
