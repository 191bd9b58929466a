"""Drop-in style front-end of the reference's inference.py: `Preprocess.wave_preprocess`
(inference.py:43-49) and the chunked style averaging of `StyleTTS2.get_styles`
(inference.py:195-217), with the log-mel computed by the HIP kernel behind
`stts_wave_preprocess` (include/stts2.h) and the style by the HIP StyleEncoder.

`Synthesizer.inference` is StyleTTS2.__inference (inference.py:219-272) from the token ids on:
text encoder, duration path, durations -> alignment, F0Ntrain and the decoder, all on the HIP
device with one host read (the alignment width, as the reference's `int(pred_dur.sum())`).

Out of scope here: text normalisation and phonemisation, audio loading
(librosa) and the optional noisereduce denoise step -- `get_style` takes the loaded, already
denoised waveform, `Synthesizer.inference` the token ids of `TextCleaner`.
"""
from __future__ import annotations

import numpy as np
import torch

from .engine import wave_preprocess_batch
from .prosody import durations, expand_frames, linear_frames


class Preprocess:
    """reference inference.py:15-56 (the wave half; the text half is out of scope)."""

    def wave_preprocess(self, wave):
        """wave: 1-D float array / tensor of L > 1024 samples -> [1, 80, 1 + L // 300] log-mel on
        the HIP device (the reference returns it on the CPU and the caller moves it `.to(device)`)."""
        w = torch.as_tensor(np.asarray(wave, dtype=np.float32)) if not isinstance(wave, torch.Tensor) else wave
        if w.dim() != 1:
            raise ValueError(f"wave must be 1-D, got {tuple(w.shape)}")
        return wave_preprocess_batch(w.reshape(1, -1))


def get_style(style_encoder, audio, sr=24000, split_dur=3, dtype="fp32"):
    """Style vector [1, style_dim] of a reference clip, as StyleTTS2.get_styles computes it
    (inference.py:195-217): the clip is cut into split_dur-second chunks when it is >= 4 s long, a
    trailing chunk shorter than split_dur counts only if it is >= 1 s, and the chunk styles are
    averaged.  All full chunks go through the mel and StyleEncoder kernels as one batch."""
    audio = np.asarray(audio, dtype=np.float32)
    if audio.ndim != 1:
        raise ValueError(f"audio must be 1-D, got shape {audio.shape}")

    def enc(chunks):
        mel = wave_preprocess_batch(torch.from_numpy(np.stack(chunks)))
        return style_encoder(mel.unsqueeze(1), dtype=dtype)

    if split_dur > 0 and len(audio) / sr >= 4:
        jump = int(sr * split_dur)
        total = len(audio)
        full = [audio[0:jump]]
        tail = None
        for i in range(jump, total, jump):
            if i + jump >= total:
                if (total - i) / sr >= 1:
                    tail = audio[i:total]
                continue
            full.append(audio[i:i + jump])
        styles = enc(full)
        ref = styles.sum(0, keepdim=True)
        count = len(full)
        if tail is not None:
            ref = ref + enc([tail])
            count += 1
        return ref / count
    return enc([audio])


class Synthesizer:
    """The model half of reference inference.py StyleTTS2 (:64-272) over drop-in modules:
    text_encoder (models.TextEncoder), predictor (models.ProsodyPredictor), decoder
    (hifigan / istftnet Decoder), all on the HIP device."""

    def __init__(self, text_encoder, predictor, decoder, decoder_dtype="fp32"):
        self.text_encoder, self.predictor, self.decoder = text_encoder, predictor, decoder
        self.decoder_dtype = decoder_dtype

    def alignment(self, tokens, ref_s, speed=1, prev_d_mean=0, t=0.1, z=None):
        """inference.py:225-263: token ids (TextCleaner output, without the 0 pads) -> intermediate
        tensors {t_en [1,C,T], d [1,T,C+S], logits, dur, pred [1,T], frames F, dur_mean}.
        `z` [T] = the standard-normal draw behind dur_stats (:249-252); None draws it on the device."""
        dev = self.predictor.F0_proj.weight.device
        speed = min(max(speed, 0.0001), 2)
        ids = [0] + [int(i) for i in tokens] + [0]  # tokens.insert(0, 0); tokens.append(0)  (:228-229)
        tok = torch.tensor(ids, dtype=torch.int64).unsqueeze(0)  # host: ids checked there, no device sync
        T = tok.shape[1]
        s = torch.as_tensor(ref_s).to(dev, torch.float32).reshape(1, -1)
        with torch.no_grad():
            t_en = self.text_encoder(tok, None)
            d = self.predictor.text_encoder(t_en, s, None)
            x, _ = self.predictor.lstm(d)
            lin = self.predictor.duration_proj.linear_layer
            logits = linear_frames(x, lin.weight.detach(), lin.bias.detach())
            if z is None:
                z = torch.randn(1, T, device=dev)
            z = torch.as_tensor(z).to(dev, torch.float32).reshape(1, T)
            dur, pred, total, dmean = durations(logits, None, z, mix=t, prev_mean=prev_d_mean, speed=speed)
        return {"t_en": t_en, "d": d, "s": s, "logits": logits, "dur": dur, "pred": pred,
                "frames": int(total[0].item()), "dur_mean": dmean[0]}

    def inference(self, tokens, ref_s, speed=1, prev_d_mean=0, t=0.1, z=None, noise=None, seed=0):
        """-> (audio [600 F] float32 on the device, duration.mean()) as inference.py:272 returns
        (the reference moves the audio to a numpy array)."""
        a = self.alignment(tokens, ref_s, speed, prev_d_mean, t, z)
        F, s = a["frames"], a["s"]
        with torch.no_grad():
            en = expand_frames(a["d"], a["pred"], F)  # d^T @ aln          (:266)
            F0, N = self.predictor.F0Ntrain(en, s)  # (:267)
            t_en = a["t_en"]
            asr = expand_frames(t_en.transpose(1, 2), a["pred"], F)  # t_en @ aln  (:268)
            out = self.decoder(asr, F0, N, s, noise=noise, seed=seed, dtype=self.decoder_dtype)
        return out.squeeze(), a["dur_mean"]


def symbol_table(config):
    """inference.py:70-86: the token table from config['symbol'] -> ({symbol: id}, n_token)."""
    sym = config["symbol"]
    symbols = (list(sym["pad"]) + list(sym["punctuation"]) + list(sym["letters"]) + list(sym["letters_ipa"])
               + list(sym["extend"]))
    table = {s: i for i, s in enumerate(symbols)}
    return table, len(table) + 1


def build_models(config):
    """inference.py:88-122 with the drop-in classes: the parsed config.yaml (a dict) ->
    {'decoder', 'predictor', 'text_encoder', 'style_encoder'} modules (parameters on the CPU,
    move them with .to('cuda'))."""
    from . import hifigan, istftnet
    from .models import ProsodyPredictor, StyleEncoder, TextEncoder
    args = config["model_params"]
    _, n_token = symbol_table(config)
    dec = args["decoder"]
    common = dict(dim_in=args["hidden_dim"], style_dim=args["style_dim"], dim_out=args["n_mels"],
                  resblock_kernel_sizes=dec["resblock_kernel_sizes"], upsample_rates=dec["upsample_rates"],
                  upsample_initial_channel=dec["upsample_initial_channel"],
                  resblock_dilation_sizes=dec["resblock_dilation_sizes"],
                  upsample_kernel_sizes=dec["upsample_kernel_sizes"])
    if dec["type"] == "istftnet":
        decoder = istftnet.Decoder(**common, gen_istft_n_fft=dec["gen_istft_n_fft"],
                                   gen_istft_hop_size=dec["gen_istft_hop_size"])
    elif dec["type"] == "hifigan":
        decoder = hifigan.Decoder(**common)
    else:  # the reference also accepts 'vocos' (Modules/vocos.py): out of scope here
        raise NotImplementedError(f"decoder type {dec['type']!r}: only hifigan / istftnet run on the HIP path")
    return {
        "decoder": decoder,
        "predictor": ProsodyPredictor(style_dim=args["style_dim"], d_hid=args["hidden_dim"], nlayers=args["n_layer"],
                                      max_dur=args["max_dur"], dropout=args["dropout"]),
        "text_encoder": TextEncoder(channels=args["hidden_dim"], kernel_size=5, depth=args["n_layer"],
                                    n_symbols=n_token),
        "style_encoder": StyleEncoder(dim_in=args["dim_in"], style_dim=args["style_dim"],
                                      max_conv_dim=args["hidden_dim"]),
    }


def load_models(model, models_path):
    """inference.py:150-174 (StyleTTS2.__load_models): checkpoint['net'][key] -> model[key], retrying
    with the 7-character 'module.' prefix stripped and strict=False as the reference does.  Loaded with
    torch.load(weights_only=True): a checkpoint that needs unpickling of code is refused.
    Returns {key: parameter count}."""
    from collections import OrderedDict
    params = torch.load(models_path, map_location="cpu", weights_only=True)["net"]
    params = {k: v for k, v in params.items() if k in model}
    counts = {}
    for key in model:
        try:
            model[key].load_state_dict(params[key])
        except Exception:
            sd = OrderedDict((k[7:], v) for k, v in params[key].items())
            model[key].load_state_dict(sd, strict=False)
        counts[key] = sum(p.numel() for p in model[key].parameters())
    return counts
