"""Drop-in driver pieces of the reference's inference.py on the HIP path.

* `Preprocess.wave_preprocess` (inference.py:43-49) -> the HIP log-mel (`stts_wave_preprocess`);
  `Preprocess.text_preprocess` (:17-42, 50-55), pure string handling, restated.
* `get_style`: the 20-s cap and chunked style averaging of `__compute_style` (:176-222) over the
  HIP StyleEncoder.
* `Synthesizer.inference` = `StyleTTS2.__inference` (:224-272) from the token ids on: text
  encoder, duration path, durations -> alignment, F0Ntrain and the decoder, all on the HIP device
  with one host read (the alignment width and duration mean, as the reference's
  `int(pred_dur.sum())` and `duration.mean()`).
* `Synthesizer.generate` = `StyleTTS2.generate` (:303-319): sentence split, `prev_d_mean`
  chaining, the [4000:-4000] trim of each sentence, concatenation and 4000-sample padding.

Out of scope here: phonemisation, nltk's `word_tokenize` (absent in this image;
the reference downloads its data at import, inference.py:12) -- `generate` takes the caller's
tokenizer, by default `TextCleaner` over whitespace-normalised text -- audio loading (librosa)
and the optional noisereduce denoise step (`get_style` takes the loaded, already denoised waveform).
"""
from __future__ import annotations

import numpy as np
import torch

import re

from .engine import wave_preprocess_batch
from .prosody import check_pending, durations, expand_frames, linear_frames

MAX_REF_SAMPLES = 24000 * 20  # inference.py:180: at most 20 s of reference audio
TRIM = 4000                   # inference.py:314, 318: per-sentence trim and final padding


class TextCleaner:
    """meldataset.py:21-35: characters -> symbol ids; unknown characters are skipped."""

    def __init__(self, symbol_dict, debug=False):
        self.word_index_dictionary = symbol_dict
        self.debug = debug

    def __call__(self, text):
        ids = []
        for ch in text:
            i = self.word_index_dictionary.get(ch)
            if i is None:
                if self.debug:
                    print("WARNING UNKNOWN IPA CHARACTERS/LETTERS: ", ch)
                continue
            ids.append(i)
        return ids


class Preprocess:
    """reference inference.py:16-59."""

    _PUNCT = re.compile("[" + "".join(re.escape(p) for p in
                                      ["，", "、", "،", ";", "(", "．", "。", "…", "!", "–", ":", "?"]) + "]")

    def text_normalize(self, text):
        """inference.py:17-25: comma/period-like punctuation -> '.', whitespace runs -> one space."""
        text = self._PUNCT.sub(".", text)
        return re.sub(r"\s+", " ", text).strip()

    @staticmethod
    def merge_fragments(texts, n):
        """inference.py:26-42: merge fragments until each has >= n words; a short last one joins
        the one before it."""
        merged = []
        i = 0
        while i < len(texts):
            fragment = texts[i]
            j = i + 1
            while len(fragment.split()) < n and j < len(texts):
                fragment += ", " + texts[j]
                j += 1
            merged.append(fragment)
            i = j
        if len(merged[-1].split()) < n and len(merged) > 1:
            merged[-2] = merged[-2] + ", " + merged[-1]
            del merged[-1]
        return merged

    def text_preprocess(self, text, n_merge=12):
        """inference.py:50-55: split into sentences on '.', drop empty ones, merge short ones."""
        parts = [p.strip() for p in self.text_normalize(text).split(".")]
        parts = [p for p in parts if p != ""]
        if not parts:
            return []
        return self.merge_fragments(parts, n_merge)

    def wave_preprocess(self, wave):
        """wave: 1-D float array / tensor of L > 1024 samples -> [1, 80, 1 + L // 300] log-mel on
        the HIP device (the reference returns it on the CPU and the caller moves it `.to(device)`)."""
        w = torch.as_tensor(np.asarray(wave, dtype=np.float32)) if not isinstance(wave, torch.Tensor) else wave
        if w.dim() != 1:
            raise ValueError(f"wave must be 1-D, got {tuple(w.shape)}")
        return wave_preprocess_batch(w.reshape(1, -1))


def get_style(style_encoder, audio, sr=24000, split_dur=3, dtype="fp32"):
    """Style vector [1, style_dim] of a reference clip, as StyleTTS2.get_styles computes it
    (inference.py:176-222): the clip is capped at 20 s (:180, 187-188), then cut into
    split_dur-second chunks when it is >= 4 s long, a trailing chunk shorter than split_dur counts
    only if it is >= 1 s, and the chunk styles are averaged.  All full chunks go through the mel
    and StyleEncoder kernels as one batch."""
    audio = np.asarray(audio, dtype=np.float32)
    if audio.ndim != 1:
        raise ValueError(f"audio must be 1-D, got shape {audio.shape}")
    if split_dur != 0:
        split_dur = max(int(split_dur), 1)  # :179
    if len(audio) > MAX_REF_SAMPLES:
        audio = audio[:MAX_REF_SAMPLES]

    def enc(chunks):
        with torch.no_grad():  # as get_styles (inference.py:194)
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

    def __init__(self, text_encoder, predictor, decoder, decoder_dtype="fp32", tokenize=None):
        self.text_encoder, self.predictor, self.decoder = text_encoder, predictor, decoder
        self.decoder_dtype = decoder_dtype
        self.tokenize = tokenize  # text -> token ids (the reference: TextCleaner(' '.join(word_tokenize(text))))
        self.preprocess = Preprocess()

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
                # the reference's draw: torch.empty(duration.shape).normal_(mean, std) on the CPU
                # generator (:249-251) = mean + std * z with z from the same generator
                z = torch.empty(1, T).normal_()
            z = torch.as_tensor(z).to(dev, torch.float32).reshape(1, T)
            dur, pred, total, dmean = durations(logits, None, z, mix=t, prev_mean=float(prev_d_mean), speed=speed)
            host = torch.stack([total[0].to(torch.float32), dmean[0]]).cpu()  # the one host read
        check_pending()  # BiLSTM error words of this sentence (the stream has passed them)
        return {"t_en": t_en, "d": d, "s": s, "logits": logits, "dur": dur, "pred": pred,
                "frames": int(host[0].item()), "dur_mean": float(host[1].item())}

    def inference(self, tokens, ref_s, speed=1, prev_d_mean=0, t=0.1, z=None, noise=None, seed=None):
        """-> (audio [600 F] float32 on the device, duration.mean() as a float) as inference.py:272
        returns (the reference moves the audio to a numpy array).  seed None: the decoder noise is
        keyed by a draw from torch's default generator (Decoder.forward)."""
        a = self.alignment(tokens, ref_s, speed, prev_d_mean, t, z)
        F, s = a["frames"], a["s"]
        with torch.no_grad():
            en = expand_frames(a["d"], a["pred"], F)  # d^T @ aln          (:266)
            F0, N = self.predictor.F0Ntrain(en, s)  # (:267)
            t_en = a["t_en"]
            asr = expand_frames(t_en.transpose(1, 2), a["pred"], F)  # t_en @ aln  (:268)
            out = self.decoder(asr, F0, N, s, noise=noise, seed=seed, dtype=self.decoder_dtype)
        return out.squeeze(), a["dur_mean"]

    def generate(self, phonem, style, stabilize=True, n_merge=16, seed=None, z=None, noise=None):
        """StyleTTS2.generate (inference.py:303-319).  `phonem`: the phoneme text (split into
        sentences by Preprocess.text_preprocess and tokenized by `self.tokenize`), or a list of
        per-sentence token-id lists.  `style`: {'style': [1, style_dim], 'speed': float} as
        get_styles returns it.  -> float32 numpy waveform: each sentence's audio trimmed by 4000
        samples at both ends, concatenated, padded with 4000 zeros at both ends.  `prev_d_mean`
        chains the duration mean from sentence to sentence.  seed: None = the decoder noise of every
        sentence from torch's default generator; an int = sentence i uses seed + i.  Parity hooks:
        z[i] (the dur_stats draw) and noise[i] (a callable F -> [1, 600 F, 9] SineGen draw) per
        sentence."""
        smooth = 0.2 if stabilize else 0.0
        if isinstance(phonem, str):
            if self.tokenize is None:
                raise ValueError("generate(text): construct the Synthesizer with tokenize= (text -> token ids)")
            sentences = [self.tokenize(x) for x in self.preprocess.text_preprocess(phonem, n_merge=n_merge)]
        else:
            sentences = [list(x) for x in phonem]
        prev_d_mean = 0.0
        pieces = []
        for i, toks in enumerate(sentences):
            zi = None if z is None else z[i]
            nfn = None if noise is None else noise[i]
            if nfn is not None:  # the draw's length is the alignment width: known after the durations
                a = self.alignment(toks, style["style"], style.get("speed", 1), prev_d_mean, smooth, zi)
                nz = nfn(a["frames"])
            else:
                nz = None
            wav, prev_d_mean = self.inference(toks, style["style"], speed=style.get("speed", 1), prev_d_mean=prev_d_mean,
                                              t=smooth, z=zi, noise=nz, seed=None if seed is None else seed + i)
            pieces.append(wav[TRIM:-TRIM])  # numpy semantics: empty when the sentence has <= 8000 samples
        dev = pieces[0].device if pieces else torch.device("cpu")
        pad = torch.zeros(TRIM, dtype=torch.float32, device=dev)
        return torch.cat([pad, *pieces, pad]).cpu().numpy()


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
    from . import hifigan, istftnet, vocos
    from .models import ProsodyPredictor, StyleEncoder, TextEncoder
    args = config["model_params"]
    _, n_token = symbol_table(config)
    dec = args["decoder"]
    if dec["type"] not in ("istftnet", "hifigan", "vocos"):  # inference.py:93
        raise AssertionError("Decoder type unknown")
    if dec["type"] == "vocos":  # inference.py:112-118 (no resblock / upsample keys in its config block)
        decoder = vocos.Decoder(dim_in=args["hidden_dim"], style_dim=args["style_dim"], dim_out=args["n_mels"],
                                intermediate_dim=dec["intermediate_dim"], num_layers=dec["num_layers"],
                                gen_istft_n_fft=dec["gen_istft_n_fft"], gen_istft_hop_size=dec["gen_istft_hop_size"])
    common = {} if dec["type"] == "vocos" else dict(dim_in=args["hidden_dim"], style_dim=args["style_dim"], dim_out=args["n_mels"],
                  resblock_kernel_sizes=dec["resblock_kernel_sizes"], upsample_rates=dec["upsample_rates"],
                  upsample_initial_channel=dec["upsample_initial_channel"],
                  resblock_dilation_sizes=dec["resblock_dilation_sizes"],
                  upsample_kernel_sizes=dec["upsample_kernel_sizes"])
    if dec["type"] == "istftnet":
        decoder = istftnet.Decoder(**common, gen_istft_n_fft=dec["gen_istft_n_fft"],
                                   gen_istft_hop_size=dec["gen_istft_hop_size"])
    elif dec["type"] == "hifigan":
        decoder = hifigan.Decoder(**common)
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
