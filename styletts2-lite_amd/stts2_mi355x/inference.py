"""Drop-in style front-end of the reference's inference.py: `Preprocess.wave_preprocess`
(inference.py:43-49) and the chunked style averaging of `StyleTTS2.get_styles`
(inference.py:195-217), with the log-mel computed by the HIP kernel behind
`stts_wave_preprocess` (include/stts2.h) and the style by the HIP StyleEncoder.

Out of scope here: text normalisation and phonemisation, audio loading
(librosa) and the optional noisereduce denoise step -- `get_style` takes the loaded, already
denoised waveform.
"""
from __future__ import annotations

import numpy as np
import torch

from .engine import wave_preprocess_batch


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
