"""Deterministic synthetic tensors (weights, inputs, noise) from a counter hash.

The LibriTTS checkpoint is download-only (reference README.md:7), so every run here
uses formula weights: value = f(parameter name, flat index).  The same formula is
evaluated by the golden-fixture generator (which loads the values into the
reference modules), by the oracle and by bench.py, so the GPU box can regenerate
exactly the tensors the fixtures were made from without shipping 217 MB.

Hash: splitmix64 over (crc32(name) * golden + index); uniform = top 53 bits.
Normal: Box-Muller over two independent streams.
"""
from __future__ import annotations

import zlib

import numpy as np

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _seed(name: str) -> np.uint64:
    return np.uint64(zlib.crc32(name.encode("utf-8")) | (len(name) << 32))


def hash_u01(name: str, n: int) -> np.ndarray:
    """n float64 values in [0, 1) keyed by `name`."""
    with np.errstate(over="ignore"):
        z = np.arange(n, dtype=np.uint64) + _seed(name) * _GOLD
        z = z * _GOLD
        z ^= z >> np.uint64(30)
        z *= _M1
        z ^= z >> np.uint64(27)
        z *= _M2
        z ^= z >> np.uint64(31)
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def dropout_mask(k: int, shape, p: float) -> np.ndarray:
    """The k-th train-mode dropout call's keep mask (1.0 = kept) for a tensor of `shape` in the REFERENCE module's
    layout: element i kept when hash_u01 >= p.  The train-mode text / duration fixtures inject these masks into the
    reference's F.dropout (tests/golden/make_golden_train_text.py) and the HIP path through
    training.set_dropout_masks, so both drop the same elements."""
    n = int(np.prod(shape))
    return (hash_u01(f"dropout:{k}:{tuple(int(v) for v in shape)}", n) >= p).astype(np.float32).reshape(shape)


def uniform(name: str, shape, lo: float = -1.0, hi: float = 1.0) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = hash_u01(name, n)
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def normal(name: str, shape, std: float = 1.0) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u1 = hash_u01(name + "#bm1", n)
    u2 = hash_u01(name + "#bm2", n)
    r = np.sqrt(-2.0 * np.log1p(-u1))  # 1-u1 in (0,1]
    return (std * r * np.cos(2.0 * np.pi * u2)).astype(np.float32).reshape(shape)


# ----------------------------------------------------------------------------------
# weights
# ----------------------------------------------------------------------------------

def _g_target(key: str) -> float:
    """Per-output-channel L2 norm of the folded weight (weight_g) by layer role."""
    if ".ups." in key:
        return 1.0
    if "conv_post" in key:
        return 0.12
    if key.endswith("pool.weight_g"):
        return 1.0
    if "F0_conv" in key or "N_conv" in key:
        return 0.8
    if "conv1x1" in key:
        return 0.9
    if "asr_res" in key:
        return 0.9
    if ".convs2." in key:
        return 0.35
    if ".convs1." in key:
        return 0.6
    return 0.8  # AdainResBlk1d conv1/conv2


def synth_param(key: str, shape) -> np.ndarray:
    """Formula value for one state-dict entry of the decoders / predictor / style encoder."""
    shape = tuple(int(s) for s in shape)
    if key.endswith("weight_v") or key.endswith("parametrizations.weight.original1"):
        return uniform(key, shape, -1.0, 1.0)
    if key.endswith("weight_g") or key.endswith("parametrizations.weight.original0"):
        return (_g_target(key) * uniform(key, shape, 0.8, 1.2)).astype(np.float32)
    if ".alpha" in key or key.startswith("generator.alphas") or ".alphas." in key:
        return uniform(key, shape, 0.6, 1.4)
    if key.endswith("fc.weight"):  # AdaIN1d fc: Linear(style_dim, 2C)
        return uniform(key, shape, -1.0, 1.0) * np.float32(0.5 / np.sqrt(shape[1]))
    if key.endswith("fc.bias"):
        return uniform(key, shape, -0.1, 0.1)
    if "l_linear.weight" in key:
        return uniform(key, shape, -0.6, 0.6)
    if "weight_ih" in key or "weight_hh" in key:  # nn.LSTM
        hidden = shape[0] // 4
        return uniform(key, shape, -1.0, 1.0) * np.float32(1.0 / np.sqrt(hidden))
    if "bias_ih" in key or "bias_hh" in key:
        return uniform(key, shape, -0.1, 0.1)
    if key.endswith("embedding.weight"):  # nn.Embedding default init N(0, 1)
        return normal(key, shape)
    if key.endswith(".weight") and len(shape) >= 2:  # plain conv / linear (no weight norm)
        fan_in = int(np.prod(shape[1:]))
        gain = 1.0
        if "noise_convs" in key:
            gain = 1.5
        elif "_proj" in key:
            gain = 1.0
        return uniform(key, shape, -1.0, 1.0) * np.float32(gain * np.sqrt(3.0 / fan_in))
    if key.endswith("bias"):
        return uniform(key, shape, -0.05, 0.05)
    if ".convnext." in key and key.endswith(".gamma"):  # Vocos ConvNeXt layer scale (init 1/num_layers)
        return uniform(key, shape, 0.1, 0.2)
    if key.endswith("layer_norm.weight"):  # Vocos final LayerNorm
        return uniform(key, shape, 0.8, 1.2)
    if key.endswith(".gamma"):
        return uniform(key, shape, 0.8, 1.2)
    if key.endswith(".beta"):
        return uniform(key, shape, -0.1, 0.1)
    raise KeyError(f"no synthesis rule for {key} {shape}")


def is_fixed_buffer(key: str) -> bool:
    """Deterministic buffers the modules compute themselves (CustomSTFT bases)."""
    return ".stft." in key and not key.endswith((".out.weight", ".out.bias"))  # Vocos ISTFTHead.out is a Linear


def synth_state_dict(named_shapes, prefix: str = "") -> dict:
    """{key: np.float32 array} for every (key, shape) that has a synthesis rule."""
    out = {}
    for k, shp in named_shapes:
        if is_fixed_buffer(k):
            continue
        out[k] = synth_param(prefix + k, shp)
    return out


# ----------------------------------------------------------------------------------
# inputs (SURVEY.md §8(d) config 2/3 distributions)
# ----------------------------------------------------------------------------------

def decoder_inputs(B: int, T: int, utt0: int = 0, tag: str = "in"):
    """asr [B,512,T] ~ N(0,1); F0 [B,2T] ~ U(60,260) with frames [2T/10, 2T/5) unvoiced;
    N [B,2T] ~ N(0,1); s [B,128] ~ N(0,1).  Utterance u of the batch is keyed by the
    GLOBAL utterance id utt0+u so a sharded batch regenerates identical inputs."""
    asr = np.stack([normal(f"{tag}:asr:{utt0 + b}:{T}", (512, T)) for b in range(B)])
    f0 = np.stack([uniform(f"{tag}:f0:{utt0 + b}:{T}", (2 * T,), 60.0, 260.0) for b in range(B)])
    lo, hi = (2 * T) // 10, (2 * T) // 5
    f0[:, lo:hi] = 0.0
    n = np.stack([normal(f"{tag}:n:{utt0 + b}:{T}", (2 * T,)) for b in range(B)])
    s = np.stack([normal(f"{tag}:s:{utt0 + b}", (128,)) for b in range(B)])
    return asr, f0, n, s


def source_noise(B: int, L: int, utt0: int = 0, tag: str = "noise") -> np.ndarray:
    """The reference's randn_like(sine_waves) draw (hifigan.py:213) as a formula: [B, L, 9]."""
    return np.stack([normal(f"{tag}:{utt0 + b}:{L}", (L, 9)) for b in range(B)])


def waves(B, T, seed):
    """Speech-like test waveforms [B, 1, T] fp32: two harmonic tones with an envelope plus formula noise (the
    discriminator / training-step fixtures' signals, tests/golden/make_golden_mpd.py)."""
    t = np.arange(T, dtype=np.float64) / 24000.0
    out = np.zeros((B, 1, T), np.float32)
    for b in range(B):
        f = 110.0 + 37.0 * (b + seed)
        env = 0.5 + 0.4 * np.sin(2 * np.pi * 3.0 * t + b)
        x = env * (0.6 * np.sin(2 * np.pi * f * t) + 0.25 * np.sin(2 * np.pi * 2.3 * f * t + 0.4))
        x = x + 0.05 * normal(f"mpd.wave.{seed}.{b}", (T,)).astype(np.float64)
        out[b, 0] = x.astype(np.float32)
    return out
