"""Drop-in `Modules.vocos.Decoder` (reference Modules/vocos.py:364-421).

Same constructor signature as the reference (inference.py:112-118 / models.py:555-561 build it
from `intermediate_dim`, `num_layers`, `gen_istft_n_fft`, `gen_istft_hop_size`), same sub-module
names and state-dict keys (the front-end's weight-norm layers use
torch.nn.utils.parametrizations.weight_norm there: `<layer>.parametrizations.weight.original0` = g,
`original1` = v; the ISTFT window is the `generator.stft.istft.window` buffer), so a Vocos
checkpoint loads unchanged.  `forward(asr, F0_curve, N, s)` runs the whole decoder as HIP kernels
through the C-ABI (`include/stts2.h`, STTS_KIND_VOCOS, `stts_decoder_fwd`); no PyTorch compute.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .params import AdaIN1d, Linear, _p


class _WNParam(nn.Module):
    """the `parametrizations.weight` entry of a parametrized module: original0 = g, original1 = v."""

    def __init__(self, g_shape, v_shape):
        super().__init__()
        self.original0 = _p(*g_shape)
        self.original1 = _p(*v_shape)


class PWNConv1d(nn.Module):
    """parametrizations.weight_norm(nn.Conv1d(cin, cout, k, ...)) parameter layout."""

    def __init__(self, cin, cout, k, stride=1, padding=0, groups=1, bias=True):
        super().__init__()
        self.cin, self.cout, self.k, self.stride, self.padding, self.groups = cin, cout, k, stride, padding, groups
        if bias:
            self.bias = _p(cout)
        else:
            self.register_parameter("bias", None)
        self.parametrizations = nn.ModuleDict({"weight": _WNParam((cout, 1, 1), (cout, cin // groups, k))})


class PWNConvT1d(nn.Module):
    """parametrizations.weight_norm(nn.ConvTranspose1d(cin, cout, k, stride, ...)): g per input channel."""

    def __init__(self, cin, cout, k, stride, padding=0, output_padding=0, groups=1):
        super().__init__()
        self.cin, self.cout, self.k, self.stride = cin, cout, k, stride
        self.padding, self.output_padding, self.groups = padding, output_padding, groups
        self.bias = _p(cout)
        self.parametrizations = nn.ModuleDict({"weight": _WNParam((cin, 1, 1), (cin, cout // groups, k))})


class AdainResBlk1d(nn.Module):
    """reference vocos.py:307-351 parameter layout (hifigan.py:359-403 with parametrized weight norm)."""

    def __init__(self, dim_in, dim_out, style_dim=64, upsample="none", dropout_p=0.0):
        super().__init__()
        self.dim_in, self.dim_out = dim_in, dim_out
        self.upsample_type = "none" if upsample in ("none", False, None) else "half"
        self.learned_sc = dim_in != dim_out
        self.conv1 = PWNConv1d(dim_in, dim_out, 3, 1, 1)
        self.conv2 = PWNConv1d(dim_out, dim_out, 3, 1, 1)
        self.norm1 = AdaIN1d(style_dim, dim_in)
        self.norm2 = AdaIN1d(style_dim, dim_out)
        if self.learned_sc:
            self.conv1x1 = PWNConv1d(dim_in, dim_out, 1, 1, 0, bias=False)
        if self.upsample_type != "none":
            self.pool = PWNConvT1d(dim_in, dim_in, 3, 2, padding=1, output_padding=1, groups=dim_in)


class ConvNeXtBlock(nn.Module):
    """reference vocos.py:27-69 parameter layout: dwconv (depthwise k7), norm (AdaIN1d), pwconv1,
    pwconv2 (Linear), gamma (layer scale)."""

    def __init__(self, dim, intermediate_dim, layer_scale_init_value, style_dim):
        super().__init__()
        self.dwconv = nn.Module()
        self.dwconv.weight = _p(dim, 1, 7)
        self.dwconv.bias = _p(dim)
        self.norm = AdaIN1d(style_dim, dim)
        self.pwconv1 = Linear(dim, intermediate_dim)
        self.pwconv2 = Linear(intermediate_dim, dim)
        # Generator always passes a positive value (vocos.py:131: `or 1 / num_layers`), so the
        # reference's gamma=None branch (:50-54) never occurs
        self.gamma = nn.Parameter(layer_scale_init_value * torch.ones(dim))


class _ISTFT(nn.Module):
    def __init__(self, n_fft):
        super().__init__()
        self.register_buffer("window", torch.hann_window(n_fft))  # vocos.py:187-188


class ISTFTHead(nn.Module):
    """reference vocos.py:248-269: out = Linear(dim, n_fft + 2), istft.window."""

    def __init__(self, dim, n_fft, hop_length):
        super().__init__()
        self.n_fft, self.hop_length = int(n_fft), int(hop_length)
        self.out = Linear(dim, n_fft + 2)
        self.istft = _ISTFT(n_fft)


class Generator(nn.Module):
    """reference vocos.py:108-162 parameter layout."""

    def __init__(self, input_channels, dim, style_dim, intermediate_dim, num_layers, gen_istft_n_fft,
                 gen_istft_hop_size, layer_scale_init_value=None):
        super().__init__()
        self.input_channels = input_channels
        self.dim, self.intermediate_dim, self.num_layers = int(dim), int(intermediate_dim), int(num_layers)
        self.n_fft, self.hop = int(gen_istft_n_fft), int(gen_istft_hop_size)
        layer_scale_init_value = layer_scale_init_value or 1 / num_layers
        self.convnext = nn.ModuleList([ConvNeXtBlock(dim, intermediate_dim, layer_scale_init_value, style_dim)
                                       for _ in range(num_layers)])
        self.final_layer_norm = nn.LayerNorm(dim, eps=1e-6)
        self.stft = ISTFTHead(dim, gen_istft_n_fft, gen_istft_hop_size)


class Decoder(nn.Module):
    """reference vocos.py:364-421; forward = HIP decoder (eval semantics)."""

    decoder_type = "vocos"

    def __init__(self, dim_in=512, style_dim=64, dim_out=80, intermediate_dim=1536, num_layers=8,
                 gen_istft_n_fft=1024, gen_istft_hop_size=256):
        super().__init__()
        self.dim_in, self.style_dim = int(dim_in), int(style_dim)
        self.decode = nn.ModuleList()
        self.encode = AdainResBlk1d(dim_in + 2, 1024, style_dim)
        self.decode.append(AdainResBlk1d(1024 + 2 + 64, 1024, style_dim))
        self.decode.append(AdainResBlk1d(1024 + 2 + 64, 1024, style_dim))
        self.decode.append(AdainResBlk1d(1024 + 2 + 64, 1024, style_dim))
        self.decode.append(AdainResBlk1d(1024 + 2 + 64, 512, style_dim, upsample=True))
        self.F0_conv = PWNConv1d(1, 1, 3, stride=2, padding=1)
        self.N_conv = PWNConv1d(1, 1, 3, stride=2, padding=1)
        self.asr_res = nn.Sequential(PWNConv1d(512, 64, 1))
        self.generator = Generator(input_channels=dim_out, dim=dim_in, style_dim=style_dim,
                                   intermediate_dim=intermediate_dim, num_layers=num_layers,
                                   gen_istft_n_fft=gen_istft_n_fft, gen_istft_hop_size=gen_istft_hop_size)
        self._engine = None

    def invalidate(self):
        """Drop the packed weights (after writes through `param.data`, which stale() cannot see)."""
        self._engine = None

    def engine(self, dtype: str = "fp32"):
        from .engine import DecoderEngine
        if self._engine is None or self._engine.dtype != dtype or self._engine.stale(self):
            self._engine = DecoderEngine(self, dtype=dtype)
        return self._engine

    def forward(self, asr, F0_curve, N, s, dtype: str = "fp32"):
        """asr [B,512,T], F0_curve [B,2T], N [B,2T], s [B,style_dim] -> [B,1,2T*hop] (float32).
        The Vocos decoder has no harmonic source, so it draws no noise."""
        from .engine import forward_only
        forward_only(self, "vocos.Decoder")
        return self.engine(dtype).forward(asr, F0_curve, N, s)
