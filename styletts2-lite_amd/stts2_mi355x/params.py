"""Parameter-holder modules that reproduce the reference state-dict layout.

The drop-in Decoder / ProsodyPredictor / StyleEncoder classes must accept the
reference checkpoints unchanged (`model[key].load_state_dict(params[key])`,
reference inference.py:158-168), so every parameter keeps the reference name and
shape.  These holders own the parameters only; no arithmetic happens in them —
the forward passes are HIP launches through the C-ABI (engine.py).

Weight-norm layout follows torch.nn.utils.weight_norm(dim=0) as applied in the
reference (Modules/hifigan.py:30-46, 292, 317, 373-382, 434-439): parameters
`weight_g` [d0,1,...] and `weight_v`; for ConvTranspose1d d0 is the *input*
channel.
"""
from __future__ import annotations

import torch
import torch.nn as nn


def _p(*shape):
    return nn.Parameter(torch.zeros(*shape))


class WNConv1d(nn.Module):
    """weight_norm(nn.Conv1d(cin, cout, k, stride, padding, dilation, groups, bias))."""

    def __init__(self, cin, cout, k, stride=1, padding=0, dilation=1, groups=1, bias=True):
        super().__init__()
        self.cin, self.cout, self.k = cin, cout, k
        self.stride, self.padding, self.dilation, self.groups = stride, padding, dilation, groups
        if bias:
            self.bias = _p(cout)
        else:
            self.register_parameter("bias", None)
        self.weight_g = _p(cout, 1, 1)
        self.weight_v = _p(cout, cin // groups, k)

    def folded(self) -> torch.Tensor:
        return torch._weight_norm(self.weight_v, self.weight_g, 0)


class WNConvT1d(nn.Module):
    """weight_norm(nn.ConvTranspose1d(cin, cout, k, stride, padding, output_padding, groups))."""

    def __init__(self, cin, cout, k, stride, padding=0, output_padding=0, groups=1):
        super().__init__()
        self.cin, self.cout, self.k = cin, cout, k
        self.stride, self.padding, self.output_padding, self.groups = stride, padding, output_padding, groups
        self.bias = _p(cout)
        self.weight_g = _p(cin, 1, 1)
        self.weight_v = _p(cin, cout // groups, k)

    def folded(self) -> torch.Tensor:
        return torch._weight_norm(self.weight_v, self.weight_g, 0)


class Conv1d(nn.Module):
    """plain nn.Conv1d parameters (weight, bias)."""

    def __init__(self, cin, cout, k, stride=1, padding=0, bias=True):
        super().__init__()
        self.cin, self.cout, self.k, self.stride, self.padding = cin, cout, k, stride, padding
        self.weight = _p(cout, cin, k)
        if bias:
            self.bias = _p(cout)
        else:
            self.register_parameter("bias", None)


class Conv2d(nn.Module):
    """plain nn.Conv2d parameters (weight, bias)."""

    def __init__(self, cin, cout, k, stride=1, padding=0, groups=1, bias=True):
        super().__init__()
        kh, kw = (k, k) if isinstance(k, int) else k
        self.cin, self.cout, self.kh, self.kw = cin, cout, kh, kw
        self.stride, self.padding, self.groups = stride, padding, groups
        self.weight = _p(cout, cin // groups, kh, kw)
        if bias:
            self.bias = _p(cout)
        else:
            self.register_parameter("bias", None)


class Linear(nn.Module):
    def __init__(self, cin, cout, bias=True):
        super().__init__()
        self.weight = _p(cout, cin)
        if bias:
            self.bias = _p(cout)
        else:
            self.register_parameter("bias", None)


class AdaIN1d(nn.Module):
    """reference hifigan.py:14-24 / models.py:303-313: InstanceNorm1d(affine=False) + fc."""

    def __init__(self, style_dim, num_features):
        super().__init__()
        self.num_features = num_features
        self.fc = Linear(style_dim, num_features * 2)


class AdaINResBlock1(nn.Module):
    """reference hifigan.py:26-80 parameter layout (convs1/convs2/adain1/adain2/alpha1/alpha2)."""

    def __init__(self, channels, kernel_size=3, dilation=(1, 3, 5), style_dim=64):
        super().__init__()
        self.channels, self.kernel_size, self.dilation = channels, kernel_size, tuple(dilation)
        self.convs1 = nn.ModuleList([
            WNConv1d(channels, channels, kernel_size, 1, dilation=d, padding=(kernel_size * d - d) // 2)
            for d in dilation])
        self.convs2 = nn.ModuleList([
            WNConv1d(channels, channels, kernel_size, 1, dilation=1, padding=(kernel_size - 1) // 2)
            for _ in dilation])
        self.adain1 = nn.ModuleList([AdaIN1d(style_dim, channels) for _ in dilation])
        self.adain2 = nn.ModuleList([AdaIN1d(style_dim, channels) for _ in dilation])
        self.alpha1 = nn.ParameterList([nn.Parameter(torch.ones(1, channels, 1)) for _ in dilation])
        self.alpha2 = nn.ParameterList([nn.Parameter(torch.ones(1, channels, 1)) for _ in dilation])


class AdainResBlk1d(nn.Module):
    """reference hifigan.py:359-403 == models.py:326-370 parameter layout."""

    def __init__(self, dim_in, dim_out, style_dim=64, upsample="none", dropout_p=0.0):
        super().__init__()
        self.dim_in, self.dim_out = dim_in, dim_out
        self.upsample_type = "none" if upsample in ("none", False, None) else "half"
        self.learned_sc = dim_in != dim_out
        self.dropout_p = dropout_p
        self.conv1 = WNConv1d(dim_in, dim_out, 3, 1, 1)
        self.conv2 = WNConv1d(dim_out, dim_out, 3, 1, 1)
        self.norm1 = AdaIN1d(style_dim, dim_in)
        self.norm2 = AdaIN1d(style_dim, dim_out)
        if self.learned_sc:
            self.conv1x1 = WNConv1d(dim_in, dim_out, 1, 1, 0, bias=False)
        if self.upsample_type != "none":
            self.pool = WNConvT1d(dim_in, dim_in, 3, 2, padding=1, output_padding=1, groups=dim_in)


class SourceModuleHnNSF(nn.Module):
    """reference hifigan.py:221-268 parameters: l_linear = Linear(harmonic_num+1, 1)."""

    def __init__(self, harmonic_num=8):
        super().__init__()
        self.harmonic_num = harmonic_num
        self.l_linear = Linear(harmonic_num + 1, 1)
