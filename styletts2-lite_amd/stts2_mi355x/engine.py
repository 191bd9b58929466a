"""ctypes binding of libstts2.so (include/stts2.h) and the per-module engines.

PyTorch is used only as the device-memory / stream container: parameters are the
module's own state-dict tensors on the HIP device, the packed-weight buffer and the
workspace are torch uint8 tensors, and every kernel is launched by the C library on
`torch.cuda.current_stream()`.  There is no compute fallback: without the library or
a HIP device every call raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

KIND_HIFIGAN, KIND_ISTFTNET, KIND_F0N, KIND_STYLE, KIND_MPD, KIND_VOCOS, KIND_MSD = 0, 1, 2, 3, 4, 5, 6
DTYPES = {"fp32": 0, "bf16": 1, "bf16x3": 2}  # bf16x3: the split-operand accuracy mode (STTS_SPLIT)

_LIB = None
_HERE = os.path.dirname(os.path.abspath(__file__))
# (STTS_LIB: another build of the same C-ABI revision, for build-against-build A/Bs on one box: tools/gpu/)
LIB_PATH = os.environ.get("STTS_LIB") or os.path.join(_HERE, "libstts2.so")
ABI_VERSION = 5  # include/stts2.h STTS_ABI_VERSION: the signatures bound below

c_int, c_ll, c_ull, c_vp, c_fp = ctypes.c_int, ctypes.c_longlong, ctypes.c_ulonglong, ctypes.c_void_p, ctypes.c_void_p


def lib():
    """Load libstts2.so (after torch, so both share torch's HIP runtime)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} missing: build it with `python -m stts2_mi355x.build` "
                           "(__graft_entry__.build()); there is no non-HIP fallback")
    L = ctypes.CDLL(LIB_PATH)
    L.stts_abi_version.argtypes = []
    L.stts_abi_version.restype = c_int
    if L.stts_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH}: C-ABI revision {L.stts_abi_version()}, these bindings expect {ABI_VERSION} "
                           "(include/stts2.h STTS_ABI_VERSION): rebuild the library")
    L.stts_model_create.argtypes = [c_int, ctypes.POINTER(c_int), c_int, ctypes.POINTER(c_vp)]
    L.stts_model_create.restype = c_int
    L.stts_model_destroy.argtypes = [c_vp]
    L.stts_model_destroy.restype = None
    L.stts_param_count.argtypes = [c_vp]
    L.stts_param_count.restype = c_int
    L.stts_param_name.argtypes = [c_vp, c_int]
    L.stts_param_name.restype = ctypes.c_char_p
    L.stts_param_numel.argtypes = [c_vp, c_int]
    L.stts_param_numel.restype = c_ll
    L.stts_set_param.argtypes = [c_vp, c_int, c_vp]
    L.stts_set_param.restype = c_int
    L.stts_packed_bytes.argtypes = [c_vp, c_int]
    L.stts_packed_bytes.restype = c_ll
    L.stts_pack.argtypes = [c_vp, c_int, c_vp, c_ll, c_vp]
    L.stts_pack.restype = c_int
    L.stts_workspace_bytes.argtypes = [c_vp, c_int, c_int, c_int]
    L.stts_workspace_bytes.restype = c_ll
    L.stts_decoder_fwd.argtypes = [c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_ull, c_ll, c_int, c_int, c_vp, c_vp,
                                   c_ll, c_vp]
    L.stts_decoder_fwd.restype = c_int
    L.stts_f0n_fwd.argtypes = [c_vp, c_int, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_ll, c_vp]
    L.stts_f0n_fwd.restype = c_int
    L.stts_style_fwd.argtypes = [c_vp, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_ll, c_vp]
    L.stts_style_fwd.restype = c_int
    L.stts_mpd_out_elems.argtypes = [c_vp, c_int, c_int]
    L.stts_mpd_out_elems.restype = c_ll
    L.stts_mpd_fwd.argtypes = [c_vp, c_int, c_vp, c_int, c_int, c_vp, c_ll, c_vp, c_ll, c_vp]
    L.stts_mpd_fwd.restype = c_int
    L.stts_mpd_losses.argtypes = [c_vp, c_int, c_int, c_vp, c_vp, c_ll, c_vp, c_vp]
    L.stts_mpd_losses.restype = c_int
    L.stts_msd_out_elems.argtypes = [c_vp, c_int, c_int]
    L.stts_msd_out_elems.restype = c_ll
    L.stts_msd_fwd.argtypes = [c_vp, c_int, c_vp, c_int, c_int, c_vp, c_ll, c_vp, c_ll, c_vp]
    L.stts_msd_fwd.restype = c_int
    L.stts_msd_losses.argtypes = [c_vp, c_int, c_int, c_vp, c_vp, c_ll, c_vp, c_vp]
    L.stts_gan_losses_scratch_bytes.argtypes = [c_vp]
    L.stts_gan_losses_scratch_bytes.restype = c_ll
    L.stts_msd_losses.restype = c_int
    for fn in ("stts_conv1d_fwd_workspace_bytes", "stts_conv1d_bwd_workspace_bytes",
               "stts_conv1d_fwd_tx_workspace_bytes", "stts_conv1d_bwd_tx_workspace_bytes"):
        getattr(L, fn).argtypes = [c_int] * 10
        getattr(L, fn).restype = c_ll
    L.stts_conv1d_fwd.argtypes = [c_int, c_vp, c_vp, c_vp] + [c_int] * 9 + [c_vp, c_vp, c_ll, c_vp]
    L.stts_conv1d_fwd.restype = c_int
    L.stts_conv1d_fwd_act.argtypes = [c_int, c_vp, c_vp, c_vp] + [c_int] * 9 + [ctypes.c_float, c_vp, c_vp, c_ll,
                                                                                  c_vp]
    L.stts_conv1d_fwd_act.restype = c_int
    L.stts_conv1d_fwd_tx.argtypes = [c_int, c_vp, c_vp, c_vp] + [c_int] * 10 + [ctypes.c_float, c_vp, c_vp, c_ll, c_vp]
    L.stts_conv1d_fwd_tx.restype = c_int
    L.stts_conv1d_bwd_tx.argtypes = [c_int, c_vp, c_vp] + [c_int] * 9 + [c_vp, c_vp, c_ll, c_vp]
    L.stts_conv1d_bwd_tx.restype = c_int
    L.stts_conv1d_wgrad_tx.argtypes = [c_int, c_vp, c_vp] + [c_int] * 9 + [c_vp, c_vp, c_vp, c_ll, c_vp]
    L.stts_conv1d_wgrad_tx.restype = c_int
    L.stts_conv1d_fwd_res.argtypes = [c_int, c_vp, c_vp, c_vp, c_vp, ctypes.c_float] + [c_int] * 9 + [c_vp, c_vp,
                                                                                                   c_ll, c_vp]
    L.stts_pool_workspace_bytes.argtypes = [c_int, c_int, c_int]
    L.stts_pool_workspace_bytes.restype = c_ll
    L.stts_pool_fwd.argtypes = [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp]
    L.stts_pool_fwd.restype = c_int
    L.stts_pool_bwd.argtypes = [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_ll, c_vp]
    L.stts_pool_bwd.restype = c_int
    L.stts_upsample2.argtypes = [c_vp, c_int, c_int, c_int, c_vp, c_vp]
    L.stts_upsample2.restype = c_int
    L.stts_upsample2_bwd.argtypes = [c_vp, c_int, c_int, c_int, c_vp, c_vp]
    L.stts_upsample2_bwd.restype = c_int
    L.stts_leaky_relu.argtypes = [c_vp, c_ll, ctypes.c_float, c_vp, c_vp]
    L.stts_leaky_relu.restype = c_int
    L.stts_leaky_relu_bwd.argtypes = [c_vp, c_vp, c_ll, ctypes.c_float, c_vp, c_vp]
    L.stts_leaky_relu_bwd.restype = c_int
    L.stts_conv1d_fwd_res.restype = c_int
    L.stts_conv_transpose1d_workspace_bytes.argtypes = [c_int] * 9
    L.stts_conv_transpose1d_workspace_bytes.restype = c_ll
    L.stts_conv_transpose1d_fwd.argtypes = [c_int, c_vp, c_vp, c_vp] + [c_int] * 8 + [c_vp, c_vp, c_ll, c_vp]
    L.stts_conv_transpose1d_fwd.restype = c_int
    L.stts_conv_transpose1d_bwd.argtypes = [c_int, c_vp, c_vp, c_vp] + [c_int] * 8 + [c_vp, c_vp, c_vp, c_vp, c_ll,
                                                                                      c_vp]
    L.stts_conv_transpose1d_bwd.restype = c_int
    L.stts_conv1d_bwd.argtypes = [c_int, c_vp, c_vp, c_vp] + [c_int] * 9 + [c_vp, c_vp, c_vp, c_vp, c_ll, c_vp]
    L.stts_conv1d_bwd.restype = c_int
    L.stts_weight_norm.argtypes = [c_vp, c_vp, c_int, c_int, c_vp, c_vp]
    L.stts_weight_norm.restype = c_int
    L.stts_adain_act_workspace_bytes.argtypes = [c_int, c_int, c_int]
    L.stts_adain_act_workspace_bytes.restype = c_ll
    L.stts_adain_act_fwd.argtypes = [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_ll, c_vp]
    L.stts_adain_act_fwd.restype = c_int
    L.stts_adain_act_bwd.argtypes = [c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp,
                                     c_vp, c_ll, c_vp]
    L.stts_adain_act_bwd.restype = c_int
    L.stts_linear_fwd.argtypes = [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp]
    L.stts_linear_fwd.restype = c_int
    L.stts_linear_bwd.argtypes = [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp]
    L.stts_linear_bwd.restype = c_int
    L.stts_weight_norm_bwd.argtypes = [c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp]
    L.stts_weight_norm_bwd.restype = c_int
    L.stts_mrstft_workspace_bytes.argtypes = [c_int, c_ll, ctypes.POINTER(c_int), c_int, c_int]
    L.stts_mrstft_workspace_bytes.restype = c_ll
    L.stts_mrstft_loss.argtypes = [c_vp, c_vp, c_int, c_ll, c_ll, ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                   ctypes.POINTER(c_int), c_int, c_int, c_int, c_vp, c_vp, c_ll, c_vp]
    L.stts_mrstft_loss.restype = c_int
    L.stts_mel_frames.argtypes = [c_ll]
    L.stts_mel_frames.restype = c_ll
    L.stts_mel_workspace_bytes.argtypes = []
    L.stts_mel_workspace_bytes.restype = c_ll
    L.stts_wave_preprocess.argtypes = [c_vp, c_int, c_ll, c_ll, c_vp, c_vp, c_ll, c_vp]
    L.stts_wave_preprocess.restype = c_int
    L.stts_error_string.argtypes = [c_int]
    L.stts_error_string.restype = ctypes.c_char_p
    L.stts_profile_enable.argtypes = [c_int]
    L.stts_profile_enable.restype = c_int
    L.stts_profile_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_ll),
                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    L.stts_profile_read.restype = c_int
    L.stts_profile_launch.argtypes = [c_ll, ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_double)]
    L.stts_profile_launch.restype = c_int
    L.stts_set_option.argtypes = [c_int, c_int]
    L.stts_set_option.restype = c_int
    L.stts_get_option.argtypes = [c_int]
    L.stts_get_option.restype = c_int
    L.stts_set_debug_buffer.argtypes = [c_vp]
    L.stts_set_debug_buffer.restype = c_int
    _LIB = L
    if os.environ.get("STTS_OPTS"):
        for k, v in OPT_DEFAULTS.items():
            check(L.stts_set_option(int(k), int(v)), "stts_set_option")
    return L


OPT_RESCONV = 1
OPT_GRID_CAP = 2
OPT_RESFUSED = 3
OPT_DEBUG = 4
OPT_STATS_SLOTS = 5


OPT_SMALL_TILES = 6
OPT_BIGCONV = 7
OPT_HEAD = 8
OPT_SKEW = 9
OPT_FRONT = 10
OPT_PW = 11
OPT_SPLITK = 12
OPT_EXP = 13
OPT_UPS = 14
OPT_WGRAD = 15
OPT_PLAINRC = 16
OPT_MSDFOLD = 17
OPT_RCPP = 18
OPT_RESSPLIT = 19
OPT_BF16F = 20
OPT_YF32 = 21
OPT_COUT1 = 22
OPT_BRANCHES = 23
OPT_NBRANCH = 24
OPT_BIGSPLIT = 25
OPT_BIGLA = 26
OPT_BIG64 = 27
OPT_BIG3 = 28
OPT_SEGPART = 29
OPT_RCOCC = 30
# the production defaults of every STTS_OPT_* (include/stts2.h)
OPT_DEFAULTS = {OPT_RESCONV: 1, OPT_GRID_CAP: 0, OPT_RESFUSED: 0, OPT_DEBUG: 0, OPT_STATS_SLOTS: 0,
                OPT_SMALL_TILES: 1, OPT_BIGCONV: 2, OPT_HEAD: 1, OPT_SKEW: 0, OPT_FRONT: 1, OPT_PW: 1, OPT_SPLITK: 1,
                OPT_EXP: 0, OPT_UPS: 1, OPT_WGRAD: 1, OPT_PLAINRC: 1, OPT_MSDFOLD: 1,
                OPT_RCPP: 3, OPT_RESSPLIT: 1, OPT_BF16F: 0, OPT_YF32: 1, OPT_COUT1: 1, OPT_BRANCHES: 8, OPT_NBRANCH: 64,
                OPT_BIGSPLIT: 1, OPT_BIGLA: 0, OPT_BIG64: 5, OPT_BIG3: 0, OPT_SEGPART: 1, OPT_RCOCC: 1}
# STTS_OPTS="KEY=VALUE,..." (A/B runs of whole suites): option values that replace the defaults for the process,
# applied when the library loads and by reset_options()
for _kv in filter(None, os.environ.get("STTS_OPTS", "").split(",")):
    _k, _v = (int(x) for x in _kv.split("="))
    OPT_DEFAULTS[_k] = _v


def set_option(key: int, value: int) -> None:
    """Process-wide engine option (include/stts2.h STTS_OPT_*)."""
    check(lib().stts_set_option(int(key), int(value)), "stts_set_option")


def get_option(key: int) -> int:
    return int(lib().stts_get_option(int(key)))


def reset_options() -> None:
    """Every engine option back to its production default (tests restore this after A/B runs)."""
    if _LIB is None:
        return
    for k, v in OPT_DEFAULTS.items():
        set_option(k, v)
    from . import prosody
    prosody.set_lstm_group(0)
    prosody.set_bilstm_debug(0, False)


def check(rc: int, what: str = "stts"):
    if rc != 0:
        msg = lib().stts_error_string(rc).decode()
        raise RuntimeError(f"{what} failed: {msg} (code {rc})")


def forward_only(module, what):
    """The HIP path of `module` has no backward: refuse to run where the caller would differentiate the
    output (grad mode on and a parameter requiring grad), instead of returning a tensor without a graph
    whose gradients would silently be lost.  Inference runs under torch.no_grad() (inference.py:234)."""
    if torch.is_grad_enabled() and any(p.requires_grad for p in module.parameters()):
        raise NotImplementedError(
            f"{what}: the HIP path is forward-only (no backward kernels for this module); call it under "
            "torch.no_grad() as inference.py does, or freeze its parameters (requires_grad_(False))")


_DEVICE_OK = False


def _require_device():
    global _DEVICE_OK
    if _DEVICE_OK:
        return
    if not torch.cuda.is_available():
        raise RuntimeError("stts2_mi355x needs a HIP device (MI355X / gfx950); no CPU fallback exists")
    _DEVICE_OK = True


# the raw query of the current stream: torch.cuda.current_stream() costs ~9 us of host time a call (device index,
# availability and environment checks), and a training step makes ~2,500 of these calls
_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_GET_DEVICE = getattr(torch._C, "_cuda_getDevice", None)


def _stream():
    if _RAW_STREAM is not None and _GET_DEVICE is not None:
        return ctypes.c_void_p(_RAW_STREAM(_GET_DEVICE()))
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _dev_f32(t, device):
    if not isinstance(t, torch.Tensor):
        t = torch.as_tensor(np.asarray(t))
    return t.detach().to(device=device, dtype=torch.float32).contiguous()


class NativeModel:
    """One stts_model handle: parameters bound by reference state-dict name, packed per dtype."""

    def __init__(self, kind: int, cfg, module: torch.nn.Module):
        _require_device()
        L = lib()
        self.kind = kind
        arr = (c_int * len(cfg))(*[int(v) for v in cfg])
        h = c_vp()
        check(L.stts_model_create(kind, arr, len(cfg), ctypes.byref(h)), "stts_model_create")
        self.h = h
        self.device = torch.device("cuda", torch.cuda.current_device())
        sd = module.state_dict(keep_vars=True)
        n = L.stts_param_count(h)
        self.names, self._keep = [], []
        # (tensor, _version, data_ptr) of every bound module tensor: an in-place update, a .to() or a
        # load_state_dict makes the packed weights stale (_Engine.stale)
        self.sources = []
        for i in range(n):
            name = L.stts_param_name(h, i).decode()
            if name not in sd:
                raise KeyError(f"parameter {name} expected by the native plan is not in the module state dict")
            src = sd[name]
            self.sources.append((src, src._version, src.data_ptr()))
            t = _dev_f32(src.detach(), self.device)
            if t.numel() != L.stts_param_numel(h, i):
                raise ValueError(f"{name}: numel {t.numel()} != plan {L.stts_param_numel(h, i)}")
            self._keep.append(t)
            self.names.append(name)
            check(L.stts_set_param(h, i, _ptr(t)), "stts_set_param")
        self._packed = {}
        self._ws = {}

    def pack(self, dtype: str):
        if dtype not in self._packed:
            L = lib()
            dt = DTYPES[dtype]
            nb = L.stts_packed_bytes(self.h, dt)
            if nb < 0:
                check(int(nb), "stts_packed_bytes")
            buf = torch.empty(max(int(nb), 1), dtype=torch.uint8, device=self.device)
            check(L.stts_pack(self.h, dt, _ptr(buf), int(nb), _stream()), "stts_pack")
            self._packed[dtype] = buf
        return self._packed[dtype]

    def workspace(self, dtype: str, B: int, T: int):
        L = lib()
        nb = L.stts_workspace_bytes(self.h, DTYPES[dtype], int(B), int(T))
        if nb < 0:
            check(int(nb), "stts_workspace_bytes")
        cur = self._ws.get(dtype)
        if cur is None or cur.numel() < nb:
            self._ws[dtype] = cur = torch.empty(max(int(nb), 1), dtype=torch.uint8, device=self.device)
        return cur, int(nb)

    def __del__(self):
        try:
            if getattr(self, "h", None) and _LIB is not None:
                _LIB.stts_model_destroy(self.h)
        except Exception:
            pass


def _watch(module, engine_attr="_engine"):
    """Drop a module's cached engine whenever new weights are loaded."""
    if getattr(module, "_stts_hooked", False):
        return

    def hook(mod, incompatible):
        setattr(mod, engine_attr, None)
    module.register_load_state_dict_post_hook(hook)
    module._stts_hooked = True


class _Engine:
    def __init__(self, module, dtype):
        if dtype not in DTYPES:
            raise ValueError(f"dtype must be one of {list(DTYPES)}")
        self.dtype = dtype
        _watch(module)

    def stale(self, module):
        """True when a bound parameter changed since packing: an in-place update (its _version moved),
        a move or re-allocation (.to(), .cuda(), a new tensor: data_ptr moved).  Writes through
        `param.data` bypass the version counter: call `module.invalidate()` after those."""
        for src, ver, ptr in self.model.sources:
            if src._version != ver or src.data_ptr() != ptr:
                return True
        return False


class DecoderEngine(_Engine):
    """HIP forward of Modules/hifigan.py / istftnet.py / vocos.py Decoder (reference :446 / :692 / :392)."""

    def __init__(self, module, dtype="fp32"):
        super().__init__(module, dtype)
        g = module.generator
        if module.decoder_type == "vocos":
            kind = KIND_VOCOS
            cfg = [module.dim_in, module.style_dim, g.intermediate_dim, g.num_layers, g.n_fft, g.hop]
            self.scale = g.hop  # output samples per F0 frame (2T frames x hop)
        else:
            kind = KIND_ISTFTNET if module.decoder_type == "istftnet" else KIND_HIFIGAN
            cfg = [module.dim_in, module.style_dim, g.upsample_initial_channel, len(g.upsample_rates),
                   *g.upsample_rates, *g.upsample_kernel_sizes, len(g.resblock_kernel_sizes),
                   *g.resblock_kernel_sizes, *[d for ds in g.resblock_dilation_sizes for d in ds]]
            if kind == KIND_ISTFTNET:
                cfg += [g.gen_istft_n_fft, g.gen_istft_hop_size]
            self.scale = g.upsample_scale
        self.kind = kind
        self.dim_in, self.style_dim = module.dim_in, module.style_dim
        self.model = NativeModel(kind, cfg, module)
        self.model.pack(dtype)

    def forward(self, asr, F0_curve, N, s, noise=None, seed=None, utt_offset=0, out=None):
        """seed None (and no noise): one draw from torch's default generator keys the device noise,
        so torch.manual_seed governs it and successive calls differ, as the reference's
        randn_like draws (hifigan.py:213) do."""
        dev = self.model.device
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if noise is None and self.kind != KIND_VOCOS else 0
        in_dev = asr.device if isinstance(asr, torch.Tensor) else torch.device("cpu")
        asr, F0_curve, N, s = (_dev_f32(t, dev) for t in (asr, F0_curve, N, s))
        B, C, T = asr.shape
        if C != self.dim_in or tuple(F0_curve.shape) != (B, 2 * T) or tuple(N.shape) != (B, 2 * T) \
                or tuple(s.shape) != (B, self.style_dim):
            raise ValueError(f"decoder inputs: asr {tuple(asr.shape)}, F0 {tuple(F0_curve.shape)}, "
                             f"N {tuple(N.shape)}, s {tuple(s.shape)}")
        if T < 2:  # the reference's InstanceNorm1d raises on a single frame (torch F.instance_norm)
            raise ValueError(f"decoder inputs: need at least 2 asr frames, got {T}")
        Lw = 2 * T * self.scale
        if noise is not None and self.kind == KIND_VOCOS:
            raise ValueError("the Vocos decoder has no harmonic source: noise must be None")
        if noise is not None:
            noise = _dev_f32(noise, dev)
            if tuple(noise.shape) != (B, Lw, 9):
                raise ValueError(f"noise must be [B, {Lw}, 9], got {tuple(noise.shape)}")
        if out is None:
            out = torch.empty(B, 1, Lw, dtype=torch.float32, device=dev)
        ws, nb = self.model.workspace(self.dtype, B, T)
        rc = lib().stts_decoder_fwd(self.model.h, DTYPES[self.dtype], _ptr(asr), _ptr(F0_curve), _ptr(N), _ptr(s),
                                    _ptr(noise), int(seed) & (2 ** 64 - 1), int(utt_offset), B, T, _ptr(out),
                                    _ptr(ws), nb, _stream())
        check(rc, "stts_decoder_fwd")
        return out if in_dev.type == "cuda" else out.to(in_dev)


class F0NEngine(_Engine):
    """HIP forward of ProsodyPredictor.F0Ntrain's conv stacks (reference models.py:451-461)."""

    def __init__(self, module, dtype="fp32"):
        super().__init__(module, dtype)
        self.d_hid, self.style_dim = module.d_hid, module.style_dim
        self.model = NativeModel(KIND_F0N, [module.d_hid, module.style_dim], module)
        self.model.pack(dtype)

    def forward_nlc(self, x, s):
        """x: shared-LSTM output [B, T, d_hid] (batch_first); s [B, style_dim] -> (F0, N) [B, 2T]."""
        dev = self.model.device
        in_dev = x.device
        x, s = _dev_f32(x, dev), _dev_f32(s, dev)
        B, T, D = x.shape
        if D != self.d_hid or tuple(s.shape) != (B, self.style_dim):
            raise ValueError(f"F0Ntrain inputs: x {tuple(x.shape)}, s {tuple(s.shape)}")
        if T < 2:  # as the reference's InstanceNorm1d on a single frame
            raise ValueError(f"F0Ntrain inputs: need at least 2 frames, got {T}")
        F0 = torch.empty(B, 2 * T, dtype=torch.float32, device=dev)
        Nn = torch.empty(B, 2 * T, dtype=torch.float32, device=dev)
        ws, nb = self.model.workspace(self.dtype, B, T)
        check(lib().stts_f0n_fwd(self.model.h, DTYPES[self.dtype], _ptr(x), _ptr(s), B, T, _ptr(F0), _ptr(Nn),
                                 _ptr(ws), nb, _stream()), "stts_f0n_fwd")
        if in_dev.type != "cuda":
            return F0.to(in_dev), Nn.to(in_dev)
        return F0, Nn


class StyleEngine(_Engine):
    """HIP forward of models.py StyleEncoder (reference models.py:145-150)."""

    def __init__(self, module, dtype="fp32"):
        super().__init__(module, dtype)
        d_in = module.shared[0].cout
        self.style_dim = module.style_dim
        max_conv = max(d for _, d in module.dims)
        self.model = NativeModel(KIND_STYLE, [d_in, module.style_dim, max_conv], module)
        self.model.pack(dtype)

    def forward(self, mel):
        dev = self.model.device
        in_dev = mel.device
        mel = _dev_f32(mel, dev)
        B, one, M, T = mel.shape
        if one != 1 or M != 80:
            raise ValueError(f"mel must be [B, 1, 80, T], got {tuple(mel.shape)}")
        out = torch.empty(B, self.style_dim, dtype=torch.float32, device=dev)
        ws, nb = self.model.workspace(self.dtype, B, T)
        check(lib().stts_style_fwd(self.model.h, DTYPES[self.dtype], _ptr(mel), B, T, _ptr(out), _ptr(ws), nb,
                                   _stream()), "stts_style_fwd")
        return out if in_dev.type == "cuda" else out.to(in_dev)


MPD_CH = (1, 32, 128, 512, 1024, 1024, 1)


def mpd_lengths(T: int, p: int):
    """Frame counts of DiscriminatorP(p)'s 6 feature maps over T samples (plan.cpp mpd_lengths)."""
    L = [(T + p - 1) // p]
    for _ in range(4):
        L.append((L[-1] + 4 - 5) // 3 + 1)
    L.append(L[-1])
    return L


class MPDEngine(_Engine):
    """HIP forward of Modules/discriminators.py MultiPeriodDiscriminator's DiscriminatorP stacks
    (reference :108-129): one batch of waveforms [B, 1, T] -> per period (scores [B, L*p], fmaps)."""

    def __init__(self, module, dtype="fp32"):
        super().__init__(module, dtype)
        self.periods = [d.period for d in module.discriminators]
        self.model = NativeModel(KIND_MPD, [len(self.periods), *self.periods], module)
        self.model.pack(dtype)

    def forward(self, x):
        dev = self.model.device
        in_dev = x.device
        w = _dev_f32(x, dev)
        if w.dim() != 3 or w.shape[1] != 1:
            raise ValueError(f"waveform must be [B, 1, T], got {tuple(w.shape)}")
        B, _, T = w.shape
        for p in self.periods:
            if (-T) % p >= T:
                raise ValueError(f"T = {T} too short for the period-{p} reflect pad")
        n = lib().stts_mpd_out_elems(self.model.h, B, T)
        check(int(n) if n < 0 else 0, "stts_mpd_out_elems")
        out = torch.empty(int(n), dtype=torch.float32, device=dev)
        ws, nb = self.model.workspace(self.dtype, B, T)
        check(lib().stts_mpd_fwd(self.model.h, DTYPES[self.dtype], _ptr(w), B, T, _ptr(out), int(n), _ptr(ws), nb,
                                 _stream()), "stts_mpd_fwd")
        self.last = (out, B, T)
        res, off = [], 0
        for p in self.periods:
            L = mpd_lengths(T, p)
            fmaps = []
            for j in range(6):
                C, Lj = MPD_CH[j + 1], L[j + 1] if j < 5 else L[5]
                k = B * p * Lj * C
                # frames [B*p][L][C] -> the reference's [B, C, L, p] (a permuted view)
                f = out[off:off + k].view(B, p, Lj, C).permute(0, 3, 2, 1)
                fmaps.append(f if in_dev.type == "cuda" else f.to(in_dev))
                off += k
            score = torch.flatten(fmaps[-1], 1, -1)  # discriminators.py:129
            res.append((score, fmaps))
        return res

    def gan_losses(self):
        """losses.py:97-128 feature_loss, generator_loss[0], discriminator_loss[0] of the last
        forward, whose batch was B real then B generated waveforms: device float64 tensor [3]."""
        out, B2, T = self.last
        if B2 % 2:
            raise ValueError("the last forward's batch is not real + generated halves")
        nb = int(lib().stts_gan_losses_scratch_bytes(self.model.h))
        check(nb if nb < 0 else 0, "stts_gan_losses_scratch_bytes")
        scratch = torch.empty(nb // 8, dtype=torch.float64, device=out.device)
        loss = torch.empty(3, dtype=torch.float64, device=out.device)
        check(lib().stts_mpd_losses(self.model.h, B2 // 2, T, _ptr(out), _ptr(scratch), nb, _ptr(loss), _stream()),
              "stts_mpd_losses")
        return loss


def msd_geometry(T, n_fft, hop):
    """SpecDiscriminator map sizes over T samples (plan.cpp:msd_geom): H frames, widths W[0..5]."""
    H = 1 + T // hop
    W = [n_fft // 2 + 1] * 2
    for _ in range(3):
        W.append((W[-1] - 1) // 2 + 1)
    W.append(W[-1])
    return H, W


class MSDEngine(_Engine):
    """HIP forward of Modules/discriminators.py MultiResSpecDiscriminator's SpecDiscriminator stacks
    (reference :47-63): one batch of waveforms [B, 1, T] -> per resolution (scores [B, H*W], fmaps)."""

    def __init__(self, module, dtype="fp32"):
        super().__init__(module, dtype)
        self.res = [(d.fft_size, d.shift_size, d.win_length) for d in module.discriminators]
        cfg = [len(self.res)] + [v for r in self.res for v in r]
        self.model = NativeModel(KIND_MSD, cfg, module)
        self.model.pack(dtype)

    def forward(self, x):
        dev = self.model.device
        in_dev = x.device
        w = _dev_f32(x, dev)
        if w.dim() == 3:
            if w.shape[1] != 1:
                raise ValueError(f"waveform must be [B, 1, T] or [B, T], got {tuple(w.shape)}")
            w = w[:, 0]
        B, T = w.shape
        for n_fft, _, _ in self.res:
            if T <= n_fft // 2:  # torch.stft's reflect pad
                raise ValueError(f"T = {T} too short for n_fft {n_fft}")
        w = w.contiguous()
        n = lib().stts_msd_out_elems(self.model.h, B, T)
        check(int(n) if n < 0 else 0, "stts_msd_out_elems")
        out = torch.empty(int(n), dtype=torch.float32, device=dev)
        ws, nb = self.model.workspace(self.dtype, B, T)
        check(lib().stts_msd_fwd(self.model.h, DTYPES[self.dtype], _ptr(w), B, T, _ptr(out), int(n), _ptr(ws), nb,
                                 _stream()), "stts_msd_fwd")
        self.last = (out, B, T)
        res, off = [], 0
        for n_fft, hop, _ in self.res:
            H, W = msd_geometry(T, n_fft, hop)
            fmaps = []
            for j in range(6):
                C, Wj = (32, W[j + 1]) if j < 5 else (1, W[5])
                k = B * H * Wj * C
                f = out[off:off + k].view(B, H, Wj, C).permute(0, 3, 1, 2)  # -> [B, C, H, W] (a view)
                fmaps.append(f if in_dev.type == "cuda" else f.to(in_dev))
                off += k
            res.append((torch.flatten(fmaps[-1], 1, -1), fmaps))  # discriminators.py:63
        return res

    def gan_losses(self):
        """losses.py:97-128 over the last forward's outputs (B real then B generated signals)."""
        out, B2, T = self.last
        if B2 % 2:
            raise ValueError("the last forward's batch is not real + generated halves")
        nb = int(lib().stts_gan_losses_scratch_bytes(self.model.h))
        check(nb if nb < 0 else 0, "stts_gan_losses_scratch_bytes")
        scratch = torch.empty(nb // 8, dtype=torch.float64, device=out.device)
        loss = torch.empty(3, dtype=torch.float64, device=out.device)
        check(lib().stts_msd_losses(self.model.h, B2 // 2, T, _ptr(out), _ptr(scratch), nb, _ptr(loss), _stream()),
              "stts_msd_losses")
        return loss


N_MELS, MEL_HOP, MEL_NFFT = 80, 300, 2048


def wave_preprocess_batch(wave):
    """HIP log-mel of B equal-length waves: wave [B, L] (any device) -> device [B, 80, 1 + L // 300]
    (reference inference.py:43-49 per row).  L must exceed 1024, as the reference's reflect
    padding requires."""
    _require_device()
    dev = torch.device("cuda", torch.cuda.current_device())
    w = _dev_f32(wave, dev)
    if w.dim() != 2:
        raise ValueError(f"wave must be [B, L], got {tuple(w.shape)}")
    B, L = w.shape
    if L <= MEL_NFFT // 2:
        raise ValueError(f"wave of {L} samples: the reflect padding of n_fft {MEL_NFFT} needs more than "
                         f"{MEL_NFFT // 2}")
    F = int(lib().stts_mel_frames(L))
    out = torch.empty(B, N_MELS, F, dtype=torch.float32, device=dev)
    nb = int(lib().stts_mel_workspace_bytes())
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    check(lib().stts_wave_preprocess(_ptr(w), B, L, L, _ptr(out), _ptr(ws), nb, _stream()), "stts_wave_preprocess")
    return out


def profile_enable(on: bool = True):
    check(lib().stts_profile_enable(1 if on else 0))


def profile_read():
    t, n, f, b = ctypes.c_double(), c_ll(), ctypes.c_double(), ctypes.c_double()
    check(lib().stts_profile_read(ctypes.byref(t), ctypes.byref(n), ctypes.byref(f), ctypes.byref(b)))
    return {"ms": t.value, "launches": n.value, "flops": f.value, "bytes": b.value}


ENGINE_KERNELS = ("conv1d_igemm_kernel", "k_resconv", "k_bigconv", "k_resfused", "k_conv_post",
                  "k_pwgemm", "k_ressplit", "k_bigconv2[SP]")  # engine ids 0..7


def profile_launches():
    """Per-launch records of the timed region: dicts with the GEMM shape, the kernel the launch
    was routed to, ms, flops, bytes."""
    out = []
    n = profile_read()["launches"]
    shape, v = (ctypes.c_int * 8)(), (ctypes.c_double * 3)()
    for i in range(n):
        check(lib().stts_profile_launch(i, shape, v))
        out.append({"B": shape[0], "rows": shape[1], "N": shape[2], "Cin": shape[3], "taps": shape[4],
                    "dil": shape[5], "Lout": shape[6], "res_acc": shape[7] & 3,
                    "kernel": ENGINE_KERNELS[(shape[7] >> 4) & 7], "ms": v[0], "flops": v[1], "bytes": v[2]})
    return out
