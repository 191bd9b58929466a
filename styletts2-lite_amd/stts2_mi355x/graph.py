"""hipGraph replay of one decoder forward (B = 1 latency).

A decoder forward is ~120 kernel launches.  `CapturedDecoder` captures them once, at a fixed
(B, T, dtype), into a torch CUDA (= HIP) graph over static input / noise / output buffers; a call
copies the inputs in, draws the SineGen noise into the static noise buffer with `normal_()` from
torch's generator (exactly the reference's per-call `randn_like` semantics, hifigan.py:213), and
replays the graph.  Weights must not change between capture and replay (re-capture after
`load_state_dict` / in-place edits: the packed copy the graph reads is the one packed at capture).

    from stts2_mi355x.graph import CapturedDecoder
    run = CapturedDecoder(decoder, B=1, T=400, dtype="bf16")
    audio = run(asr, F0, N, s)          # [B, 1, 600 T] on the GPU (a view of the static output)
"""
from __future__ import annotations

import torch


class CapturedDecoder:
    def __init__(self, decoder, B: int, T: int, dtype: str = "bf16", warmup: int = 2):
        if not torch.cuda.is_available():
            raise RuntimeError("CapturedDecoder needs the MI355X (HIP) device")
        dev = next(decoder.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("move the decoder to the GPU before capturing")
        self.decoder, self.B, self.T, self.dtype = decoder, B, T, dtype
        eng = decoder.engine(dtype)
        L = 2 * T * eng.scale
        f32 = dict(dtype=torch.float32, device=dev)
        self.asr = torch.zeros(B, eng.dim_in, T, **f32)
        self.f0 = torch.zeros(B, 2 * T, **f32)
        self.n = torch.zeros(B, 2 * T, **f32)
        self.s = torch.zeros(B, eng.style_dim, **f32)
        self.noise = torch.zeros(B, L, 9, **f32)
        self.out = torch.empty(B, 1, L, **f32)
        self._eng = eng
        # warm up on a side stream (first launches set kernel attributes, size the workspace)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._launch()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._launch()
        torch.cuda.synchronize()
        # the graph holds raw pointers into the engine's workspace: keep that allocation alive even
        # if a later eager forward at a larger size replaces the engine's buffer
        self._ws = eng.model._ws[dtype]

    def _launch(self):
        self._eng.forward(self.asr, self.f0, self.n, self.s, noise=self.noise, out=self.out)

    def __call__(self, asr, F0_curve, N, s, noise=None):
        """Inputs as Decoder.forward; `noise` [B, 600T, 9] (parity) or None: a fresh normal_() draw."""
        if self._eng.stale(self.decoder):
            raise RuntimeError("decoder weights changed since capture: build a new CapturedDecoder")
        self.asr.copy_(asr)
        self.f0.copy_(F0_curve)
        self.n.copy_(N)
        self.s.copy_(s)
        if noise is None:
            self.noise.normal_()
        else:
            self.noise.copy_(noise)
        self.graph.replay()
        return self.out
