"""fp64 truth for the decoder gradients at the config-5 shape (B = 2 segments of 155 frames = 93,000 samples,
train.py:235 max_len 310), made in the survey container (hours of CPU are not available on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train_c5.py

The oracle's decoder (oracle.decoder_hifigan) reproduces the reference's Decoder forward and autograd
bit-exactly in fp32 (tests/test_train_oracle_cpu.py, tests/golden/make_golden_train.py), so its fp64 run is
the reference's computation without fp32 rounding (the SineGen phase stays fp32, as the reference computes
it).  A fixed linear probe of the output, loss = sum(y * r), is differentiated in fp64 and in fp32; stored
per parameter tensor: L2 norm, max |g|, values at 24 formula indices, for both dtypes, plus the input
gradients in full (tests/golden/train_c5_decoder_grads.npz).  At this size some fp32 gradients (e.g.
l_linear's, a sum of 186,000 terms that cancel to ~1e-3 of their magnitude) are themselves inaccurate;
the GPU test compares the HIP gradients with the fp64 values next to the fp32 reference's error.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd"), os.path.join(ROOT, "tests")]
from helpers import HIFI_CFG, make_decoder  # noqa: E402
from oracle import stts_oracle as orc  # noqa: E402
from stts2_mi355x import synth  # noqa: E402

NPROBE = 24


def probe_idx(name, n):
    return np.minimum((synth.hash_u01("probe_idx." + name, NPROBE) * n).astype(np.int64), n - 1)


def main(B=2, T=155):
    torch.set_num_threads(os.cpu_count())
    dec, _ = make_decoder("hifigan")
    sd = {k: v.detach().clone() for k, v in dec.state_dict().items()}
    asr, f0, n, s = (torch.from_numpy(a) for a in synth.decoder_inputs(B, T, tag="train"))
    L = 600 * T
    noise = torch.from_numpy(synth.source_noise(B, L, tag="train_noise"))
    r = torch.from_numpy(synth.normal("dec_probe_c5", (B, 1, L)))
    rec = {"B": np.int64(B), "T": np.int64(T)}
    names = sorted(sd)
    rec["names"] = np.array(names)
    for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
        t0 = time.time()
        leaf = {k: v.detach().to(dt).clone().requires_grad_(True) for k, v in sd.items()}
        ins = [t.detach().to(dt).clone().requires_grad_(True) for t in (asr, f0, n, s)]
        y = orc.decoder_hifigan(*ins, leaf, HIFI_CFG, noise)
        (y * r.to(dt)).sum().backward()
        l2, mx, idx, val = [], [], [], []
        for k in names:
            g = leaf[k].grad.detach().reshape(-1).double().numpy()
            ix = probe_idx(k, g.size)
            l2.append(np.sqrt((g * g).sum()))
            mx.append(np.abs(g).max())
            idx.append(ix)
            val.append(g[ix])
        rec[f"{tag}.l2"], rec[f"{tag}.maxabs"] = np.array(l2), np.array(mx)
        rec["idx"], rec[f"{tag}.val"] = np.stack(idx), np.stack(val)
        for k, t in zip(("asr", "F0_curve", "N", "s"), ins):
            rec[f"{tag}.grad_in.{k}"] = t.grad.detach().numpy().astype(np.float32 if tag == "f32" else np.float64)
        rec[f"{tag}.y_absmax"] = np.float64(y.detach().abs().max())
        print(tag, f"{time.time() - t0:.1f} s", flush=True)
    path = os.path.join(HERE, f"train_c5_decoder_grads.npz")
    np.savez_compressed(path, **rec)
    e = np.abs(rec["f32.val"] - rec["f64.val"]).max(1) / np.maximum(rec["f64.maxabs"], 1e-3 * rec["f64.maxabs"].max())
    print(path, os.path.getsize(path), "fp32 reference's worst per-tensor error vs fp64:",
          f"{e.max():.2e} ({names[int(e.argmax())]})")


if __name__ == "__main__":
    main()
