"""Gradient fixtures of the two modules train.py differentiates besides the decoder (train.py:258, 265, 323-324):
ProsodyPredictor.F0Ntrain (models.py:448-461: the shared BiLSTM, the F0 / N AdainResBlk1d stacks and the 1x1
projections) and StyleEncoder (models.py:125-150), from the REFERENCE modules' own autograd.

Run in the survey container only (needs /root/reference; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train_pred.py

Formula weights and inputs (stts2_mi355x/synth.py); the modules in eval mode (dropout off: train.py runs the
predictor in train mode, whose dropout draws no implementation reproduces; the HIP dropout is tested on its own).
A fixed linear probe of the outputs, loss = sum(F0 r_F0) + sum(N r_N) (resp. sum(s r_s)), is differentiated in
fp64 (the truth) and in fp32 (the reference as it runs).  Stored per parameter tensor: L2 norm, max |g| and the
values at 24 formula indices for both dtypes; the input gradients and the outputs in full.  Data only.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import fill, import_models  # noqa: E402
from stts2_mi355x import synth  # noqa: E402

NPROBE = 24


def probe_idx(name, n):
    return np.minimum((synth.hash_u01("probe_idx." + name, NPROBE) * n).astype(np.int64), n - 1)


def summarize(rec, tag, params, names):
    l2, mx, idx, val = [], [], [], []
    for k in names:
        g = params[k].grad.detach().reshape(-1).double().numpy()
        ix = probe_idx(k, g.size)
        l2.append(np.sqrt((g * g).sum()))
        mx.append(np.abs(g).max())
        idx.append(ix)
        val.append(g[ix])
    rec[f"{tag}.l2"] = np.array(l2)
    rec[f"{tag}.maxabs"] = np.array(mx)
    rec[f"{tag}.idx"] = np.stack(idx)
    rec[f"{tag}.val"] = np.stack(val)


def f0n_case(B, T):
    models = import_models()
    en = torch.from_numpy(np.stack([synth.normal(f"tp:en:{b}:{T}", (640, T)) for b in range(B)]))
    s = torch.from_numpy(np.stack([synth.normal(f"tp:s:{b}", (128,)) for b in range(B)]))
    rF, rN = (torch.from_numpy(synth.normal(f"tp:probe:{k}:{T}", (B, 2 * T))) for k in ("F0", "N"))
    rec = {"B": np.int64(B), "T": np.int64(T)}
    for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
        torch.manual_seed(0)
        pp = fill(models.ProsodyPredictor(style_dim=128, d_hid=512, nlayers=3, max_dur=50, dropout=0.2)).eval().to(dt)
        params = {k: p for k, p in pp.named_parameters()
                  if k.startswith(("shared.", "F0.", "N.", "F0_proj.", "N_proj."))}
        x, sd = en.to(dt).clone().requires_grad_(True), s.to(dt).clone().requires_grad_(True)
        F0, N = pp.F0Ntrain(x, sd)
        ((F0 * rF.to(dt)).sum() + (N * rN.to(dt)).sum()).backward()
        names = sorted(params)
        rec["names"] = np.array(names)
        summarize(rec, tag, params, names)
        rec[f"{tag}.F0"], rec[f"{tag}.N"] = F0.detach().numpy(), N.detach().numpy()
        rec[f"{tag}.grad_en"], rec[f"{tag}.grad_s"] = x.grad.numpy(), sd.grad.numpy()
    return rec


def style_case(B, Fr):
    models = import_models()
    mel = torch.from_numpy(np.stack([synth.normal(f"tp:mel:{b}:{Fr}", (1, 80, Fr)) for b in range(B)]))
    r = torch.from_numpy(synth.normal(f"tp:probe:style:{Fr}", (B, 128)))
    rec = {"B": np.int64(B), "F": np.int64(Fr)}
    for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
        se = fill(models.StyleEncoder(dim_in=64, style_dim=128, max_conv_dim=512)).eval().to(dt)
        params = dict(se.named_parameters())
        x = mel.to(dt).clone().requires_grad_(True)
        out = se(x)
        (out * r.to(dt)).sum().backward()
        names = sorted(params)
        rec["names"] = np.array(names)
        summarize(rec, tag, params, names)
        rec[f"{tag}.out"] = out.detach().numpy()
        rec[f"{tag}.grad_mel"] = x.grad.numpy()
    return rec


def main():
    torch.set_num_threads(8)
    for B, T in ((2, 12),):
        rec = f0n_case(B, T)
        np.savez_compressed(os.path.join(HERE, f"train_f0n_T{T}_B{B}.npz"), **rec)
        print("f0n", B, T, {k: getattr(v, "shape", None) for k, v in rec.items() if not k.startswith("f32.")})
    for B, Fr in ((2, 80), (1, 97)):
        rec = style_case(B, Fr)
        np.savez_compressed(os.path.join(HERE, f"train_style_F{Fr}_B{B}.npz"), **rec)
        print("style", B, Fr, rec["f64.out"].shape)


if __name__ == "__main__":
    main()
