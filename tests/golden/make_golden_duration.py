"""Golden fixtures for the duration / text path, made by running the
REFERENCE TextEncoder and ProsodyPredictor (models.py) in the survey container:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_duration.py

Weights, tokens, styles and alignments come from the formulas of stts2_mi355x/synth.py, so the
GPU box regenerates the inputs without the reference; the fixtures hold DATA only (inputs'
lengths and the reference's outputs).  Cases use ragged batches so the pack_padded_sequence
semantics and the masks are exercised.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import fill, import_models  # noqa: E402

sys.path.insert(0, os.path.dirname(HERE))
from helpers import DURATION_CASES as CASES, duration_inputs as case_inputs  # noqa: E402

def run(T, lengths):
    models = import_models()
    te = fill(models.TextEncoder(channels=512, kernel_size=5, depth=3, n_symbols=178), "te.").eval()
    pp = fill(models.ProsodyPredictor(style_dim=128, d_hid=512, nlayers=3, max_dur=50, dropout=0.2), "pp.").eval()
    tok, ln, s, aln = case_inputs(T, lengths)
    tok_t, ln_t = torch.from_numpy(tok), torch.from_numpy(ln)
    m = pp.length_to_mask(ln_t)
    with torch.no_grad():
        t_en = te(tok_t, ln_t, m)
        d = pp.text_encoder(t_en, torch.from_numpy(s), ln_t, m)
        duration, en = pp(t_en, torch.from_numpy(s), ln_t, torch.from_numpy(aln), m)
        x, _ = pp.lstm(d)  # inference.py:246: no packing
        dur_inf = torch.sigmoid(pp.duration_proj(x)).sum(-1)
        asr = t_en @ torch.from_numpy(aln)
    return {"lengths": ln, "t_en": t_en.numpy(), "d": d.numpy(), "duration": duration.numpy(), "en": en.numpy(),
            "dur_inference": dur_inf.numpy(), "asr": asr.numpy()}


def main():
    torch.set_num_threads(8)
    meta_path = os.path.join(HERE, "meta.json")
    meta = json.load(open(meta_path))
    for T, lengths in CASES:
        r = run(T, lengths)
        name = f"duration_T{T}_B{len(lengths)}"
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **r)
        meta["cases"][name] = {"kind": "duration", "T": T, "lengths": list(lengths), "keys": sorted(r.keys()),
                               "generator": "tests/golden/make_golden_duration.py",
                               "param_prefixes": {"TextEncoder": "te.", "ProsodyPredictor": "pp."}}
        print(name, {k: v.shape for k, v in r.items()}, flush=True)
    with open(meta_path, "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
