"""Checkpoint tooling of the reference, on plain state dicts:

* `prune_for_inference` <- Demo/del_training.ipynb: keep only `ckpt['net']` and, inside it, the four
  modules inference.py loads (decoder, predictor, text_encoder, style_encoder).
* `extend_token_table` <- Extend/extend.ipynb: grow the four token-indexed tables (TextEncoder
  embedding, the ASR aligner's CTC projection, its S2S embedding and symbol projection) from the
  checkpoint's n_token rows to `extend_to`; old rows are kept, new weight rows ~ N(0, 0.01^2), new bias
  entries 0, and the result is saved in the notebook's {'net', 'optimizer', 'iters', 'val_loss',
  'epoch'} layout.

Host-side data plumbing (the reference runs these as notebooks on the CPU); checkpoints are read with
`torch.load(weights_only=True)` only.
"""
from __future__ import annotations

from collections import OrderedDict

import torch

INFERENCE_MODULES = ("decoder", "predictor", "text_encoder", "style_encoder")  # del_training.ipynb `keep`
# extend.ipynb keys_to_keep: the modules the extended checkpoint carries
TRAINING_MODULES = ("predictor", "decoder", "text_encoder", "style_encoder", "text_aligner", "pitch_extractor",
                    "mpd", "msd")
# (module, parameter prefix, has bias) of the token-indexed tables extend.ipynb resizes
TOKEN_TABLES = (
    ("text_encoder", "embedding", False),                     # models.py:257 nn.Embedding(n_symbols, C)
    ("text_aligner", "ctc_linear.2.linear_layer", True),      # Modules/ASR/models.py:28-31 LinearNorm(., n_token)
    ("text_aligner", "asr_s2s.embedding", False),             # Modules/ASR/models.py:82
    ("text_aligner", "asr_s2s.project_to_n_symbols", True),   # Modules/ASR/models.py:87
)


def load(path: str) -> dict:
    """torch.load with weights_only=True (executes nothing from the file)."""
    return torch.load(path, map_location="cpu", weights_only=True)


def prune_for_inference(ckpt: dict) -> dict:
    """Demo/del_training.ipynb: drop every top-level key but 'net' and every module of 'net' not in
    INFERENCE_MODULES.  Returns a new dict (the tensors are shared, not copied)."""
    if "net" not in ckpt:
        raise KeyError("checkpoint has no 'net' entry")
    return {"net": {k: v for k, v in ckpt["net"].items() if k in INFERENCE_MODULES}}


def _strip(sd: dict) -> "OrderedDict":
    """A module state dict without the DataParallel `module.` prefix (the reference strips it on load,
    inference.py:158-168 / extend.ipynb, and saves model[key].state_dict(), which has none)."""
    return OrderedDict((k[7:] if k.startswith("module.") else k, v) for k, v in sd.items())


def extend_token_table(ckpt: dict, extend_to: int, n_token: int | None = None,
                       generator: torch.Generator | None = None, fresh: dict | None = None) -> dict:
    """Extend/extend.ipynb on a training checkpoint: returns the notebook's saved layout with the
    token tables grown to `extend_to` rows.  `n_token` (len(symbols) + 1 from the config) defaults to
    the rows of the TextEncoder embedding; extend_to <= n_token raises ValueError as the notebook
    exits.  The new rows are drawn from `generator` (torch's default when None).

    The notebook builds all eight TRAINING_MODULES from the config and saves every one of them, so a
    module the checkpoint lacks (e.g. mpd / msd in a fine-tune checkpoint) is saved freshly
    initialised.  `fresh` (module name -> state dict of a module built from the config) supplies
    those; without it such modules are left out of the result (the notebook's layout then differs
    only by the missing entries)."""
    out = {k: _strip(v) for k, v in ckpt["net"].items() if k in TRAINING_MODULES}
    for k in TRAINING_MODULES:
        if k not in out and fresh is not None and k in fresh:
            out[k] = _strip(fresh[k])
    if n_token is None:
        n_token = out["text_encoder"]["embedding.weight"].shape[0]
    if extend_to - n_token <= 0:
        raise ValueError(f"Cannot extend from {n_token} to {extend_to}.")
    for mod, prefix, has_bias in TOKEN_TABLES:
        if mod not in out:
            continue
        sd = out[mod]
        wk = prefix + ".weight"
        w = sd[wk]
        new_w = torch.randn((extend_to, w.shape[1]), generator=generator) * 0.01
        new_w[: w.shape[0], :] = w.detach().clone()
        sd[wk] = new_w
        if has_bias:
            bk = prefix + ".bias"
            b = sd[bk]
            new_b = torch.zeros(extend_to)
            new_b[: b.shape[0]] = b.clone()
            sd[bk] = new_b
    return {"net": out, "optimizer": None, "iters": 0, "val_loss": 0, "epoch": 0}
