"""Golden fixtures for the MultiPeriodDiscriminator forward (training step),
made by running the REFERENCE module in the survey container (never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_mpd.py

Imports /root/reference/Modules/discriminators.py read-only (it needs only torch and its own
Modules/utils.py), fills every parameter from the formula in stts2_mi355x/synth.py, runs
MultiPeriodDiscriminator.forward(y, y_hat) on formula waveforms and stores the scores and every
feature map as .npz DATA (tests/golden/mpd_*.npz).
"""
from __future__ import annotations

import os
import sys
import warnings

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "styletts2-lite_amd"))
sys.path.insert(0, REF)
warnings.filterwarnings("ignore")

from stts2_mi355x import synth  # noqa: E402


def import_losses():
    """losses.py imports torchaudio at module level (losses.py:4; absent here, used only by
    STFTLoss's MelSpectrogram): stub it.  feature_loss / generator_loss / discriminator_loss
    (:97-128) are plain torch."""
    import importlib.machinery
    import types
    if "torchaudio" not in sys.modules:
        ta = types.ModuleType("torchaudio")
        ta.__spec__ = importlib.machinery.ModuleSpec("torchaudio", None)  # transformers probes it
        ta.transforms = types.SimpleNamespace(MelSpectrogram=None, Resample=None)
        sys.modules["torchaudio"] = ta
        sys.modules["torchaudio.transforms"] = ta.transforms
    import losses  # noqa
    return losses


waves = synth.waves  # moved to stts2_mi355x/synth.py (GPU-side tests and tools import it from there)


def main():
    from Modules.discriminators import MultiPeriodDiscriminator
    torch.manual_seed(0)
    mpd = MultiPeriodDiscriminator().eval()
    sd = {k: torch.from_numpy(synth.synth_param("mpd." + k, tuple(v.shape))) for k, v in mpd.state_dict().items()}
    mpd.load_state_dict(sd, strict=True)
    # (B=1, T=1200): scores + feature maps 0, 3 and 5 of every period (fixture size); (B=2,
    # T=1001): scores only, with the reflect pad exercised by periods 2, 3, 5, 7 and 11
    for B, T, maps in ((1, 1200, (0, 3, 5)), (2, 1001, ())):
        y, yh = waves(B, T, 0), waves(B, T, 1)
        with torch.no_grad():
            y_d_rs, y_d_gs, fmap_rs, fmap_gs = mpd(torch.from_numpy(y), torch.from_numpy(yh))
        L = import_losses()
        rec = {"y": y, "y_hat": yh,
               "loss_fm": np.float64(L.feature_loss(fmap_rs, fmap_gs).item()),
               "loss_gen": np.float64(L.generator_loss(y_d_gs)[0].item()),
               "loss_disc": np.float64(L.discriminator_loss(y_d_rs, y_d_gs)[0].item())}
        for i in range(len(y_d_rs)):
            rec[f"score_r{i}"] = y_d_rs[i].numpy()
            rec[f"score_g{i}"] = y_d_gs[i].numpy()
            for j in maps:
                rec[f"fmap_r{i}_{j}"] = fmap_rs[i][j].numpy()
                rec[f"fmap_g{i}_{j}"] = fmap_gs[i][j].numpy()
        path = os.path.join(HERE, f"mpd_B{B}_T{T}.npz")
        np.savez_compressed(path, **rec)
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
