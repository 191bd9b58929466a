"""Forward half of the training step at BASELINE configs[4] / SURVEY §8(d) config 5's shape (B = 2
segments of mel_len 155 -> 93,000 samples): decoder forward (y_rec = decoder(en, F0, N, s),
train.py:266), the discriminator losses' MPD + MSD forwards over (wav, y_rec) (train.py:272, 276), the
multi-resolution mel loss (train.py:282) and the GAN losses, on the HIP path.  Median hipEvent ms per
piece and in all, per dtype; the oracle (torch-CPU) for the same pieces on the host as the CPU
baseline.  Backward is not built, so this is not a training-step time.

    python tools/bench_train_fwd.py [--iters 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from helpers import make_decoder
    from stts2_mi355x import synth
    from stts2_mi355x.discriminators import MultiPeriodDiscriminator, mpd_gan_losses, msd_gan_losses
    from stts2_mi355x.losses import MultiResolutionSTFTLoss
    from test_msd_oracle import msd_module
    torch.cuda.set_device(0)
    B, T = 2, 155
    dec, cfg = make_decoder("hifigan")
    dsd = {k: v.clone() for k, v in dec.state_dict().items()}
    dec = dec.cuda()
    mpd = MultiPeriodDiscriminator()
    psd = {k: torch.from_numpy(synth.synth_param("mpd." + k, tuple(v.shape))) for k, v in mpd.state_dict().items()}
    mpd.load_state_dict(psd)
    mpd = mpd.cuda()
    msd, ssd = msd_module()
    msd = msd.cuda()
    stft = MultiResolutionSTFTLoss()
    asr, f0, n, s = (torch.from_numpy(x).cuda() for x in synth.decoder_inputs(B, T, tag="train"))
    gen = torch.Generator().manual_seed(0)
    wav = (torch.randn(B, 1, 600 * T, generator=gen) * 0.2).cuda()
    line = {"workload": f"training-step forward pieces, B = {B} segments x {600 * T} samples (config 5 shape)"}
    with torch.no_grad():
        for dtype in ("fp32", "bf16"):
            y_rec = dec(asr, f0, n, s, seed=1, dtype=dtype)
            r = {"decoder_ms": timed(lambda: dec(asr, f0, n, s, seed=1, dtype=dtype), a.iters),
                 "mpd_fwd_losses_ms": timed(lambda: mpd_gan_losses(mpd, wav, y_rec, dtype=dtype), a.iters),
                 "msd_fwd_losses_ms": timed(lambda: msd_gan_losses(msd, wav, y_rec, dtype=dtype), a.iters),
                 "mel_loss_ms": timed(lambda: stft(y_rec, wav), a.iters)}
            r["total_ms"] = sum(r.values())
            line[dtype] = r
    # CPU baseline: the oracle's same pieces on the host (one pass)
    from oracle import stts_oracle as orc
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1)
    c = [t.cpu() for t in (asr, f0, n, s)]
    w = wav.cpu()
    noise = torch.from_numpy(synth.source_noise(B, 600 * T))
    t0 = time.perf_counter()
    with torch.no_grad():
        yr = orc.decoder_hifigan(*c, dsd, cfg, noise)
        orc.gan_losses(*orc.mpd(w, yr, psd))
        orc.gan_losses(*orc.msd(w, yr, ssd))
        orc.mrstft_loss(yr, w)
    line["cpu_baseline"] = {"ms": (time.perf_counter() - t0) * 1e3, "cores": torch.get_num_threads(), "kind": "port",
                            "sample": "oracle/stts_oracle.py decoder + mpd + msd + gan_losses + mrstft_loss, fp32"}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
