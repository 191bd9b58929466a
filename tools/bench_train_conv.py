"""Conv1d backward throughput (training step, config 5 shapes): dx-only and dw-only calls of
stts_conv1d_bwd, timed with HIP events.  Prints one JSON line per shape (TFLOP/s of the algorithmic
2 * B * Lq * Cout * Cin * K flops)."""
import json
import sys

import torch

sys.path.insert(0, "styletts2-lite_amd")
from stts2_mi355x import engine as E  # noqa: E402
from stts2_mi355x.training import out_length  # noqa: E402

# config 5: B = 2 segments of 93,000 samples (155 asr frames); HiFi-GAN stages (C, L) and the
# discriminators' widest convs
SHAPES = [  # (name, B, Cin, Cout, K, stride, dil, pad, Lin)
    ("front_1090_1024_k3", 2, 1090, 1024, 3, 1, 1, 1, 155),
    ("s0_256_k3_d1", 2, 256, 256, 3, 1, 1, 1, 3100),
    ("s0_256_k11_d5", 2, 256, 256, 11, 1, 5, 25, 3100),
    ("s1_128_k7_d3", 2, 128, 128, 7, 1, 3, 9, 18600),
    ("s2_64_k11_d5", 2, 64, 64, 11, 1, 5, 25, 93000),
    ("mpd_32_128_k5_s3", 10, 32, 128, 5, 3, 1, 2, 9300),
]


def main():
    L = E.lib()
    for dt in (0, 1):
        for name, B, Cin, Cout, K, s, d, p, Lin in SHAPES:
            Lq = out_length(Lin, K, s, p, d)
            x = torch.randn(B, Lin, Cin, device="cuda")
            w = torch.randn(Cout, Cin, K, device="cuda") * 0.05
            dy = torch.randn(B, Lq, Cout, device="cuda")
            dx = torch.empty_like(x)
            dw = torch.empty_like(w)
            nb = L.stts_conv1d_bwd_workspace_bytes(dt, B, Lin, Cin, Cout, K, s, d, p, Lq)
            ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
            res = {"shape": name, "dtype": ["fp32", "bf16"][dt]}
            flops = 2.0 * B * Lq * Cout * Cin * K
            for tag, args in (("dx", (dx, None)), ("dw", (None, dw))):
                if tag == "dw" and dt == 1:
                    continue  # dw is fp32 in both modes

                def call():
                    E.check(L.stts_conv1d_bwd(dt, E._ptr(x), E._ptr(w), E._ptr(dy), B, Lin, Cin, Cout, K, s, d, p,
                                              Lq, E._ptr(args[0]), E._ptr(args[1]), None, E._ptr(ws), nb,
                                              E._stream()), "bwd")
                for _ in range(3):
                    call()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                n = 10
                for _ in range(n):
                    call()
                b.record()
                torch.cuda.synchronize()
                ms = a.elapsed_time(b) / n
                res[tag + "_ms"] = round(ms, 4)
                res[tag + "_tflops"] = round(flops / ms / 1e9, 1)
            print(json.dumps(res), flush=True)


if __name__ == "__main__" and "--resblocks" not in sys.argv and "--mpd" not in sys.argv:
    main()


def bench_resblocks():
    """Forward + backward of one trainable AdaINResBlock1 (dilations 1, 3, 5) at config 5's stage shapes."""
    from stts2_mi355x.training import AdaINResBlock1
    for C, K, L in ((256, 3, 3100), (128, 7, 18600), (64, 11, 93000)):
        torch.manual_seed(0)
        mod = AdaINResBlock1(C, K, (1, 3, 5), 128).cuda()
        x = torch.randn(2, C, L, device="cuda", requires_grad=True)
        s = torch.randn(2, 128, device="cuda")
        R = torch.randn(2, C, L, device="cuda")

        def step():
            mod.zero_grad(set_to_none=True)
            x.grad = None
            (mod(x, s) * R).sum().backward()
        for _ in range(2):
            step()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            step()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 5
        flops = 3 * 2 * (2.0 * 2 * L * C * C * K)  # 6 convs: fwd + dx + dw
        print(json.dumps({"resblock": f"C{C}_K{K}_L{L}_B2", "fwd_bwd_ms": round(ms, 3),
                          "conv_tflops": round(flops / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__" and "--resblocks" in sys.argv:
    bench_resblocks()


def bench_mpd():
    """Forward + backward of the trainable MPD (periods 2, 3, 5, 7, 11) at config 5's shape: y and y_hat
    (2 x 93,000 samples each) as one batch of 4, loss = sum of squared scores + feature-map sums."""
    from stts2_mi355x.training import DiscriminatorP
    torch.manual_seed(0)
    dtype = "bf16" if "--bf16" in sys.argv else "fp32"
    ds = [DiscriminatorP(p, dtype_compute=dtype).cuda() for p in (2, 3, 5, 7, 11)]
    x = torch.randn(4, 1, 93000, device="cuda") * 0.3

    def step():
        for d in ds:
            d.zero_grad(set_to_none=True)
        loss = 0
        for d in ds:
            score, fmap = d(x)
            loss = loss + score.square().mean() + sum(f.mean() for f in fmap)
        loss.backward()
    for _ in range(2):
        step()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        step()
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"mpd_fwd_bwd": "5 periods, 4 x 93000 samples", "dtype": dtype,
                      "ms": round(a.elapsed_time(b) / 5, 3)}),
          flush=True)


if __name__ == "__main__" and "--mpd" in sys.argv:
    bench_mpd()
