"""Probe: return codes of the conv engine test hook vs stts_conv1d_fwd for a few shapes."""
import ctypes
import sys

import torch

sys.path.insert(0, "styletts2-lite_amd")
from stts2_mi355x import engine as E  # noqa: E402
from stts2_mi355x.training import out_length  # noqa: E402

L = E.lib()
L.stts_test_conv1d.restype = ctypes.c_int
for (B, Cin, Cout, K, s, d, p, Lin) in [(2, 1090, 1024, 3, 1, 1, 1, 40), (2, 1090, 512, 3, 1, 1, 1, 40),
                                        (2, 1, 1, 3, 2, 1, 1, 80), (2, 16, 1, 3, 2, 1, 1, 80)]:
    Lq = out_length(Lin, K, s, p, d)
    x = torch.randn(B, Lin, Cin, device="cuda")
    w = torch.randn(Cout, Cin, K, device="cuda")
    y = torch.empty(B, Lq, Cout, device="cuda")
    for dt in (0, 1):
        for pm in (0, 5):
            gb = torch.ones(B, 2 * Cin, device="cuda")
            rc = L.stts_test_conv1d(dt, E._ptr(x), B, Lin, Cin, E._ptr(w), None, Cout, K, 0, s, d, p, 0, pm,
                                    E._ptr(gb), None, ctypes.c_float(0.2), None, ctypes.c_float(1.0), E._ptr(y),
                                    Lq, None)
            print("test hook", (B, Cin, Cout, K, s, d, p, Lin), "dt", dt, "pro", pm, "rc", rc, flush=True)
        nb = L.stts_conv1d_fwd_workspace_bytes(dt, B, Lin, Cin, Cout, K, s, d, p, Lq)
        ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
        rc = L.stts_conv1d_fwd(dt, E._ptr(x), E._ptr(w), None, B, Lin, Cin, Cout, K, s, d, p, Lq, E._ptr(y),
                               E._ptr(ws), nb, E._stream())
        print("fwd", (B, Cin, Cout, K, s, d, p, Lin), "dt", dt, "rc", rc, flush=True)
torch.cuda.synchronize()
