"""Calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on known byte counts in the conv engines' own access
patterns (csrc/calib.hip, `stts_calib_traffic`).

    python tools/calib_traffic.py run   [--rows R --ld C --tile T --halo H]   (under rocprofv3 --pmc ...)
    python tools/calib_traffic.py reduce <pmc_root_fetch> <pmc_root_write> <out.json> [same sizes]

`run` launches every mode twice on a bf16 frames buffer of rows x ld (default 2,097,152 x 256 =
1 GiB: 4x the Infinity Cache, so nothing is served on-die between launches) with a 256 MiB scrub
write between launches; `reduce` prints, per mode, the counter value (KiB) against the bytes the mode
moves, i.e. the factor that turns the counter into bytes for that pattern.
"""
import argparse
import csv
import ctypes
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd")]

MODES = {0: "coalesced 16-B loads", 1: "LDS-DMA 1 KiB", 2: "bigconv2 window 64-B segments",
         3: "bigconv2 window + halo", 4: "coalesced 16-B stores", 5: "bigconv2 epilogue stores",
         6: "bigconv2 residual loads", 7: "upsampler epilogue stores", 8: "upsampler residual loads"}


def expected_bytes(mode, rows, ld, tile, halo):
    b = rows * ld * 2
    if mode == 3:
        ntile = (rows + tile - 1) // tile
        # interior halos: 2 * halo rows per tile, minus the rows outside [0, rows) at both ends
        return b + (2 * halo * ntile - 2 * halo) * ld * 2
    return b


def run(a):
    import torch
    from stts2_mi355x import engine as E
    L = E.lib()
    L.stts_calib_traffic.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    buf = torch.zeros(a.rows * a.ld, dtype=torch.bfloat16, device="cuda")
    scrub = torch.empty(64 * 1024 * 1024, dtype=torch.float32, device="cuda")
    grid = 1024
    sink = torch.zeros(grid, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for mode in MODES:
        if mode in (7, 8) and a.rows % a.halo:
            raise SystemExit("modes 7 / 8: --rows must be a multiple of --halo (the upsampling factor)")
        for _ in range(2):
            scrub.fill_(1.0)
            r = L.stts_calib_traffic(mode, buf.data_ptr(), a.rows, a.ld, a.tile, a.halo, grid, sink.data_ptr(), s)
            if r != 0:
                raise SystemExit(f"stts_calib_traffic mode {mode}: {r}")
            torch.cuda.synchronize()
        print(f"mode {mode} ({MODES[mode]}) ok", flush=True)


def per_dispatch(root, counter):
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and "k_calib" in r["Kernel_Name"]:
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"]),
                             int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    agg = {}
    for d, v, t in rows:
        x = agg.setdefault(d, [0.0, t])
        x[0] += v
    return [agg[d] for d in sorted(agg)]


def reduce(a):
    fetch = per_dispatch(a.fetch_root, "FETCH_SIZE")
    write = per_dispatch(a.write_root, "WRITE_SIZE")
    n = len(MODES) * 2
    if len(fetch) != n or len(write) != n:
        raise SystemExit(f"expected {n} k_calib dispatches per pass, got {len(fetch)} / {len(write)}")
    res = {"rows": a.rows, "ld": a.ld, "tile": a.tile, "halo": a.halo, "modes": {}}
    for i, mode in enumerate(MODES):
        exp = expected_bytes(mode, a.rows, a.ld, a.tile, a.halo)
        fk = [fetch[2 * i + j][0] for j in range(2)]
        wk = [write[2 * i + j][0] for j in range(2)]
        us = [fetch[2 * i + j][1] / 1e3 for j in range(2)]
        writes = mode in (4, 5, 7)
        cnt = min(wk) if writes else min(fk)
        res["modes"][mode] = {
            "pattern": MODES[mode], "bytes": exp, "fetch_kib": fk, "write_kib": wk, "dispatch_us_fetch_pass": us,
            "bytes_per_counted_byte": exp / (cnt * 1024.0) if cnt else None}
        print(f"mode {mode} {MODES[mode]:32s} bytes {exp / 2**20:9.1f} MiB  FETCH {min(fk) / 1024:9.1f} MiB  "
              f"WRITE {min(wk) / 1024:9.1f} MiB  -> bytes / counter {res['modes'][mode]['bytes_per_counted_byte']:.3f}"
              f"  ({min(us):.0f} us)")
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["run", "reduce"])
    ap.add_argument("fetch_root", nargs="?")
    ap.add_argument("write_root", nargs="?")
    ap.add_argument("out", nargs="?")
    ap.add_argument("--rows", type=int, default=2 * 1024 * 1024)
    ap.add_argument("--ld", type=int, default=256)
    ap.add_argument("--tile", type=int, default=256)
    ap.add_argument("--halo", type=int, default=5)
    a = ap.parse_args()
    run(a) if a.cmd == "run" else reduce(a)


if __name__ == "__main__":
    main()
