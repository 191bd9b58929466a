"""HBM traffic per launch of one kernel from rocprofv3 --pmc passes (tools/gpu/gpu_traffic.sh).

    python tools/pmc_traffic.py <pmc_root> <kernel> <out.json> [--decoder hifigan --dtype bf16 --batch 32 --frames 400]

<kernel> is a kernel-name substring, or bench.py's family label "k_bigconv2[SP]" (the split-operand instances).

FETCH_SIZE and WRITE_SIZE come from separate passes (they share the TCC counter budget).
Both are in KiB.  On gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) streaming
read (MI355X_MICROARCH.md, HBM section), so reads are doubled:
    traffic = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024   bytes per launch
averaged over every dispatch of the kernel in the run.  bench.py picks the JSON up as
roofline.traffic when kernel / decoder / dtype / batch / frames match its workload.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def _is_sp(name):
    """bigconv2's split-operand (accuracy mode) instances: template argument 13 (SP) is true."""
    if "k_bigconv2<" not in name:
        return False
    args = name[name.index("<") + 1:name.rindex(">")].split(", ")
    return len(args) >= 16 and args[12] == "true"


def per_dispatch(root, counter, kernel):
    vals = defaultdict(float)
    dur = {}
    sp = kernel.endswith("[SP]")  # bench.py's family label of the split-operand bigconv2 launches
    sub = kernel[:-4] if sp else kernel
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or sub not in r["Kernel_Name"] or (sp and not _is_sp(r["Kernel_Name"])):
                continue
            d = (f, int(r["Dispatch_Id"]))
            vals[d] += float(r["Counter_Value"])
            dur[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return vals, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("kernel")
    ap.add_argument("out")
    ap.add_argument("--decoder", default="hifigan")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--frames", type=int, default=400)
    a = ap.parse_args()
    fetch, dur = per_dispatch(a.root, "FETCH_SIZE", a.kernel)
    write, _ = per_dispatch(a.root, "WRITE_SIZE", a.kernel)
    if not fetch or not write:
        raise SystemExit(f"no FETCH_SIZE / WRITE_SIZE rows for {a.kernel} under {a.root}")
    nf, nw = len(fetch), len(write)
    rd = 2.0 * 1024.0 * sum(fetch.values()) / nf
    wr = 1024.0 * sum(write.values()) / nw
    res = {"kernel": a.kernel, "decoder": a.decoder, "dtype": a.dtype, "batch": a.batch, "frames": a.frames,
           "dispatches": nf, "dispatches_fetch_pass": nf, "dispatches_write_pass": nw,
           "read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
           "avg_dispatch_us_fetch_pass": sum(dur.values()) / len(dur) / 1e3,
           "correction": "reads = 2 x FETCH_SIZE KiB (gfx950 wide-read halving), writes = WRITE_SIZE KiB"}
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
