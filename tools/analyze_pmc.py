"""Pivot rocprofv3 --pmc counter CSVs (several passes) by dispatch and print derived metrics."""
import csv
import glob
import sys
from collections import defaultdict


def load(root):
    D = defaultdict(dict)
    meta = {}
    for f in glob.glob(f"{root}/*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"][:120], int(r["Grid_Size"]))
            d = int(r["Dispatch_Id"])
            D[(f, d)][r["Counter_Name"]] = D[(f, d)].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta[(f, d)] = (key, int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return D, meta


def main(root, nlast=120):
    D, meta = load(root)
    # align passes by order of conv dispatches within each file
    per_file = defaultdict(list)
    for (f, d) in sorted(D):
        per_file[f].append((d, D[(f, d)], meta[(f, d)]))
    files = sorted(per_file)
    n = min(len(v) for v in per_file.values())
    rows = []
    for i in range(n):
        c = {}
        name, dur = None, 0
        for f in files:
            d, cnt, (key, du) = per_file[f][i]
            c.update(cnt)
            name = key[0]
            dur = du
        rows.append((name, dur, c))
    rows = rows[-nlast:]
    # wait% (SQ_WAIT_ANY: parked on s_waitcnt / barrier) + winst% (issue stalls) + active ~ 100 %
    # mfma% = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 256 CUs x 4 SIMDs), GB/s = (FETCH x2 + WRITE) / dur
    hdr = "idx  dur_us  cfg                    waveCyc  valu%  lds%  wait%  winst%  mfma%  bankc  FETCH_MB WRITE_MB  GB/s"
    print(hdr)
    for i, (name, dur, c) in enumerate(rows):
        cfg = name.split("conv1d_igemm_kernel")[-1][:22] if "conv1d" in name else name[:22]
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1  # quad-cycles, like SQ_WAIT_* / SQ_ACTIVE_INST_*
        act = c.get("SQ_ACTIVE_INST_ANY", 0)
        gui = c.get("GRBM_GUI_ACTIVE", 0) or 1
        mb = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        fetch = c.get("FETCH_SIZE", 0) * 1024 * 2 / 1e6  # gfx950: x2 for wide streaming reads
        write = c.get("WRITE_SIZE", 0) * 1024 / 1e6
        print(f"{i:3d} {dur / 1e3:7.1f} {cfg:22s} {wc / 1e6:8.1f} {100 * c.get('SQ_ACTIVE_INST_VALU', 0) / wc:5.1f} "
              f"{100 * c.get('SQ_ACTIVE_INST_LDS', 0) / wc:5.1f} {100 * c.get('SQ_WAIT_ANY', 0) / wc:5.1f} "
              f"{100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:5.1f} {100 * mb / (gui * 256 * 4 + 1e-9):6.1f} "
              f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / 1e6:6.2f} {fetch:8.1f} {write:8.1f} {(fetch + write) * 1e6 / max(dur, 1):6.0f}")
    keys = sorted(rows[-1][2].keys())
    print("counters:", keys)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 120)
