"""HBM traffic of the bigconv family per kernel instance, with the counter calibration of
tools/calib_traffic.py applied.

    python tools/traffic_calibrated.py <pmc_root> <calib_c256.json> <calib_c128.json> <out.json>

<pmc_root> holds the FETCH_SIZE and WRITE_SIZE passes of tools/gpu/gpu_traffic.sh (one headline bench step,
HiFi-GAN bf16, B = 32 x 400 frames).  Per dispatch:
  * writes = WRITE_SIZE (calibrated exact for the epilogue's store pattern, calib mode 5);
  * reads  = FETCH_SIZE x f_win, with f_win the measured bytes-per-counted-byte of bigconv2's own
    64-B window row segments for the launch's row pitch (mode 2: 1.84 for 256-channel rows, 1.50 for
    128-channel rows), except that a residual launch's residual rows are read in the epilogue's
    32-B-per-lane pieces (mode 6): reads = (FETCH - res / f_res) x f_win + res.
The algorithmic bytes of a launch are one read of its input rows and one write of its output rows (plus
the residual / running-sum rows it reads), the §8(d) model.  Instances are named by their template
arguments <C, waves, taps, dilation, residual, running sum>.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROWS = {256: 32 * 8000, 128: 32 * 40000}  # headline workload: B = 32, stage 0 / 1 frames per utterance


def load(root, counter):
    out = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or "k_bigconv" not in r["Kernel_Name"]:
                continue
            d = (f, int(r["Dispatch_Id"]))
            if d not in out:
                out[d] = [r["Kernel_Name"], 0.0]
            out[d][1] += float(r["Counter_Value"]) * 1024.0
    return list(out.values())


def factor(cal, mode):
    return cal["modes"][str(mode)]["bytes_per_counted_byte"]


def main():
    root, c256, c128, dst = sys.argv[1:5]
    cal = {256: json.load(open(c256)), 128: json.load(open(c128))}
    fetch = load(os.path.join(root, "fetch"), "FETCH_SIZE")
    write = load(os.path.join(root, "write"), "WRITE_SIZE")
    per = defaultdict(lambda: {"n": 0, "fetch": 0.0, "write": 0.0})
    for name, v in fetch:
        per[name]["n"] += 1
        per[name]["fetch"] += v
    for name, v in write:
        per[name]["write"] += v
    res = {"workload": "hifigan bf16, B = 32 x 400 frames, one step", "instances": {}}
    tot_cal = tot_alg = tot_raw = 0.0
    # family level (every k_bigconv* dispatch): calibrated where the instance's read pattern was calibrated
    # (bigconv2 resblock convs, 256- / 128-channel rows), else the guide's x2 for wide reads
    fam_bytes, fam_n, fam_uncal = 0.0, 0, 0
    for name, d in per.items():
        m = re.search(r"k_bigconv2<(\d+), \d+, \d+, \d+, (true|false), (true|false), 0, (\d+)", name)
        C = int(m.group(1)) if m else 0
        if m and C in ROWS and int(m.group(4)) == C:
            act = ROWS[C] * C * 2
            resb = act * ((m.group(2) == "true") + (m.group(3) == "true"))
            fe = d["fetch"] / d["n"]
            rd = (fe - resb / factor(cal[C], 6)) * factor(cal[C], 2) + resb if resb else fe * factor(cal[C], 2)
            fam_bytes += (rd + d["write"] / d["n"]) * d["n"]
        else:
            fam_bytes += 2 * d["fetch"] + d["write"]
            fam_uncal += d["n"]
        fam_n += d["n"]
    for name, d in sorted(per.items()):
        m = re.search(r"k_bigconv2<(\d+), (\d+), (\d+), (\d+), (true|false), (true|false), (\d+), (\d+)", name)
        if not m:
            continue
        C, NW, K, DIL = (int(m.group(i)) for i in range(1, 5))
        RES, ACC, PRO, CINP = m.group(5) == "true", m.group(6) == "true", int(m.group(7)), int(m.group(8))
        if PRO != 0 or C not in ROWS:
            continue  # the front-end variant (1,090-channel rows): not calibrated, left out
        n = d["n"]
        fe, wr = d["fetch"] / n, d["write"] / n
        act = ROWS[C] * C * 2
        fw = factor(cal[C], 2)
        resb = act * (RES + ACC)
        reads = (fe - resb / factor(cal[C], 6)) * fw + resb if resb else fe * fw
        alg = act * (2 + RES + ACC)
        raw = 2 * fe + wr  # the uncalibrated x2 correction of round 2
        key = f"<{C}, {NW}, {K}, {DIL}, {'res' if RES else '-'}, {'acc' if ACC else '-'}>"
        res["instances"][key] = {"dispatches": n, "fetch_counter_bytes": fe, "write_bytes": wr,
                                 "reads_calibrated": reads, "hbm_calibrated": reads + wr, "algorithmic": alg,
                                 "ratio_calibrated": (reads + wr) / alg, "ratio_x2_correction": raw / alg}
        tot_cal += (reads + wr) * n
        tot_alg += alg * n
        tot_raw += raw * n
        print(f"{key:28s} x{n:3d}  calibrated {(reads + wr) / 1e6:7.1f} MB  x2-corrected {raw / 1e6:7.1f} MB  "
              f"algorithmic {alg / 1e6:7.1f} MB  ratio {(reads + wr) / alg:.3f} (x2: {raw / alg:.3f})")
    res["total"] = {"calibrated": tot_cal, "algorithmic": tot_alg, "x2_corrected": tot_raw,
                    "ratio_calibrated": tot_cal / tot_alg if tot_alg else None}
    res["calibration"] = {"window_f_c256": factor(cal[256], 2), "window_f_c128": factor(cal[128], 2),
                          "residual_f_c256": factor(cal[256], 6), "residual_f_c128": factor(cal[128], 6),
                          "store_f_c256": factor(cal[256], 5)}
    print(f"total: calibrated {tot_cal / 1e9:.2f} GB vs algorithmic {tot_alg / 1e9:.2f} GB "
          f"({tot_cal / tot_alg:.3f}); x2-corrected {tot_raw / 1e9:.2f} GB")
    res.update({"kernel": "k_bigconv", "decoder": "hifigan", "dtype": "bf16", "batch": 32, "frames": 400,
                "hbm_bytes_per_launch": fam_bytes / fam_n, "dispatches": fam_n, "dispatches_uncalibrated": fam_uncal,
                "correction": "per-pattern calibration (tools/calib_traffic.py): bigconv2 resblock launches "
                              "reads = FETCH x f_window (+ residual rows at f_residual), writes = WRITE_SIZE; "
                              "other k_bigconv* launches (front-end, v1, upsamplers) 2 x FETCH + WRITE"})
    print(f"family k_bigconv: {fam_bytes / fam_n / 1e6:.1f} MB per launch over {fam_n} dispatches "
          f"({fam_uncal} with the uncalibrated x2)")
    with open(dst, "w") as fh:
        json.dump(res, fh, indent=1)




# ---------------------------------------------------------------- round 6: every instance of the family calibrated
# 
#     python tools/traffic_calibrated.py --calib-dir <dir with c64/c128/c256/c512/c1024.json> <pmc_root> <out.json>
# Per dispatch, by instance (template arguments):
#   * bigconv2 resblock convs (PRO 0, CINP = C): reads = (FETCH - res / f6(C)) f2(C) + res, writes = WRITE f5(C);
#   * the polyphase upsamplers (UPS): reads = (FETCH - res / f8(Cout, up)) f2(Cin) + res, writes = WRITE f7(Cout, up),
#     res = the output rows of the noise-branch residual (algorithmic);
#   * the front-end k3 convs (PRO 1, CINP 1120; input rows of 514-1,090 channels): the window factor of 1,024-channel
#     rows, f2(1024); residual at f6(Cout); writes f5(Cout);
#   * bigconv v1 (C = 128 k3: 16-B coalesced staging loads): reads = FETCH f0(128), writes = WRITE f5(128).
# Algorithmic bytes (one read of the input rows, one write of the output rows, plus residual / running-sum rows) are
# known per instance for the resblocks and the upsamplers; the front-end's input width varies by launch, so its
# instances carry calibrated bytes only.
UPS_ROWS = {2560: (32 * 800, 10, 512, 256), 640: (32 * 8000, 5, 256, 128), 192: (32 * 40000, 3, 128, 64)}


def main_r06(cdir, root, dst):
    cal = {ld: json.load(open(os.path.join(cdir, f"c{ld}.json"))) for ld in (64, 128, 256, 512, 1024)}
    up_cal = {10: cal[256], 5: cal[128], 3: cal[64]}  # (modes 7 / 8 were run with halo = up at ld = Cout)
    fetch = load(os.path.join(root, "fetch"), "FETCH_SIZE")
    write = load(os.path.join(root, "write"), "WRITE_SIZE")
    per = defaultdict(lambda: {"n": 0, "fetch": 0.0, "write": 0.0})
    for name, v in fetch:
        per[name]["n"] += 1
        per[name]["fetch"] += v
    for name, v in write:
        per[name]["write"] += v
    res = {"workload": "hifigan bf16, B = 32 x 400 frames, one step", "instances": {}}
    fam, fam_n, fam_alg, alg_n = 0.0, 0, 0.0, 0
    for name, d in sorted(per.items()):
        n = d["n"]
        fe, wr = d["fetch"] / n, d["write"] / n
        m2 = re.search(r"k_bigconv2<(\d+), (\d+), (\d+), (\d+), (true|false), (true|false), (\d+), (\d+), "
                       r"(true|false), (true|false), (\d+)", name)
        m1 = re.search(r"k_bigconv<(\d+), (\d+), (\d+), (true|false)>", name)
        alg = None
        if m2:
            C, NW, K, DIL = (int(m2.group(i)) for i in range(1, 5))
            RES, ACC, PRO, CINP = m2.group(5) == "true", m2.group(6) == "true", int(m2.group(7)), int(m2.group(8))
            UPS, CO = m2.group(10) == "true", int(m2.group(11))
            if UPS:
                rows_in, up, cin, cout = UPS_ROWS[C]
                resb = rows_in * up * cout * 2
                c = up_cal[up]
                reads = (fe - resb / factor(c, 8)) * factor(cal[cin], 2) + resb
                writes = wr * factor(c, 7)
                alg = rows_in * cin * 2 + 2 * resb
                kind = f"ups <{C}, {NW}, Cin {cin}, Cout {cout}, x{up}>"
            elif PRO == 1:
                resb_f = 1.0 / factor(cal[min(CO, 1024)], 6)
                # (residual bytes unknown without the launch's rows: bound through the residual read factor of the
                # output width; the front-end's residual launches read Cout-channel rows at 400 or 800 frames)
                rows = 32 * (800 if CO == 512 else 400)
                resb = rows * CO * 2 if RES else 0
                reads = (fe - resb * resb_f) * factor(cal[1024], 2) + resb
                writes = wr * factor(cal[min(CO, 1024)], 5)
                kind = f"front <{C}, {NW}, {'res' if RES else '-'}>"
            else:
                act = ROWS[C] * C * 2
                resb = act * (RES + ACC)
                reads = (fe - resb / factor(cal[C], 6)) * factor(cal[C], 2) + resb if resb else fe * factor(cal[C], 2)
                writes = wr * factor(cal[C], 5)
                alg = act * (2 + RES + ACC)
                kind = f"<{C}, {NW}, {K}, {DIL}, {'res' if RES else '-'}, {'acc' if ACC else '-'}>"
        elif m1:
            C = int(m1.group(1))
            reads = fe * factor(cal[C], 0)
            writes = wr * factor(cal[C], 5)
            kind = f"v1 <{C}, {m1.group(2)}, {m1.group(3)}, {m1.group(4)}>"
        else:
            raise SystemExit(f"unknown k_bigconv instance: {name}")
        hbm = reads + writes
        inst = res["instances"].setdefault(kind, {"dispatches": 0, "hbm_calibrated": 0.0, "algorithmic": alg})
        inst["dispatches"] += n
        inst["hbm_calibrated"] += hbm * n
        fam += hbm * n
        fam_n += n
        if alg:
            fam_alg += alg * n
            alg_n += hbm * n
    for kind, inst in sorted(res["instances"].items()):
        inst["hbm_calibrated"] /= inst["dispatches"]
        r = f"  ratio {inst['hbm_calibrated'] / inst['algorithmic']:.3f}" if inst["algorithmic"] else ""
        alg = f"algorithmic {inst['algorithmic'] / 1e6:7.1f} MB" if inst["algorithmic"] else "algorithmic       —   "
        print(f"{kind:36s} x{inst['dispatches']:3d}  calibrated {inst['hbm_calibrated'] / 1e6:7.1f} MB  {alg}{r}")
    res["calibration"] = {f"c{ld}": {str(m): v["bytes_per_counted_byte"] for m, v in c["modes"].items()}
                          for ld, c in cal.items()}
    res.update({"kernel": "k_bigconv", "decoder": "hifigan", "dtype": "bf16", "batch": 32, "frames": 400,
                "hbm_bytes_per_launch": fam / fam_n, "dispatches": fam_n, "dispatches_uncalibrated": 0,
                "calibrated_vs_algorithmic_where_known": alg_n / fam_alg if fam_alg else None,
                "correction": "every instance by its own calibrated patterns (tools/traffic_calibrated.py main_r06)"})
    print(f"family k_bigconv: {fam / fam_n / 1e6:.1f} MB per launch over {fam_n} dispatches, all calibrated; "
          f"{alg_n / fam_alg:.3f} x algorithmic over the instances with known algorithmic bytes")
    with open(dst, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--calib-dir":
        main_r06(*sys.argv[2:5])
    else:
        main()
