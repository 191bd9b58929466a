"""Per-dispatch PMC summary of one kernel family from the rocprofv3 --pmc passes of tools/gpu/gpu_pmc.sh
(same format as profiles/r01_pmc_*.txt).

    python tools/pmc_summary.py gpurun_out/pmc [kernel-substring]

Per wave: instruction counts (SQ_INSTS_* / SQ_WAVES).  wait / winst / valu / lds: SQ_WAIT_ANY,
SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_VALU, SQ_ACTIVE_INST_LDS as % of SQ_WAVE_CYCLES.
mfmabusy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): GRBM_GUI_ACTIVE is summed
over the 8 XCDs.  bank = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.  HBM MB: FETCH_SIZE x 2 (gfx950
wide-read correction, MI355X_MICROARCH.md) + WRITE_SIZE, KiB -> MB.
"""
import csv
import glob
import re
import sys
from collections import defaultdict


def main(root, sub="k_bigconv"):
    per_pass = defaultdict(list)  # pass dir -> [(dispatch, name, dur, counters)]
    for f in sorted(glob.glob(f"{root}/*/run_counter_collection.csv")):
        acc = {}
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            e = acc.setdefault(d, [r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), {}])
            e[2][r["Counter_Name"]] = e[2].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        per_pass[f] = [(d, *acc[d]) for d in sorted(acc)]
    n = min(len(v) for v in per_pass.values())
    print(f"{sub}, one bench step ({n} dispatches); mfmabusy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 "
          "SIMDs); bank = LDS bank-conflict cycles / LDS active cycles; HBM = 2 x FETCH_SIZE + WRITE_SIZE")
    tot = defaultdict(float)
    for i in range(n):
        c, name, dur = {}, "", 0
        for v in per_pass.values():
            _, nm, du, cnt = v[i]
            c.update(cnt)
            name, dur = nm, du
        m = re.search(r"<(.*)>", name)
        args = m.group(1) if m else name[:40]
        w = c.get("SQ_WAVES", 0) or 1
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        gui = c.get("GRBM_GUI_ACTIVE", 0) or 1
        mb = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui / 8 * 1024)
        bank = c.get("SQ_LDS_BANK_CONFLICT", 0) / (c.get("SQ_LDS_IDX_ACTIVE", 0) or 1)
        hbm = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024 / 1e6
        kind = "v2" if "bigconv2" in name else ("v1" if "bigconv" in name else "")
        print(f"{i:3d} {kind} <{args}> {dur / 1e3:6.0f}us VALU/w {c.get('SQ_INSTS_VALU', 0) / w:6.0f} "
              f"MFMA/w {c.get('SQ_INSTS_MFMA', 0) / w:5.0f} LDS/w {c.get('SQ_INSTS_LDS', 0) / w:5.0f} "
              f"SALU/w {c.get('SQ_INSTS_SALU', 0) / w:6.0f} wait {100 * c.get('SQ_WAIT_ANY', 0) / wc:3.0f}% "
              f"winst {100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:3.0f}% valu {100 * c.get('SQ_ACTIVE_INST_VALU', 0) / wc:3.0f}% "
              f"mfmabusy {mb:.2f} bank {bank:.3f} HBM {hbm:6.0f} MB")
        tot["dur"] += dur
        tot["mb_w"] += mb * dur
    print(f"duration-weighted mfmabusy over the {n} dispatches: {tot['mb_w'] / max(tot['dur'], 1):.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_bigconv")
