"""Summarise a rocprofv3 kernel-trace CSV: per-kernel totals, and the per-launch sequence of
one decoder forward (the last one in the trace)."""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    n = name.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    n = n.split("(")[0]
    for k in ("conv1d_igemm_kernel", "k_"):
        if k in n:
            return n[n.find(k):][:90]
    return n[:90]


def family(name):
    """Kernel template family (k_bigconv<256, 7, 1, false> -> k_bigconv)."""
    return re.split(r"[<I(]", short(name), maxsplit=1)[0] if short(name).startswith("k_") else \
        ("conv1d_igemm_kernel" if "conv1d_igemm_kernel" in name else short(name))


def main(path, per_step=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tot = defaultdict(lambda: [0, 0.0])
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        t = tot[short(r["Kernel_Name"])]
        t[0] += 1
        t[1] += d
    all_us = sum(v[1] for v in tot.values())
    print(f"{'kernel':90s} {'n':>6s} {'total_ms':>10s} {'avg_us':>10s} {'%':>6s}")
    for k, (n, us) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:90s} {n:6d} {us / 1e3:10.3f} {us / n:10.2f} {100 * us / all_us:6.1f}")
    fam = defaultdict(lambda: [0, 0.0])
    for k, (n, us) in tot.items():
        f = fam[family(k)]
        f[0] += n
        f[1] += us
    print(f"\n{'family':40s} {'n':>6s} {'total_ms':>10s} {'avg_us':>10s} {'%':>6s}")
    for k, (n, us) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:40s} {n:6d} {us / 1e3:10.3f} {us / n:10.2f} {100 * us / all_us:6.1f}")
    if per_step:
        seq = rows[-per_step:]
        print("\nlast forward:")
        for i, r in enumerate(seq):
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            print(f"{i:4d} {d:10.1f} us  grid={r.get('Grid_Size', r.get('Grid_Size_X', '?'))} "
                  f"lds={r.get('LDS_Block_Size', r.get('Lds_Size', '?'))} vgpr={r.get('VGPR_Count', r.get('Arch_VGPR_Count', '?'))} "
                  f"{short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
