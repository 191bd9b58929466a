"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output (stdin): one line per kernel instantiation."""
import re
import sys

cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"remark:\s+Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
    elif "error" in line:
        print(line.rstrip())
for r in rows:
    n = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", r["name"])
    print(f"{n[:70]:70s} vgpr {r.get('VGPRs', '?'):>4} agpr {r.get('AGPRs', '?'):>4} vspill {r.get('VGPRs Spill', '?'):>4} "
          f"sspill {r.get('SGPRs Spill', '?'):>4} occ {r.get('Occupancy', '?')}")
