"""MFMA utilization per kernel family from a rocprofv3 --pmc pass holding
SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (tools/gpu_sq.sh, pass "sqb").

SQ_VALU_MFMA_BUSY_CYCLES counts matrix-core busy cycles summed over every SIMD
(= 32 x N_mfma for 32x32x16 bf16, MI355X_MICROARCH.md); GRBM_GUI_ACTIVE is summed over
the 8 XCDs.  util = MFMA_BUSY / (1024 SIMDs x GRBM_GUI_ACTIVE / 8).
usage: python tools/mfma_util.py <sqb dir> [--top N]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 20
f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    k = k.split("(")[0] if not k.startswith("void") else k[:k.index(">(") + 1] if ">(" in k else k
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
rows = []
for k, c in acc.items():
    g = c.get("GRBM_GUI_ACTIVE", 0.0)
    if g <= 0 or "SQ_VALU_MFMA_BUSY_CYCLES" not in c:
        continue
    util = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * g / 8)
    rows.append((g, k, util, len(disp[k])))
rows.sort(reverse=True)
print(f"{'kernel':70s} {'launches':>8s} {'MFMA busy':>9s}")
for g, k, u, n in rows[:top]:
    print(f"{k[:70]:70s} {n:8d} {100 * u:8.1f}%")
