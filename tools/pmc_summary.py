"""Aggregate rocprofv3 --pmc counter_collection.csv files per kernel.

usage: python tools/pmc_summary.py DIR [DIR ...] [--top N]
Each DIR is a rocprofv3 -d output directory (one counter pass).  Prints, per kernel
(sorted by total duration), the dispatch count, average duration and every collected
counter averaged per dispatch, plus derived ratios when their inputs are present:
  wait%/inst%/active% = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES,
  valu/mfma = SQ_INSTS_VALU / SQ_INSTS_MFMA, bank% = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE,
  fetchMB = 2 x FETCH_SIZE (gfx950 tallies 128-B streaming requests at 64 B), writeMB = WRITE_SIZE.
"""
import collections
import csv
import glob
import os
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
top = 25
if "--top" in sys.argv:
    top = int(sys.argv[sys.argv.index("--top") + 1])

kern = collections.OrderedDict()
for d in args:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            k = kern.setdefault(name, {"disp": set(), "dur": {}, "ctr": collections.defaultdict(float)})
            key = (f, row["Dispatch_Id"])
            k["disp"].add(key)
            k["dur"][key] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3
            k["ctr"][row["Counter_Name"]] += float(row["Counter_Value"])


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    return n[:70]


rows = []
for name, k in kern.items():
    nd = len(k["disp"])
    # counters are summed over every pass's dispatches: average per dispatch of the pass
    # that collected them (each pass saw the same dispatch sequence)
    passes = len({key[0] for key in k["disp"]})
    per = nd / max(passes, 1)
    avg = {c: v / per for c, v in k["ctr"].items()}
    rows.append((sum(k["dur"].values()) / max(passes, 1), name, per, avg))
rows.sort(key=lambda r: -r[0])
for tot, name, per, c in rows[:top]:
    line = f"{tot / 1e3:8.3f} ms x{per:5.0f} {tot / per:9.1f} us  {short(name)}"
    d = []
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for key, lab in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "inst"), ("SQ_ACTIVE_INST_ANY", "act")):
            if key in c:
                d.append(f"{lab} {100 * c[key] / wc:4.1f}%")
    if c.get("SQ_INSTS_MFMA"):
        d.append(f"valu/mfma {c.get('SQ_INSTS_VALU', 0) / c['SQ_INSTS_MFMA']:5.2f} lds/mfma {c.get('SQ_INSTS_LDS', 0) / c['SQ_INSTS_MFMA']:5.2f}")
    elif "SQ_INSTS_VALU" in c:
        d.append(f"valu {c['SQ_INSTS_VALU']:.3g}")
    if c.get("SQ_LDS_IDX_ACTIVE"):
        d.append(f"bank {100 * c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE']:4.1f}%")
    if "FETCH_SIZE" in c:
        d.append(f"fetch {2 * c['FETCH_SIZE'] / 1024:8.1f} MB")   # FETCH_SIZE is in KB
    if "WRITE_SIZE" in c:
        d.append(f"write {c['WRITE_SIZE'] / 1024:8.1f} MB")
    if c.get("GRBM_GUI_ACTIVE"):
        d.append(f"clk {c['GRBM_GUI_ACTIVE'] / 8 / (tot / per) / 1e3:4.2f} GHz")
    print(line)
    if d:
        print("      " + "  ".join(d))
