"""Aggregate rocprofv3 --pmc counter_collection.csv files per kernel.

usage: python tools/pmc_summary.py DIR [DIR ...] [--top N]
Each DIR is a rocprofv3 -d output directory (one counter pass).  Prints, per kernel
(sorted by total duration), the dispatch count, average duration and every collected
counter averaged per dispatch, plus derived ratios when their inputs are present:
  wait%/inst%/active% = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES,
  valu/mfma = SQ_INSTS_VALU / SQ_INSTS_MFMA, bank% = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE,
  fetchMB = 2 x FETCH_SIZE (gfx950 tallies 128-B streaming requests at 64 B), writeMB = WRITE_SIZE,
  clk = GRBM_GUI_ACTIVE / 8 (sum over the XCDs) / duration, printed only for dispatches of
  >= 0.3 ms (MI355X_MICROARCH.md "DVFS give-back": the quotient reads high below that, so no
  clock is derived for shorter kernels).  Each counter is averaged over the dispatches of the
  passes that collected it (GRBM_GUI_ACTIVE is in every pass).
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
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            k = kern.setdefault(name, {"disp": collections.defaultdict(set), "dur": {},
                                       "ctr": collections.defaultdict(lambda: collections.defaultdict(float))})
            key = (f, row["Dispatch_Id"])
            k["disp"][f].add(key)
            k["dur"][key] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3
            # one row per counter instance (XCD / SE): summed, as rocprofv3 reports them
            k["ctr"][f][row["Counter_Name"]] += float(row["Counter_Value"])


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    return n[:70]


rows = []
for name, k in kern.items():
    passes = len(k["disp"])
    per = sum(len(v) for v in k["disp"].values()) / max(passes, 1)     # dispatches per pass
    # a counter collected in several passes (GRBM_GUI_ACTIVE rides along in each) is averaged
    # over the dispatches of exactly the passes that collected it, never summed across them
    tot_c, n_c = collections.defaultdict(float), collections.defaultdict(int)
    for f, cs in k["ctr"].items():
        for cn, v in cs.items():
            tot_c[cn] += v
            n_c[cn] += len(k["disp"][f])
    avg = {cn: tot_c[cn] / n_c[cn] for cn in tot_c}
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
        # effective clock = GRBM_GUI_ACTIVE / 8 XCDs / wall (MI355X_MICROARCH.md "DVFS give-back");
        # it reads high on dispatches shorter than ~0.3 ms, so none is derived for those
        us = tot / per
        d.append(f"clk {c['GRBM_GUI_ACTIVE'] / 8 / us / 1e3:4.2f} GHz" if us >= 300 else "clk n/a (<0.3 ms)")
    print(line)
    if d:
        print("      " + "  ".join(d))
