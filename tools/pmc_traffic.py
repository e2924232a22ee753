"""Per-launch HBM traffic of one forward from rocprofv3 --pmc passes (tools/pmc_step.py).

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR [-o out.json]
Keeps the dispatches after the last FillFunctor delimiter, groups them into the kernel
families bench.py's roofline pass uses, and reports per launch:
  fetch = 2 x FETCH_SIZE (gfx950 tallies 128-B streaming read requests at 64 B;
          MI355X_MICROARCH.md "HBM"), write = WRITE_SIZE, both KiB -> bytes.
"""
import collections
import csv
import glob
import hashlib
import json
import os
import re
import sys

FAMILIES = [  # (family in bench.py's roofline pass, rocprof kernel-name regex)
    ("gemm_bf16", r"(?<![a-z])gemm\d?_kernel"),
    ("rows_gemm", r"pgemm_kernel"), ("rows_mlp", r"pmlp_kernel"), ("conv3x3", r"conv3x3_kernel|conv_ring_kernel"),
    ("attention", r"attn_kernel<[^,]+, 64,"), ("attention_window", r"attn_kernel<[^,]+, 32,"),
    ("linear_attention", r"linattn_kernel"), ("layernorm", r"rownorm_kernel"),
]


def load(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]),
                             int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    last = max((i for i, (_, n, _, _) in enumerate(rows) if "FillFunctor" in n), default=-1)
    return rows[last + 1:]


def family(name):
    for fam, rx in FAMILIES:
        if re.search(rx, name):
            return fam
    return None


def main():
    args = [a for i, a in enumerate(sys.argv[1:], 1) if not a.startswith("-") and sys.argv[i - 1] not in ("-o", "--head")]
    out = sys.argv[sys.argv.index("-o") + 1] if "-o" in sys.argv else None
    fetch = load(args[0], "FETCH_SIZE")
    write = load(args[1], "WRITE_SIZE")
    assert [n for _, n, _, _ in fetch] == [n for _, n, _, _ in write], "passes saw different dispatch sequences"
    fam = collections.OrderedDict()
    for (_, name, fv, ns), (_, _, wv, _) in zip(fetch, write):
        key = family(name) or re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))[:60]
        e = fam.setdefault(key, {"launches": 0, "fetch_bytes": 0.0, "write_bytes": 0.0, "ns": 0})
        e["launches"] += 1
        e["fetch_bytes"] += 2 * fv * 1024
        e["write_bytes"] += wv * 1024
        e["ns"] += ns
    res = {}
    for k, e in sorted(fam.items(), key=lambda kv: -kv[1]["ns"]):
        n = e["launches"]
        res[k] = {"launches": n, "fetch_bytes_per_launch": round(e["fetch_bytes"] / n),
                  "write_bytes_per_launch": round(e["write_bytes"] / n),
                  "traffic_bytes_per_launch": round((e["fetch_bytes"] + e["write_bytes"]) / n),
                  "avg_us_under_pmc": round(e["ns"] / n / 1e3, 2)}
        print(f"{k:40s} x{n:4d} fetch {res[k]['fetch_bytes_per_launch'] / 1e6:9.2f} MB  "
              f"write {res[k]['write_bytes_per_launch'] / 1e6:9.2f} MB  {res[k]['avg_us_under_pmc']:9.1f} us")
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cat-seg_amd", "cat_seg",
                       "libcatseg_hip.so")
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]
    head = sys.argv[sys.argv.index("--head") + 1] if "--head" in sys.argv else None
    if out:
        json.dump({"lib_sha16": sha, "git_head": head, "bench_config": 3,
                   "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over tools/pmc_step.py "
                             "(one L/14@336 T=150 bs=8 bf16 forward, eager); fetch = 2 x FETCH_SIZE",
                   "families": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
