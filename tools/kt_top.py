"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv (default gpurun_out/kt)."""
import csv, sys, glob
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/kt"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:n]:
    name = r["Name"].replace("(anonymous namespace)::", "")[:90]
    print(f"{float(r['TotalDurationNs'])/1e6:8.3f} ms x{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us  {name}")
