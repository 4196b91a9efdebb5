"""Per-(kernel, grid) time table of a rocprofv3 kernel trace:
    python dev/trace_table.py gpurun_out/<tag>/trace [frames] [rows]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
frames = float(sys.argv[2]) if len(sys.argv) > 2 else None
nrows = int(sys.argv[3]) if len(sys.argv) > 3 else 30
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
agg = collections.defaultdict(list)
for r in rows:
    g = (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    agg[(r["Kernel_Name"][:70], g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in agg.values())
print(f"total kernel time {tot / 1e3:.1f} us over {sum(len(v) for v in agg.values())} launches"
      + (f" = {tot / frames / 1e3:.1f} us / {sum(len(v) for v in agg.values()) / frames:.0f} launches per frame" if frames else ""))
for (k, g), v in sorted(agg.items(), key=lambda x: -sum(x[1]))[:nrows]:
    per = f" {sum(v) / frames / 1000:7.2f}us/frame" if frames else ""
    print(f"{sum(v) / tot * 100:5.1f}% n={len(v):4d} avg={sum(v) / len(v) / 1000:7.2f}us{per} grid={'x'.join(g)} {k}")
