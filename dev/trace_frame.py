"""Timeline of one frame of a rocprofv3 kernel trace (start offset, duration,
queue) -- which kernels overlap and which sit on the critical path:
    python dev/trace_frame.py gpurun_out/<tag>/trace <first-kernel-substring> [frame]"""
import csv
import glob
import sys

d, anchor = sys.argv[1], sys.argv[2]
which = int(sys.argv[3]) if len(sys.argv) > 3 else -3
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
i0, i1 = starts[which], starts[which + 1] if which + 1 < len(starts) and which != -1 else len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
busy_end = t0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - busy_end) / 1000
    busy_end = max(busy_end, e)
    name = r["Kernel_Name"].replace("_ZN12_GLOBAL__N_1", "").replace("(anonymous namespace)::", "")[:60]
    print(f"{(s - t0) / 1000:8.1f} {(e - s) / 1000:7.1f}us q{r['Queue_Id']:>2} gap {gap:6.1f} "
          f"grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']} lds={r['LDS_Block_Size']} {name}")
print(f"frame span {(busy_end - t0) / 1000:.1f} us")
