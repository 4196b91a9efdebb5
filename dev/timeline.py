"""One frame's kernel timeline from a rocprofv3 kernel trace of bench.py:
start / end offsets from the frame's first kernel, duration, queue, grid, name,
and the busy/idle picture (union of kernel intervals) -- shows what the second
stream overlaps and where the critical path idles.
    python dev/timeline.py gpurun_out/<tag>/trace [frame_index_from_end]
A frame starts at the shared_conv launch (gemm_dma_kernel<...,1> / gemm_x3_kernel<256, 1> =
CONV3X3, conv_halo_x3_kernel = CONV3X3_NCHW)."""
import csv
import glob
import sys

d = sys.argv[1]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("_ZN12_GLOBAL__N_1", "")
    return n[:90]


starts = [i for i, r in enumerate(rows) if "gemm_dma_kernel" in r["Kernel_Name"]
          and ("Li1EEEv" in r["Kernel_Name"] or "Li1ELb" in r["Kernel_Name"])
          or "gemm_x3_kernel<256, 1>" in r["Kernel_Name"] or "conv_halo_x3_kernel" in r["Kernel_Name"]]
if len(starts) < back + 1:
    sys.exit(f"only {len(starts)} frames in the trace")
i0, i1 = starts[-back - 1], starts[-back]
frame = rows[i0:i1]
# the side stream's first kernels may start just before the conv: take kernels
# that start before the conv but end after the previous frame's last one
t0 = frame[0]["s"]
pre = [r for r in rows[max(0, i0 - 40):i0] if r["s"] >= rows[i0 - 1]["s"] and r is not rows[i0 - 1]]
frame = pre + frame
t0 = min(r["s"] for r in frame)
qcol = "Queue_Id" if "Queue_Id" in frame[0] else ("Stream_Id" if "Stream_Id" in frame[0] else None)
print(f"{'start':>8} {'end':>8} {'dur':>7}  q  grid        kernel")
for r in frame:
    q = r[qcol] if qcol else "?"
    g = f"{r['Grid_Size_X']}"
    print(f"{(r['s'] - t0) / 1e3:8.2f} {(r['e'] - t0) / 1e3:8.2f} {(r['e'] - r['s']) / 1e3:7.2f} {q:>2}  {g:>10}  "
          f"{short(r['Kernel_Name'])}")
# busy union
iv = sorted((r["s"], r["e"]) for r in frame)
busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = max(r["e"] for r in frame) - t0
ksum = sum(r["e"] - r["s"] for r in frame)
print(f"frame span {span / 1e3:.2f} us, busy (union) {busy / 1e3:.2f} us, idle {(span - busy) / 1e3:.2f} us, "
      f"kernel time sum {ksum / 1e3:.2f} us, {len(frame)} kernels")
