"""GPU busy fraction of a rocprofv3 kernel trace over its last ``steps`` steps (split at the
largest gaps is not attempted: the window is the last fraction ``tail`` of the trace), and the
idle gaps by size: python dev/trace_busy.py <trace dir> [tail=0.8]"""
import csv
import glob
import sys

d = sys.argv[1]
tail = float(sys.argv[2]) if len(sys.argv) > 2 else 0.8
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in csv.DictReader(open(f)))
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
w0 = t1 - (t1 - t0) * tail
busy, cur_s, cur_e, gaps = 0, None, None, []
prev_name = ""
for s, e, n in iv:
    if e < w0:
        continue
    s = max(s, w0)
    if cur_e is None:
        cur_s, cur_e = s, e
    elif s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, prev_name, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev_name = n
busy += cur_e - cur_s
span = t1 - w0
print(f"window {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms ({100 * busy / span:.1f} %), idle {(span - busy) / 1e6:.2f} ms")
for lo, hi in ((0, 5e3), (5e3, 2e4), (2e4, 1e5), (1e5, 1e12)):
    g = [x for x in gaps if lo <= x[0] < hi]
    print(f"gaps {lo / 1e3:6.0f}-{hi / 1e3:6.0f} us: n={len(g):5d} total {sum(x[0] for x in g) / 1e6:7.2f} ms")
for gap, a, b in sorted(gaps, reverse=True)[:25]:
    print(f"{gap / 1e3:8.1f} us after {a} before {b}")
