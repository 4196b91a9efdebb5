"""Busy / idle picture of the training step from a rocprofv3 kernel trace of
bench.py --train: per step (delimited by the shared_conv forward of the first
agent) the span, the union of kernel intervals, and the largest idle gaps with
the kernels either side -- where the GPU waits on the Python thread.
    python dev/train_gaps.py gpurun_out/<tag>/trace"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("_ZN12_GLOBAL__N_1", "").replace("void ", "")[:60]


starts = [i for i, r in enumerate(rows) if "gemm_x3_kernel<256, 1>" in r["Kernel_Name"]]
starts = starts[::2]   # two agents' convs per step
for a, b in zip(starts[-4:-1], starts[-3:]):
    st = rows[a:b]
    t0, t1 = st[0]["s"], st[-1]["e"]
    busy, cs, ce = 0, st[0]["s"], st[0]["e"]
    gaps = []
    prev = st[0]
    for r in st[1:]:
        if r["s"] > ce:
            busy += ce - cs
            gaps.append((r["s"] - ce, prev, r))
            cs, ce = r["s"], r["e"]
        elif r["e"] > ce:
            ce = r["e"]
        if r["e"] >= prev["e"]:
            prev = r
    busy += ce - cs
    small = sum(g for g, _, _ in gaps if g < 20000)
    print(f"step span {(t1 - t0) / 1e3:.0f} us, busy {busy / 1e3:.0f} us, idle {(t1 - t0 - busy) / 1e3:.0f} us "
          f"({len(gaps)} gaps; gaps < 20 us sum {small / 1e3:.0f} us), {len(st)} kernels")
    for g, p, n in sorted(gaps, key=lambda x: -x[0])[:8]:
        print(f"   gap {g / 1e3:8.1f} us at +{(p['e'] - t0) / 1e3:8.0f}: {short(p['Kernel_Name'])} -> {short(n['Kernel_Name'])}")
