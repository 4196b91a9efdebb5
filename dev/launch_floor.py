"""Floor of a dependent kernel launch inside a HIP graph on this box: N back-to-back
tiny cmt_cast launches (each reads the previous one's output) captured once and
replayed; prints the mean per launch.  The decoder's query side at the reference
numerics is ten dependent launches per layer, so this floor
times ten is the least that side can cost as separate kernels.

    python dev/launch_floor.py [--n 200] [--elems 256]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmt-cooperative-perception_amd"))

import torch  # noqa: E402

from projects.mmdet3d_plugin import native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--elems", type=int, default=256)
    a = ap.parse_args()
    N.lib()
    dev = torch.device("cuda")
    bufs = [torch.zeros(a.elems, dtype=torch.float32, device=dev), torch.zeros(a.elems, dtype=torch.float32, device=dev)]

    def chain():
        for i in range(a.n):
            N.cast(bufs[i & 1], bufs[(i + 1) & 1])

    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        chain()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        chain()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    e1.synchronize()
    per = e0.elapsed_time(e1) * 1e3 / reps / a.n
    print(f"graph-replayed dependent launches: {per:.2f} us per kernel ({a.n} kernels of {a.elems} elements)")


if __name__ == "__main__":
    main()
