"""Where the coop training step's torch glue ops come from: runs a few steps of bench.train_bench's
step under torch.profiler (with_stack) and prints, per aten op, the call counts per step by the
innermost frame in this repository (forward ops) or by the autograd node that ran them (backward).
    python dev/train_op_sources.py"""
import collections
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402

OPS = ("aten::add", "aten::add_", "aten::mul", "aten::fill_", "aten::zero_", "aten::copy_", "aten::cat",
       "aten::div", "aten::sub", "aten::where", "aten::index", "aten::index_put_", "aten::sum", "aten::stack",
       "aten::clone", "aten::masked_fill", "aten::nonzero", "aten::item", "aten::_local_scalar_dense")
NSTEP = 3


def fake_timed(step, steps, warmup, env, sync, device):
    for _ in range(warmup):
        step()
    sync()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        for _ in range(NSTEP):
            step()
        sync()
    counts = collections.defaultdict(collections.Counter)
    parent = {}
    evs = prof.events()
    for e in evs:
        for c in e.cpu_children:
            parent[id(c)] = e
    for e in evs:
        if e.name not in OPS:
            continue
        where = None
        for fr in e.stack or []:
            if "repo/" in fr and "torch/" not in fr:
                where = fr.split("repo/")[-1]
                break
        if where is None:
            p = parent.get(id(e))
            while p is not None and where is None:
                if "Backward" in p.name or p.name.startswith("autograd::engine"):
                    where = "bwd: " + p.name.replace("autograd::engine::evaluate_function: ", "")
                p = parent.get(id(p))
        counts[e.name][where or "?"] += 1
    for op in OPS:
        if op not in counts:
            continue
        tot = sum(counts[op].values())
        print(f"{op}: {tot / NSTEP:.0f} per step")
        for w, n in counts[op].most_common(12):
            print(f"    {n / NSTEP:6.1f}  {w}")
    return 1.0, 1.0


def main():
    bench.dp.timed_frames = fake_timed
    env = bench.dp.dp_env()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    bench.native.lib()
    bench.set_precision(bench.WORKLOADS["coop"]["precision"])
    bench.train_bench("coop", 3, 3, env, dev)


if __name__ == "__main__":
    main()
