"""Host-side profile of the coop training step (bench.py --train --workload coop): cProfile over a
few steps after warm-up, plus the step's wall time with and without a trailing device sync, to see
how much of the step is the Python thread issuing launches and waiting on host syncs."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402


def fake_timed(step, steps, warmup, env, sync, device):
    for _ in range(warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    t1 = time.perf_counter()
    sync()
    t2 = time.perf_counter()
    print(f"issue {1e3 * (t1 - t0) / steps:.2f} ms/step, with drain {1e3 * (t2 - t0) / steps:.2f} ms/step", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    sync()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(45)
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        for _ in range(3):
            step()
        sync()
    ka = prof.key_averages()
    print(ka.table(sort_by="count", row_limit=40, max_name_column_width=40))
    print(ka.table(sort_by="self_cpu_time_total", row_limit=30, max_name_column_width=40))
    kb = prof.key_averages(group_by_stack_n=3)
    print(kb.table(sort_by="count", row_limit=60, max_name_column_width=30, max_src_column_width=120))
    return t2 - t0, steps / (t2 - t0)


def main():
    bench.dp.timed_frames = fake_timed
    env = bench.dp.dp_env()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    bench.native.lib()
    bench.set_precision(bench.WORKLOADS["coop"]["precision"])
    bench.train_bench("coop", 10, 4, env, dev)


if __name__ == "__main__":
    main()
