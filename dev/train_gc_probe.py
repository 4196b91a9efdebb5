"""Coop training step rate with Python's cyclic GC as is, frozen after warm-up (gc.freeze: the
warm-up's objects leave the collected generations), or disabled during the timed steps -- does
the collector's work show in the step (the training forward allocates many small objects)?"""
import gc
import os
import sys
import time
import types

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402

MODE = os.environ.get("GC_MODE", "default")


def timed(step, steps, warmup, env, sync, device):
    for _ in range(warmup):
        step()
    sync()
    if MODE == "freeze":
        gc.collect()
        gc.freeze()
    elif MODE == "disable":
        gc.collect()
        gc.disable()
    n0 = sum(s["collections"] for s in gc.get_stats())
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    el = time.perf_counter() - t0
    n1 = sum(s["collections"] for s in gc.get_stats())
    print(f"gc {MODE}: {steps / el:.2f} steps/s ({1e3 * el / steps:.2f} ms), {n1 - n0} collections", flush=True)
    return el, steps / el


def main():
    bench.dp.timed_frames = timed
    args = types.SimpleNamespace(workload="coop", steps=40, warmup=8)
    env = bench.dp.dp_env()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    bench.native.lib()
    bench.set_precision(bench.WORKLOADS["coop"]["precision"])
    bench.train_bench(args, env, dev)


if __name__ == "__main__":
    main()
