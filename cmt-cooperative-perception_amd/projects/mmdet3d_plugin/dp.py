"""Data-parallel frame harness.

Frames are independent units: each rank runs whole frames of its own (seeded
by ``seed + rank``), nothing is exchanged on the data path, and the only
collectives are a barrier around the timed region and one MAX all-reduce of
the elapsed time (weak scaling: the job's throughput is all ranks' frames over
the slowest rank's time).  Backend "nccl" is RCCL over xGMI on the GPU box;
the same code runs on "gloo" for the CPU tests.
"""
import os
import time
from dataclasses import dataclass

import torch
import torch.distributed as dist

__all__ = ["DPEnv", "dp_env", "init", "timed_frames", "frame_seed"]


@dataclass(frozen=True)
class DPEnv:
    world: int
    rank: int
    local_rank: int


def dp_env():
    """RANK / LOCAL_RANK / WORLD_SIZE as set by torch.distributed.run."""
    return DPEnv(int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
                 int(os.environ.get("LOCAL_RANK", "0")))


def init(env, backend="nccl", device=None):
    """Join the process group (no-op for one rank)."""
    if env.world > 1 and not dist.is_initialized():
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        dist.init_process_group(backend=backend, **kw)


def spawn(script, argv, nproc, env=None):
    """Start ``nproc`` ranks of ``script argv`` as child processes through
    torch.distributed.run on 127.0.0.1 (one process per GPU; the caller must
    not have touched the GPU) and return their exit status."""
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", script] + list(argv)
    e = dict(os.environ if env is None else env)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=e)


def frame_seed(base, env, i=0):
    """Per-rank, per-frame seed: ranks never share frames."""
    return base + env.rank + i * env.world


def timed_frames(run, *, steps, warmup, env, sync=lambda: None, device=None):
    """Warm up, then time exactly ``steps`` calls of ``run`` bracketed by a
    barrier + ``sync()`` on both sides; return (elapsed_max_over_ranks_s,
    frames_per_s_whole_job)."""
    for _ in range(warmup):
        run()
    sync()
    if env.world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    sync()
    if env.world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if env.world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, steps * env.world / elapsed
