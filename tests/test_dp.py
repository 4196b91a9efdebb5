"""The N > 1 bench harness on CPU: world_size-2 gloo ranks run the same
barrier / timed region / MAX all-reduce as bench.py does over RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "cmt-cooperative-perception_amd"))
    from projects.mmdet3d_plugin import dp
    env = dp.dp_env()
    dp.init(env, backend="gloo")
    import time
    calls = []

    def run():       # rank 1 is the slow rank: 20 ms per frame vs 5 ms
        time.sleep(0.02 if rank == 1 else 0.005)
        calls.append(1)
    elapsed, fps = dp.timed_frames(run, steps=5, warmup=2, env=env)
    seeds = [dp.frame_seed(100, env, i) for i in range(3)]
    q.put((rank, elapsed, fps, len(calls), seeds))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_harness_two_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, e0, f0, n0, s0), (r1, e1, f1, n1, s1) = res
    assert n0 == n1 == 7                                  # warmup + timed steps on every rank
    assert e0 == e1 and e0 >= 5 * 0.02                    # everyone reports the slowest rank's time
    assert f0 == f1 == pytest.approx(10 / e0)             # whole-job frames over the max time
    assert not set(s0) & set(s1)                          # ranks never share frame seeds


def test_dp_single_rank_no_collectives():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "cmt-cooperative-perception_amd"))
    from projects.mmdet3d_plugin import dp
    env = dp.DPEnv(1, 0, 0)
    n = []
    elapsed, fps = dp.timed_frames(lambda: n.append(1), steps=4, warmup=1, env=env)
    assert len(n) == 5 and fps == pytest.approx(4 / elapsed)
    assert not dist.is_initialized()


def test_spawned_ranks_run_head_frames(tmp_path):
    """bench.py's own N > 1 launch path (dp.spawn -> torch.distributed.run ->
    WORLD_SIZE/RANK env -> dp.init -> dp.timed_frames) at world size 2 on gloo,
    each rank timing real (CPU-oracle) head frames on its own seed."""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "cmt-cooperative-perception_amd"))
    from projects.mmdet3d_plugin import dp
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_dp_worker.py")
    out = str(tmp_path / "res")
    rc = dp.spawn(worker, [out], 2, env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert rc == 0
    r = [json.load(open(f"{out}.{i}")) for i in range(2)]
    assert [x["world"] for x in r] == [2, 2]
    assert r[0]["elapsed"] == r[1]["elapsed"]                   # max over ranks
    assert r[0]["fps"] == pytest.approx(2 * 3 / r[0]["elapsed"])   # whole-job frames / max time
    assert r[0]["frames"] == r[1]["frames"] == 4
    assert r[0]["checksum"] != r[1]["checksum"]                 # each rank its own frames
