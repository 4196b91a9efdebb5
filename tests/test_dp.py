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


def _shard_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "cmt-cooperative-perception_amd")]
    import torch.distributed as dist
    from projects.mmdet3d_plugin import set_precision
    from projects.mmdet3d_plugin import synthetic as S
    from projects.mmdet3d_plugin.models.dense_heads.cmt_head import CmtHead
    dist.init_process_group("gloo", rank=rank, world_size=world)
    set_precision("exact")     # fp32 GEMM policy: no compute-dtype copy of the outputs
    head, _, _ = S.build_synthetic_head("cmtcoop_lidar_tumtraf", num_query=8, num_layers=2)
    decoded = []

    def fake_decode(self, x, x_img, metas, B, out, flags, variant, prec, out16=None):
        # agent-specific values; MAX_INTO semantics of the post-norm kernel
        decoded.append(int(x[0, 0, 0, 0].item()))
        val = torch.sin(torch.arange(out.numel(), dtype=torch.float32) * (1 + x[0, 0, 0, 0])).view_as(out)
        if flags & 2:   # native.LN_MAX_INTO
            torch.maximum(out, val, out=out)
        else:
            out.copy_(val)
    CmtHead._decode_agent = fake_decode
    CmtHead._task_outputs = lambda self, outs, B, prec, outs16=None: [dict(outs=outs.clone())]
    CmtHead._check_eval = lambda self: None
    agents = [(f"agent{i}_", torch.full((1, 4, 2, 2), float(i)), None) for i in range(5)]
    single = head.forward_agents(agents, [dict()])[0]["outs"]
    n_single = len(decoded)
    decoded.clear()
    sharded = head.forward_agents(agents, [dict()], group=True)[0]["outs"]
    q.put((rank, decoded, n_single, torch.equal(single, sharded)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_agent_sharding_assignment_and_max(world):
    """forward_agents(group=...): rank r decodes agents r, r + world, ... and
    the MAX all-reduce reproduces the single-process max-fused outputs
    (the decoder itself is faked: the GPU test covers it bit-exactly)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=120) for _ in range(world)), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, dec, n_single, eq in res:
        assert n_single == 5
        assert dec == [i for i in range(5) if i % world == rank]
        assert eq
