"""Agent sharding of the 4-agent CMTCoop stress shape (BASELINE configs[4];
SURVEY 8(e)'s optional second axis): each rank of a process group decodes its
own agents and ONE all_reduce(MAX) of the post-normed decoder outputs replaces
the in-process max over agents (cmt_head_coop.py:383-389).

gloo ranks (world 2 and world 4), all on cuda:0, each with the same head and
the same four agents: every rank's sharded forward must equal the
single-process 4-agent forward bit for bit, under the 'ref' policy and the
stress config's fp16 policy.  Reduced spatial size (32x32 BEV, 4 x 8x20 image
maps per agent, 2 layers, 1500 queries) so the four ranks share the card.

This file's name sorts among the first GPU tests: the ranks are spawned before
the pytest process itself touches the GPU (a process that has initialised the
GPU must not start programs on this pool)."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ("center", "height", "dim", "rot", "vel", "cls_logits")
YAWS = (0.0, 90.0, 180.0, -90.0)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "cmt-cooperative-perception_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from projects.mmdet3d_plugin import set_precision
    from projects.mmdet3d_plugin import synthetic as S
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        head, _, _ = S.build_synthetic_head("cmtcoop_fusion_tumtraf", seed=0, num_query=1500, num_layers=2,
                                            grid_size=[256, 256, 40], device=dev)
        head.box_epilogue = False
        agents, metas = [], {}
        for i in range(4):
            p = f"agent{i}_"
            x = S.synthetic_bev(1, 32, 32, seed=70 + 10 * i).to(dev)
            xi = S.synthetic_img(len(YAWS), 8, 20, seed=71 + 10 * i).to(dev)
            metas.update(S.synthetic_metas(1, yaws=YAWS, prefix=p, pad_shape=(128, 320, 3), seed=72 + 10 * i)[0])
            agents.append((p, x, xi))
        res = {}
        for prec in ("ref", "fp16"):
            set_precision(prec)
            with torch.no_grad():
                single = head.forward_agents(agents, [metas])[0]
                sharded = head.forward_agents(agents, [metas], group=True)[0]
            torch.cuda.synchronize()
            res[prec] = {k: (torch.equal(single[k], sharded[k]),
                             (single[k] - sharded[k]).abs().max().item(), sharded[k].float().abs().sum().item())
                         for k in KEYS}
        q.put((rank, res))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_agent_sharding_equals_single_process(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in range(world)), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, r in res:
        for prec, per_key in r.items():
            for k, (eq, diff, _) in per_key.items():
                assert eq, (world, rank, prec, k, diff)
    # every rank holds the same fused outputs
    for prec in ("ref", "fp16"):
        sums = {tuple(r[prec][k][2] for k in KEYS) for _, r in res}
        assert len(sums) == 1, (prec, sums)
