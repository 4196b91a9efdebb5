"""One rank of the DP launch test (tests/test_dp.py): launched by
dp.spawn -> torch.distributed.run exactly as ``bench.py --gpus N`` launches
itself, joins a gloo group, and times real decoder-head frames (the CPU
restatement of a 1-layer, 32-query CMT-L head on a 16x16 BEV map: the head
itself needs a GPU) through the same dp.timed_frames harness bench.py uses."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmt-cooperative-perception_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from projects.mmdet3d_plugin import dp  # noqa: E402
from projects.mmdet3d_plugin import synthetic as S  # noqa: E402


def main():
    from oracle import cmt_oracle as O
    out = sys.argv[1]
    env = dp.dp_env()
    dp.init(env, backend="gloo")
    torch.set_num_threads(1)
    head, cfg, _ = S.build_synthetic_head("cmt_lidar_nus", num_query=32, num_layers=1, grid_size=[128, 128, 40])
    oc, sd = O.cfg_from_head_cfg(cfg), S.head_state_dict(head)
    x = S.synthetic_bev(1, 16, 16, seed=dp.frame_seed(5, env))
    res = []

    def run():
        res.append(O.head_forward(oc, sd, x, None, [dict()], "lidar")[0]["cls_logits"].sum().item())
    elapsed, fps = dp.timed_frames(run, steps=3, warmup=1, env=env)
    with open(f"{out}.{env.rank}", "w") as f:
        json.dump(dict(rank=env.rank, world=env.world, elapsed=elapsed, fps=fps, frames=len(res),
                       checksum=res[-1]), f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
