#!/usr/bin/env python3
"""Decoder-frame throughput of the MI355X-native CMT head (BASELINE.json metric).

Workload (BASELINE.json configs[1]): CMT-L (LiDAR-only) nuScenes-shape
synthetic frame -- BEV [1, 512, 180, 180] (= 32 400 memory tokens), 900
queries, 6-layer decoder, bf16 compute (fp32 accumulate), the whole
CmtLidarHead forward per step: shared_conv, coordinate encodings, decoder,
task heads, box epilogue.  The ~30k-point voxel scatter-mean is timed
separately.  Inputs and weights are resident in HBM before
the timed region; one step = one frame per rank, captured as a HIP graph.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
For N > 1 launch one process per GPU with torch.distributed.run; frames are
independent, so ranks share nothing on the data path (weak scaling) and the
only collectives are the barrier and the max-over-ranks of the elapsed time.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cmt-cooperative-perception_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from projects.mmdet3d_plugin import dp, native, set_precision  # noqa: E402
from projects.mmdet3d_plugin import synthetic as S  # noqa: E402
from projects.mmdet3d_plugin.mmcv_custom.ops.voxel import SPConvVoxelization  # noqa: E402
from projects.mmdet3d_plugin.profiling import region_timer  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0      # dense bf16 MFMA, MI355X_MICROARCH.md (no sparsity)
PEAK_HBM_GBS = 8000.0
C, NQ, NK, L, H = 256, 900, 32400, 6, 8


def cross_attn_flops(nq=NQ, nk=NK, c=C):
    """Algorithmic FLOPs of one cross-attention core launch (QK^T + PV), SURVEY 8(d)."""
    return 4.0 * nq * nk * c


def decoder_frame_flops(nq=NQ, nk=NK, c=C, layers=L, ffn=1024):
    """F_layer = 12 Nq C^2 + 4 Nq^2 C + 4 Nk C^2 + 4 Nq Nk C + 4 Nq C F_ffn."""
    return layers * (12 * nq * c * c + 4 * nq * nq * c + 4 * nk * c * c + 4 * nq * nk * c + 4 * nq * c * ffn)


def init_dist(args):
    env = dp.dp_env()
    if env.world > 1:
        torch.cuda.set_device(env.local_rank)
        dp.init(env, backend="nccl", device=torch.device("cuda", env.local_rank))
    return env


WORKLOADS = {
    # name: (head config, agents as (meta prefix, camera yaws or None), description)
    "lidar": ("cmt_lidar_nus", [("", None)],
              "CMT-L (LiDAR-only) nuScenes-shape: BEV 512x180x180 (32400 tokens), 900 queries, 6-layer decoder, "
              "CmtLidarHead forward (shared_conv + encodings + decoder + task heads), batch 1 frame per GPU"),
    "fusion": ("cmt_fusion_nus", [("", S.NUS_YAWS)],
               "CMT camera+LiDAR nuScenes-shape (configs[2]): BEV 512x180x180 + 6 views x 256x40x100 image feats "
               "(56400 tokens), 900 queries, 6-layer decoder, CmtHead forward, batch 1 frame per GPU"),
    "coop": ("cmtcoop_fusion_tumtraf", [("vehicle_", S.VEHICLE_YAWS), ("infrastructure_", S.INFRA_YAWS)],
             "CMTCoop TUMTraf-shape forward (configs[3] forward leg): vehicle BEV 180x180 + 1 cam, infrastructure "
             "BEV 180x180 + 3 cams (36400 + 44400 tokens), 900 queries, 6-layer decoder per agent, max fusion, "
             "CmtHeadCoop forward, batch 1 frame per GPU"),
}


def make_workload(name, seed, device=None):
    """(head, head cfg, forward closure, per-agent memory lengths, oracle closure)
    for one synthetic frame of ``name``; tensors on ``device`` (CPU if None)."""
    cfg_name, agents, _ = WORKLOADS[name]
    head, cfg, _ = S.build_synthetic_head(cfg_name, seed=0, device=device)
    inputs, nks, metas = [], [], [dict()]
    for i, (prefix, yaws) in enumerate(agents):
        x = S.synthetic_bev(1, 180, 180, seed=seed + 1 + 10 * i, device=device)
        xi = None
        if yaws is not None:
            xi = S.synthetic_img(len(yaws), 40, 100, seed=seed + 2 + 10 * i, device=device)
            m = S.synthetic_metas(1, yaws=yaws, prefix=prefix, seed=seed + 3 + 10 * i)[0]
            metas[0].update(m)
        inputs.append((prefix, x, xi))
        nks.append(180 * 180 + (0 if yaws is None else len(yaws) * 40 * 100))
    if len(agents) == 1:
        _, x, xi = inputs[0]
        fwd = lambda: head([x], [xi] if xi is not None else None, metas)  # noqa: E731
    else:
        (_, xv, iv), (_, xi_, ii) = inputs
        fwd = lambda: head([xv], [xi_], [iv], [ii], metas)  # noqa: E731

    def oracle_fwd():
        from oracle import cmt_oracle as O
        oc = O.cfg_from_head_cfg(cfg)
        sd = S.head_state_dict(head)
        cpu = [(p, x.cpu(), None if xi is None else xi.cpu()) for p, x, xi in inputs]
        variant = "lidar" if name == "lidar" else "fusion"
        if len(cpu) == 1:
            return lambda: O.head_forward(oc, sd, cpu[0][1], cpu[0][2], metas, variant)
        return lambda: O.head_coop_forward(oc, sd, cpu, metas, variant)

    return head, cfg, fwd, nks, oracle_fwd


def cpu_baseline(workload, seconds, seed):
    """The oracle (CPU restatement, fp32 exact math, PyTorch CPU) on the same
    workload, bounded to about ``seconds`` of host time."""
    _, _, _, nks, oracle_fwd = make_workload(workload, seed)
    run = oracle_fwd()
    threads = torch.get_num_threads()
    t0 = time.perf_counter()
    n = 0
    times = []
    with torch.no_grad():
        while True:
            t = time.perf_counter()
            run()
            times.append(time.perf_counter() - t)
            n += 1
            if time.perf_counter() - t0 > seconds or n >= 20:
                break
    times.sort()
    med = times[len(times) // 2]
    return {"value": round(1.0 / med, 4), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} full {workload} frames (Nq 900, memory tokens {'+'.join(map(str, nks))}, 6 layers, "
                      f"shared_conv + coordinate encodings + decoder + task heads) through oracle/cmt_oracle.py in "
                      f"fp32 on {threads} host threads; median frame time {med:.3f} s"}


def load_traffic():
    """HBM bytes per cross-attention launch from the committed rocprofv3 PMC
    summary (profiles/*pmc*.json), corrected as MI355X_MICROARCH.md prescribes
    (FETCH_SIZE x2 for wide streaming reads).  None when absent."""
    import glob
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "*attn_pmc_summary.json")))
    if not cands:
        return None
    with open(cands[-1]) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp16", "ref"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", default="lidar", choices=sorted(WORKLOADS),
                    help="lidar = BASELINE configs[1] (the headline line); fusion / coop = configs[2] / [3] forward")
    args = ap.parse_args()

    env = init_dist(args)
    world, rank, local = env.world, env.rank, env.local_rank
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    native.lib()
    set_precision(args.precision)

    head, cfg, step, nks, _ = make_workload(args.workload, seed=dp.frame_seed(0, env), device=dev)
    with torch.no_grad():
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        graph = None
        if not args.no_graph:
            graph = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                step()
                torch.cuda.synchronize()
                with torch.cuda.graph(graph):
                    static_out = step()
            torch.cuda.current_stream().wait_stream(s)
            run = graph.replay
        else:
            run = step
        elapsed, value = dp.timed_frames(run, steps=args.steps, warmup=args.warmup, env=env,
                                         sync=torch.cuda.synchronize, device=dev)

        # --- dominant kernel: cross-attention, HIP events on its launch stream
        with region_timer() as rt:
            for _ in range(3):
                step()
        attn_ms_all = rt.durations_ms("cross_attn")
        attn_ms = sum(attn_ms_all) / len(attn_ms_all)

        # --- voxel scatter-mean of ~30k points (timed separately)
        vl = SPConvVoxelization(voxel_size=[0.075, 0.075, 0.2], point_cloud_range=[-54.0, -54.0, -5.0, 54.0, 54.0, 3.0],
                                max_num_points=10, max_voxels=(120000, 160000), num_point_features=5).eval()
        pts = S.synthetic_points(30000, [-54.0, -54.0, -5.0, 54.0, 54.0, 3.0], seed=rank, device=dev)
        for _ in range(3):
            vl.forward_mean(pts)
        torch.cuda.synchronize()
        nvox = 20
        tv = time.perf_counter()
        for _ in range(nvox):
            vl.forward_mean(pts)
        torch.cuda.synchronize()
        vox_ms = (time.perf_counter() - tv) / nvox * 1e3

    ms_per_step = elapsed / args.steps * 1e3
    # mean algorithmic FLOPs of one cross-attention launch (agents may differ in Nk)
    flop_launch = sum(cross_attn_flops(nk=nk) for nk in nks) / len(nks)
    achieved = flop_launch / (attn_ms * 1e-3) / 1e12
    result = {
        "metric": "decoder frames/sec at 900 queries x (BEV+6-cam) tokens; 1/2/4/8 MI355X",
        "value": round(value, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {"bf16": "bf16", "fp16": "fp16", "ref": "fp32+fp16attn"}[args.precision],
        "data": "synthetic (seeded BEV features relu(N(0,1)), image feats N(0,1) where used, random-init weights "
                "of the head)",
        "config": {"workload": WORKLOADS[args.workload][2],
                   "global_batch": world, "seq_len": sum(nks), "parallelism": f"dp{world}",
                   "graph": graph is not None,
                   "decoder_gflop_per_frame": round(sum(decoder_frame_flops(nk=nk) for nk in nks) / 1e9, 2)},
        "roofline": {"kernel": "cmt_attn_fwd (cross-attention core, + split combine)", "bound": "mfma",
                     "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": load_traffic() if args.workload == "lidar" else None,
                     "avg_launch_ms": round(attn_ms, 5),
                     "flop_per_launch": flop_launch},
        "voxel_scatter_mean_ms": round(vox_ms, 4),
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.workload, args.cpu_seconds,
                                                seed=dp.frame_seed(0, env))
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
