"""Full-size logit parity sweep (diagnostic; imports the oracle, so it lives in
dev/, never in the product): configs[1]-[3] x seeds x numerics variants of the
native head against the fp16-core oracle (the reference's numerics), plus the
oracle's own fp16-core vs fp32-core gap as the scale of the fp16 noise.

Variants:
  ref       -- the headline policy (split-f16 GEMMs, Q*scale*log2e as hi+lo f16)
  ref_fold  -- as ref, Q*scale*log2e rounded once to f16 (one QK^T MFMA pass)
  exact     -- exact-f32 GEMMs (v_mfma_f32_32x32x2_f32), QS core: separates the
               split-GEMM error from the attention core's

    python tests/diag/parity_sweep.py [--seeds 0 1 2] [--variants ref ref_fold] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cmt-cooperative-perception_amd")]
import torch  # noqa: E402

from oracle import cmt_oracle as O  # noqa: E402
from projects.mmdet3d_plugin import set_precision  # noqa: E402
from projects.mmdet3d_plugin import synthetic as S  # noqa: E402
from projects.mmdet3d_plugin.runtime import PRECISIONS, SPLIT, Precision  # noqa: E402

KEYS = ("center", "height", "dim", "rot", "vel", "cls_logits")
VARIANTS = {
    "ref": PRECISIONS["ref"],
    "ref_fold": Precision("ref_fold", SPLIT, torch.float16, SPLIT, True, True),
    "exact": PRECISIONS["exact"],
}
# nuScenes yaws (55 deg apart, ~10 deg overlaps) and a crowded rig in which many
# queries project into two or three views (cmt_head.py:454-466 masked view sum)
OVERLAP_YAWS = (0.0, 20.0, -20.0, 40.0, -40.0, 60.0)


def errs(got, ref):
    return {k: (got[k].detach().cpu().double() - ref[k].double()).abs().max().item() for k in KEYS}


def case(name, seed, dev):
    """(head, cfg, native forward thunk, oracle thunk(core))"""
    s = 100 * seed
    if name == "lidar":
        head, cfg, _ = S.build_synthetic_head("cmt_lidar_nus", seed=seed, num_query=900)
        oc, sd = O.cfg_from_head_cfg(cfg), S.head_state_dict(head)
        x = S.synthetic_bev(1, 180, 180, seed=41 + s)
        head.to(dev)
        xd = x.to(dev)
        return head, (lambda: head([xd], None, [dict()])), \
            (lambda core: O.head_forward(oc, sd, x, None, [dict()], "lidar", cross_core=core, epilogue=False))
    if name in ("fusion", "fusion_overlap"):
        head, cfg, _ = S.build_synthetic_head("cmt_fusion_nus", seed=seed, num_query=900)
        oc, sd = O.cfg_from_head_cfg(cfg), S.head_state_dict(head)
        x = S.synthetic_bev(1, 180, 180, seed=42 + s)
        xi = S.synthetic_img(6, 40, 100, seed=43 + s)
        metas = S.synthetic_metas(1, yaws=S.NUS_YAWS if name == "fusion" else OVERLAP_YAWS, seed=44 + s)
        head.to(dev)
        xd, xid = x.to(dev), xi.to(dev)
        return head, (lambda: head([xd], [xid], metas)), \
            (lambda core: O.head_forward(oc, sd, x, xi, metas, "fusion", cross_core=core, epilogue=False))
    if name == "coop":
        head, cfg, _ = S.build_synthetic_head("cmtcoop_fusion_tumtraf", seed=seed, num_query=900)
        oc, sd = O.cfg_from_head_cfg(cfg), S.head_state_dict(head)
        xv, xr = S.synthetic_bev(1, 180, 180, seed=45 + s), S.synthetic_bev(1, 180, 180, seed=46 + s)
        iv, ir = S.synthetic_img(1, 40, 100, seed=47 + s), S.synthetic_img(3, 40, 100, seed=48 + s)
        mv = S.synthetic_metas(1, yaws=S.VEHICLE_YAWS, prefix="vehicle_", seed=49 + s)
        mi = S.synthetic_metas(1, yaws=S.INFRA_YAWS, prefix="infrastructure_", seed=50 + s)
        metas = [dict(mv[0], **mi[0])]
        head.to(dev)
        d = [t.to(dev) for t in (xv, xr, iv, ir)]
        agents = [("vehicle_", xv, iv), ("infrastructure_", xr, ir)]
        return head, (lambda: head([d[0]], [d[1]], [d[2]], [d[3]], metas)), \
            (lambda core: O.head_coop_forward(oc, sd, agents, metas, "fusion", cross_core=core, epilogue=False))
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["lidar", "fusion", "coop", "fusion_overlap"])
    ap.add_argument("--seeds", nargs="+", type=int, default=[0, 1, 2])
    ap.add_argument("--variants", nargs="+", default=["ref", "ref_fold"])
    ap.add_argument("--no-fp32-gap", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.set_num_threads(min(16, os.cpu_count() or 8))
    dev = torch.device("cuda:0")
    rows = []
    for name in a.configs:
        for seed in a.seeds:
            t0 = time.time()
            head, fwd, oracle = case(name, seed, dev)
            head.box_epilogue = False
            ref = oracle("fp16")[0]
            row = {"config": name, "seed": seed}
            if not a.no_fp32_gap:
                ref32 = oracle("fp32")[0]
                row["oracle_fp16_vs_fp32"] = max(errs({k: ref[k] for k in KEYS}, ref32).values())
            for v in a.variants:
                set_precision(VARIANTS[v])
                try:
                    with torch.no_grad():
                        out = fwd()
                    torch.cuda.synchronize()
                finally:
                    set_precision("ref")
                got = out[0][0] if isinstance(out, tuple) else out[0]
                e = errs(got, ref)
                row[v] = max(e.values())
                row[v + "_keys"] = e
            rows.append(row)
            print(json.dumps(row), f"({time.time() - t0:.1f} s)", flush=True)
            del head
            torch.cuda.empty_cache()
    summary = {v: max(r[v] for r in rows) for v in a.variants}
    print("worst per variant:", json.dumps(summary), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"rows": rows, "worst": summary}, f, indent=1)


if __name__ == "__main__":
    main()
