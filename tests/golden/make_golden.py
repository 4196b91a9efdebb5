"""Generate the golden fixtures under tests/golden/ from the CPU restatement
(oracle/) on seeded synthetic inputs ("the CPU restatement's
outputs on seeded inputs are committed as small fixtures and used to check the
HIP path").

Only data is stored: the case descriptor (config name, shapes, seeds -- the
inputs and the random-init weights are regenerated from these seeds by
projects/mmdet3d_plugin/synthetic.py on the CPU torch RNG) and the expected
outputs of the last decoder layer for both reference numerics ('fp16' flash
core) and exact fp32 math, and the task heads' logits of every decoder layer
(no box epilogue) for both.  Reference outputs cannot be produced here: running
the reference was refused by the environment; parity stays
"unpinned" in that sense, and these fixtures pin the oracle against drift and
carry it to the GPU box.

    python tests/golden/make_golden.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "cmt-cooperative-perception_amd"))

from oracle import cmt_oracle as O  # noqa: E402
from projects.mmdet3d_plugin import synthetic as S  # noqa: E402

KEYS = ("center", "height", "dim", "rot", "vel", "cls_logits")


def host_fingerprint():
    """What decides the host's fp32 matmul rounding: CPU model, torch build,
    intra-op threads.  The fixtures are bit-exact on the host that made them
    (test_golden.py checks them with zero tolerance there)."""
    import platform
    model = platform.processor()
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), model)
    except OSError:
        pass
    return {"cpu": model, "torch": torch.__version__.split("+")[0], "threads": torch.get_num_threads()}

CASES = {
    "lidar_q32_l1": dict(name="cmt_lidar_nus", variant="lidar", num_query=32, num_layers=1, grid=[128, 128, 40],
                         B=1, cams=0),
    "fusion_q32_l2": dict(name="cmt_fusion_nus", variant="fusion", num_query=32, num_layers=2, grid=[128, 128, 40],
                          B=1, cams=2),
    "coop_lidar_q24_l1": dict(name="cmtcoop_lidar_tumtraf", variant="coop_lidar", num_query=24, num_layers=1,
                              grid=[128, 128, 40], B=1, cams=0),
}


def case_inputs(c):
    """Regenerate head, state_dict, inputs and metas of a fixture case (CPU)."""
    head, cfg, _ = S.build_synthetic_head(c["name"], seed=0, num_query=c["num_query"], num_layers=c["num_layers"],
                                          grid_size=c["grid"])
    head.eval()
    sd = S.head_state_dict(head)
    H, W = c["grid"][0] // 8, c["grid"][1] // 8
    x = S.synthetic_bev(c["B"], H, W, seed=1)
    xi = S.synthetic_img(c["B"] * c["cams"], 8, 20, seed=2) if c["cams"] else None
    if c["variant"] == "coop_lidar":
        x2 = S.synthetic_bev(c["B"], H, W, seed=4)
        metas = [dict() for _ in range(c["B"])]
        return head, cfg, sd, (x, x2), None, metas
    metas = S.synthetic_metas(c["B"], yaws=S.NUS_YAWS[:max(c["cams"], 1)], pad_shape=(128, 320, 3), seed=3)
    return head, cfg, sd, x, xi, metas


def oracle_outputs(c, core, epilogue=True):
    """Per task, the dict of [L, B, Nq, k] outputs: after the box epilogue (center / height
    sigmoid-scaled to pc_range) or, with epilogue=False, the task heads' logits."""
    head, cfg, sd, x, xi, metas = case_inputs(c)
    oc = O.cfg_from_head_cfg(cfg)
    if c["variant"] == "coop_lidar":
        agents = [("vehicle_", x[0], None), ("infrastructure_", x[1], None)]
        out = O.head_coop_forward(oc, sd, agents, metas, "lidar", cross_core=core, self_core="fp32",
                                  epilogue=epilogue)
    else:
        out = O.head_forward(oc, sd, x, xi, metas, c["variant"], cross_core=core, self_core="fp32",
                             epilogue=epilogue)
    return out


def make_voxel_fixture(path):
    from oracle import __file__ as _of  # noqa: F401
    lib_path = os.path.join(ROOT, "oracle", "_build", "libvoxel_oracle.so")
    if not os.path.exists(lib_path):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = ctypes.CDLL(lib_path)
    rng = np.random.default_rng(7)
    N = 3000
    pc = np.array([-54, -54, -5, 54, 54, 3], np.float32)
    pts = np.empty((N, 5), np.float32)
    pts[:, :3] = rng.uniform(pc[:3] - 2, pc[3:] + 2, size=(N, 3))      # some out of range
    pts[:, 3] = rng.uniform(0, 255, N)
    pts[:, 4] = rng.uniform(0, 0.5, N)
    pts[N // 2:N // 2 + 40, :3] = pts[N // 2, :3]                       # one overfull voxel
    vsize = np.array([0.6, 0.6, 0.8], np.float32)                     # 180 x 180 x 10 grid
    grid = np.array([180, 180, 10], np.int32)
    maxp, maxv = 10, 1500                                              # voxel budget binds
    v = np.zeros((maxv, maxp, 5), np.float32)
    co = np.zeros((maxv, 3), np.int32)
    n = np.zeros((maxv,), np.int32)
    m = np.zeros((maxv, 5), np.float32)
    fp, ip = ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)
    M = lib.cmt_oracle_voxelize(pts.ctypes.data_as(fp), N, 5, vsize.ctypes.data_as(fp), pc.ctypes.data_as(fp),
                                grid.ctypes.data_as(ip), maxp, maxv, 5, v.ctypes.data_as(fp), co.ctypes.data_as(ip),
                                n.ctypes.data_as(ip), m.ctypes.data_as(fp))
    np.savez_compressed(path, points=pts, voxel_size=vsize, coors_range=pc, grid=grid, max_points=maxp,
                        max_voxels=maxv, num_voxels=M, voxels=v[:M], coors=co[:M], num_points=n[:M], means=m[:M])
    return M


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    index = {"cases": {}, "kat_pos2embed": {}, "host": host_fingerprint()}
    for cname, c in CASES.items():
        arrs = {}
        for core in ("fp16", "fp32"):
            out = oracle_outputs(c, core)
            for t, task in enumerate(out):
                for k in KEYS:
                    arrs[f"{core}.{t}.{k}"] = task[k][-1].detach().cpu().numpy().astype(np.float32)   # last layer
            # the task heads' logits of EVERY decoder layer (no box epilogue): the north_star's
            # 1e-3-abs parity target
            for t, task in enumerate(oracle_outputs(c, core, epilogue=False)):
                for k in KEYS:
                    arrs[f"logits.{core}.{t}.{k}"] = task[k].detach().cpu().numpy().astype(np.float32)
        np.savez_compressed(os.path.join(HERE, f"{cname}.npz"), **arrs)
        index["cases"][cname] = c
        print(cname, {k: v.shape for k, v in list(arrs.items())[:3]})
    # pos2embed KATs at a few points (closed form, F = 256)
    pts = [[0.4963, 0.7682], [0.0, 1.0], [0.25, 0.125]]
    pe = O.pos2embed(torch.tensor(pts, dtype=torch.float32), 256)
    index["kat_pos2embed"] = {"pos": pts, "F": 256, "cols": [0, 1, 2, 3, 254, 255, 256, 257, 511],
                              "values": pe[:, [0, 1, 2, 3, 254, 255, 256, 257, 511]].tolist()}
    index["voxel"] = {"num_voxels": int(make_voxel_fixture(os.path.join(HERE, "voxel_3k.npz")))}
    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump(index, f, indent=1)


if __name__ == "__main__":
    main()
