"""Phase timing of the split row-block chains (rowchain_x3.hip) from the
diagnostic build's s_memtime stamps (CMT_STAMPS): wave 0 of the first 16
workgroups of the last launch of each chain kind.
    make -C cmt-cooperative-perception_amd/csrc OUT=../lib_stamps HIPFLAGS="... -DCMT_STAMPS"
    CMT_HIP_LIB=cmt-cooperative-perception_amd/lib_stamps/libcmt_hip.so python dev/chain_stamps.py"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, "cmt-cooperative-perception_amd")
from projects.mmdet3d_plugin import native, set_precision  # noqa: E402
from projects.mmdet3d_plugin import synthetic as S  # noqa: E402

dev = torch.device("cuda")
set_precision("ref")
head, cfg, _ = S.build_synthetic_head("cmt_fusion_nus", seed=0, num_query=900, device=dev)
x = S.synthetic_bev(1, 180, 180, seed=1).to(dev)
xi = S.synthetic_img(6, 40, 100, seed=2).to(dev)
metas = S.synthetic_metas(1, yaws=S.NUS_YAWS, seed=3)
with torch.no_grad():
    for _ in range(5):
        head([x], [xi], metas)
torch.cuda.synchronize()
L = native.lib()
fn = L.cmt_debug_chain_stamps
fn.argtypes = [ctypes.c_void_p]
buf = np.zeros((3, 16, 16), dtype=np.uint64)
rc = fn(buf.ctypes.data)
assert rc == 0, rc
names = {0: ["entry", "prologue issued", "prologue barrier", "out_proj", "LN0", "put_act+bar", "Q proj", "stores"],
         1: ["entry", "prologue issued", "prologue barrier", "out_proj", "LN1", "put_act+bar", "fc1", "put_act+bar",
             "fc2", "stores"],
         2: ["entry", "prologue issued", "prologue barrier", "LN2", "post LN", "put_act+bar", "in_proj", "end"]}
for k in range(3):
    st = buf[k].astype(np.int64)
    n = len(names[k])
    d = st[:, 1:n] - st[:, 0:n - 1]
    med = np.median(d, axis=0)
    tot = np.median(st[:, n - 1] - st[:, 0])
    print(f"chain kind {k}: total {tot:.0f} cycles (wave 0, median of 16 WGs)")
    for i in range(1, n):
        print(f"   {names[k][i - 1]:>18} -> {names[k][i]:<18} {med[i - 1]:8.0f}")
