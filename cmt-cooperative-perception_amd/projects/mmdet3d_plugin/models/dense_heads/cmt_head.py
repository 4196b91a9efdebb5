"""CmtHead / CmtLidarHead / CmtImageHead and SeparateTaskHead with the
reference's constructor kwargs, forward signatures, output layout and
state_dict keys; the forward runs on the gfx950 kernels (engine.py).

Reference: projects/mmdet3d_plugin/models/dense_heads/cmt_head.py
  pos2embed 40-50, LayerNormFunction 53-81, GroupLayerNorm1d 84-94,
  SeparateTaskHead 97-203, CmtHead 206-919, CmtImageHead 922-999,
  CmtLidarHead 1002-1085.
Outputs: ``forward`` returns the multi_apply layout -- a tuple over tasks of a
list over feature levels (one) of dicts {center, height, dim, rot, vel,
cls_logits}, each [L, B, Nq, k] fp32 (cmt_head.py:549-554).  In training mode
forward_single runs forward_train (DN queries, native training kernels,
train_engine.py) and ``loss`` the Hungarian-matched focal / L1 / DN losses.
"""
import copy
import math

import numpy as np
import torch
import torch.nn as nn

from ... import native
from ...registry import HEADS, build_bbox_coder, build_from_cfg, build_transformer
from ...runtime import check_f16_range, get_precision, is_split, op_empty
from ..utils.packing import PackCache, to_dtype
from .engine import HeadEngineMixin, _inv_lidar2img
from .train_engine import HeadTrainMixin

__all__ = ["pos2embed", "GroupLayerNorm1d", "SeparateTaskHead", "ConvModule", "CmtHead", "CmtLidarHead",
           "CmtImageHead", "multi_apply"]


def multi_apply(func, *args, **kwargs):
    """mmdet.core.multi_apply."""
    from functools import partial
    pfunc = partial(func, **kwargs) if kwargs else func
    map_results = map(pfunc, *args)
    return tuple(map(list, zip(*map_results)))


def pos2embed(pos, num_pos_feats=128, temperature=10000):
    """cmt_head.py:40-50 on the native kernel (``temperature`` is ignored, as in
    the reference).  pos [..., >=2] on device -> [..., 2*num_pos_feats]."""
    shape = pos.shape
    flat = pos.reshape(-1, shape[-1]).contiguous().float()
    out = torch.empty((flat.shape[0], 2 * num_pos_feats), dtype=torch.float32, device=pos.device)
    native.pos2embed(flat, out, n=flat.shape[0], F=num_pos_feats, pos_stride=shape[-1])
    return out.view(*shape[:-1], 2 * num_pos_feats)


class GroupLayerNorm1d(nn.Module):
    """cmt_head.py:84-94 (per-group LayerNorm over channels, eps 1e-6).  Its
    forward runs inside the task-head tail kernel."""

    def __init__(self, channels, groups=1, eps=1e-6):
        super().__init__()
        self.register_parameter("weight", nn.Parameter(torch.ones(channels)))
        self.register_parameter("bias", nn.Parameter(torch.zeros(channels)))
        self.groups = groups
        self.eps = eps


@HEADS.register_module()
class SeparateTaskHead(nn.Module):
    """cmt_head.py:97-203.  Per head: grouped Conv1d(in*G -> head_conv*G, k) ->
    GroupLayerNorm1d -> ReLU -> grouped Conv1d(head_conv*G -> classes*G, k),
    G = number of decoder layers, k = final_kernel convolving along the query
    axis.  Only num_conv == 2 (every CMT config) is supported natively."""

    def __init__(self, in_channels, heads, groups=1, head_conv=64, final_kernel=1, init_bias=-2.19, init_cfg=None,
                 **kwargs):
        assert init_cfg is None, "To prevent abnormal initialization behavior, init_cfg is not allowed to be set"
        super().__init__()
        self.heads = heads
        self.groups = groups
        self.init_bias = init_bias
        self.in_channels = in_channels
        self.head_conv = head_conv
        self.final_kernel = final_kernel
        for head in self.heads:
            classes, num_conv = self.heads[head]
            layers = []
            c_in = in_channels
            for _ in range(num_conv - 1):
                layers.extend([
                    nn.Conv1d(c_in * groups, head_conv * groups, kernel_size=final_kernel, stride=1,
                              padding=final_kernel // 2, groups=groups, bias=False),
                    GroupLayerNorm1d(head_conv * groups, groups=groups),
                    nn.ReLU(inplace=True)])
                c_in = head_conv
            layers.append(nn.Conv1d(head_conv * groups, classes * groups, kernel_size=final_kernel, stride=1,
                                    padding=final_kernel // 2, groups=groups, bias=True))
            self.__setattr__(head, nn.Sequential(*layers))
        self._pack = PackCache()

    def init_weights(self):
        """mmcv Kaiming init of every Conv1d (fan_out, relu, normal, bias 0),
        then cls bias = init_bias (cmt_head.py:164-172)."""
        for m in self.modules():
            if isinstance(m, nn.Conv1d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
        for head in self.heads:
            if head == "cls_logits":
                self.__getattr__(head)[-1].bias.data.fill_(self.init_bias)

    def packed(self, prec):
        names = list(self.heads)
        for n in names:
            if self.heads[n][1] != 2:
                raise NotImplementedError("native SeparateTaskHead supports num_conv == 2")
        if self.head_conv != 64:
            raise NotImplementedError("native SeparateTaskHead supports head_conv == 64")

        def build():
            G, C, hc, k = self.groups, self.in_channels, self.head_conv, self.final_kernel
            w1, gw, gb, w2, b2, outs = [], [], [], [], [], []
            for n in names:
                seq = getattr(self, n)
                c1, gln, c2 = seq[0], seq[1], seq[3]
                # [G*hc, C, k] -> [G][hc][k*C] (tap-major rows for the implicit conv1d GEMM)
                w1.append(c1.weight.view(G, hc, C, k).permute(0, 1, 3, 2).reshape(G, hc, k * C))
                gw.append(gln.weight.view(G, hc))
                gb.append(gln.bias.view(G, hc))
                out_n = self.heads[n][0]
                w2.append(c2.weight.view(G, out_n, hc, k).permute(0, 1, 3, 2))       # [G][out][k][hc]
                b2.append(c2.bias.view(G, out_n))
                outs.append(out_n)
            center_col = height_col = -1
            start = 0
            for n, o in zip(names, outs):
                if n == "center":
                    center_col = start
                if n == "height":
                    height_col = start
                start += o
            return dict(names=names, head_out=outs, out_total=start, k=k, center_col=center_col,
                        height_col=height_col,
                        w1=to_dtype(torch.cat(w1, 1), prec.gemm),
                        gw=torch.cat(gw, 1).detach().float().contiguous(),
                        gb=torch.cat(gb, 1).detach().float().contiguous(),
                        w2=torch.cat(w2, 1).detach().float().contiguous(),
                        b2=torch.cat(b2, 1).detach().float().contiguous())
        return self._pack.get("w", list(self.parameters()), prec.name, build)

    def forward(self, x):
        """x [N, B, Nq, C] -> dict of [N, B, Nq, classes] (no box epilogue)."""
        prec = get_precision()
        tp = self.packed(prec)
        L, B, Nq, C = x.shape
        width = len(tp["names"]) * 64
        k = tp["k"]
        X = x.reshape(L, B * Nq, C).contiguous().float()
        if is_split(tp["w1"]):
            X = native.split_rows(X.view(L * B * Nq, C)).view(L, B * Nq, 2, C)
        H1 = torch.empty((L, B * Nq, width), dtype=torch.float32, device=x.device)
        native.gemm(X, tp["w1"], H1, M=B * Nq, N=width, K=k * C, lda=C, ldw=k * C, ldc=width, batch=L,
                    a_bstride=B * Nq * C, w_bstride=width * k * C, c_bstride=B * Nq * width,
                    a_mode=native.A_CONV1D3 if k == 3 else native.A_ROWS, seg_len=Nq)
        OUT = torch.empty((L, B, Nq, tp["out_total"]), dtype=torch.float32, device=x.device)
        dummy_ref = torch.zeros((B, Nq, 3), dtype=torch.float32, device=x.device)
        native.task_head_tail(H1, tp["gw"], tp["gb"], tp["w2"], tp["b2"], dummy_ref, OUT, L=L, B=B, Nq=Nq,
                              nheads=len(tp["names"]), hc=64, head_out=tp["head_out"], k=k, center_col=-1,
                              height_col=-1, pc_range=[0, 0, 0, 1, 1, 1])
        ret, start = {}, 0
        for n, o in zip(tp["names"], tp["head_out"]):
            ret[n] = OUT[..., start:start + o]
            start += o
        return ret


class ConvModule(nn.Module):
    """mmcv ConvModule(conv 3x3 no bias, BN2d, ReLU) -- cmt_head.py:280-287."""

    def __init__(self, in_channels, out_channels, kernel_size=3, padding=1, conv_cfg=None, norm_cfg=None,
                 act_cfg=dict(type="ReLU"), **kwargs):
        super().__init__()
        assert kernel_size == 3 and padding == 1, "shared_conv is a 3x3 / pad 1 conv in every CMT config"
        self.with_norm = norm_cfg is not None
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, padding=padding, bias=not self.with_norm)
        if self.with_norm:
            self.bn = nn.BatchNorm2d(out_channels)
        self.activate = nn.ReLU(inplace=True)

    def init_weights(self):
        nn.init.kaiming_normal_(self.conv.weight, mode="fan_out", nonlinearity="relu")
        if self.with_norm:
            nn.init.ones_(self.bn.weight)
            nn.init.zeros_(self.bn.bias)


def _common_init(self, in_channels, num_query, hidden_dim, depth_num, norm_bbox, downsample_scale, scalar,
                 noise_scale, noise_trans, dn_weight, split, train_cfg, test_cfg, common_heads, tasks, transformer,
                 bbox_coder, loss_cls, loss_bbox, loss_heatmap, separate_head):
    """Shared constructor of CmtHead (cmt_head.py:209-318) and CmtHeadCoop
    (cmt_head_coop.py:75-184)."""
    self.num_classes = [len(t["class_names"]) for t in tasks]
    self.class_names = [t["class_names"] for t in tasks]
    self.hidden_dim = hidden_dim
    self.train_cfg = train_cfg
    self.test_cfg = test_cfg
    self.num_query = num_query
    self.in_channels = in_channels
    self.depth_num = depth_num
    self.norm_bbox = norm_bbox
    self.downsample_scale = downsample_scale
    self.scalar = scalar
    self.bbox_noise_scale = noise_scale
    self.bbox_noise_trans = noise_trans
    self.dn_weight = dn_weight
    self.split = split
    # losses are built by the training path; keep the cfgs
    self.loss_cls_cfg, self.loss_bbox_cfg, self.loss_heatmap_cfg = loss_cls, loss_bbox, loss_heatmap
    self.bbox_coder = build_bbox_coder(bbox_coder)
    self.pc_range = list(self.bbox_coder.pc_range)
    if len(self.pc_range) != 6:
        raise ValueError("bbox_coder.pc_range must have 6 entries")
    self.fp16_enabled = False
    self.shared_conv = ConvModule(in_channels, hidden_dim, kernel_size=3, padding=1, conv_cfg=dict(type="Conv2d"),
                                  norm_cfg=dict(type="BN2d"))
    self.transformer = build_transformer(transformer)
    self.reference_points = nn.Embedding(num_query, 3)
    self.bev_embedding = nn.Sequential(nn.Linear(hidden_dim * 2, hidden_dim), nn.ReLU(inplace=True),
                                       nn.Linear(hidden_dim, hidden_dim))
    self.rv_embedding = nn.Sequential(nn.Linear(depth_num * 3, hidden_dim * 4), nn.ReLU(inplace=True),
                                      nn.Linear(hidden_dim * 4, hidden_dim))
    self.task_heads = nn.ModuleList()
    for num_cls in self.num_classes:
        heads = copy.deepcopy(common_heads)
        heads.update(dict(cls_logits=(num_cls, 2)))
        separate_head.update(in_channels=hidden_dim, heads=heads, num_cls=num_cls,
                             groups=transformer["decoder"]["num_layers"])
        self.task_heads.append(build_from_cfg(separate_head, HEADS))
    self._pack = PackCache()


def _common_init_weights(self):
    """mmcv BaseModule.init_weights recursion + reference_points U(0,1)
    (cmt_head.py:320-322)."""
    self.transformer.init_weights()
    for t in self.task_heads:
        t.init_weights()
    if self.shared_conv is not None:
        self.shared_conv.init_weights()
    for seq in (self.bev_embedding, self.rv_embedding):
        if seq is not None:
            for m in seq:
                if isinstance(m, nn.Linear):
                    nn.init.kaiming_uniform_(m.weight, a=math.sqrt(5))
    nn.init.uniform_(self.reference_points.weight.data, 0, 1)


_DEFAULT_TASKS = [
    dict(num_class=1, class_names=["car"]),
    dict(num_class=2, class_names=["truck", "construction_vehicle"]),
    dict(num_class=2, class_names=["bus", "trailer"]),
    dict(num_class=1, class_names=["barrier"]),
    dict(num_class=2, class_names=["motorcycle", "bicycle"]),
    dict(num_class=2, class_names=["pedestrian", "traffic_cone"]),
]


def gt_from_metas(img_metas):
    """The GT the reference's prepare_for_dn reads from img_metas
    (cmt_head.py:341-342): 'gt_bboxes_3d' (LiDARInstance3DBoxes-like, a
    DataContainer around one, or a [n, 9] gravity-centre tensor) and
    'gt_labels_3d'.  Returns (gravity-centre boxes list, labels list)."""
    boxes, labels = [], []
    for m in img_metas:
        b, l = m["gt_bboxes_3d"], m["gt_labels_3d"]
        b = getattr(b, "_data", b)
        l = getattr(l, "_data", l)
        if not torch.is_tensor(b):
            b = torch.cat([b.gravity_center, b.tensor[:, 3:]], 1)
        boxes.append(b)
        labels.append(l)
    return boxes, labels


@HEADS.register_module()
class CmtHead(HeadTrainMixin, HeadEngineMixin, nn.Module):
    """cmt_head.py:206-919 (fusion head: BEV + multi-view image memory)."""
    variant = "fusion"

    def __init__(self, in_channels, num_query=900, hidden_dim=128, depth_num=64, norm_bbox=True,
                 downsample_scale=8, scalar=10, noise_scale=1.0, noise_trans=0.0, dn_weight=1.0, split=0.75,
                 train_cfg=None, test_cfg=None,
                 common_heads=dict(center=(2, 2), height=(1, 2), dim=(3, 2), rot=(2, 2), vel=(2, 2)),
                 tasks=None, transformer=None, bbox_coder=None,
                 loss_cls=dict(type="FocalLoss", use_sigmoid=True, reduction="mean", gamma=2, alpha=0.25,
                               loss_weight=1.0),
                 loss_bbox=dict(type="L1Loss", reduction="mean", loss_weight=0.25),
                 loss_heatmap=dict(type="GaussianFocalLoss", reduction="mean"),
                 separate_head=dict(type="SeparateMlpHead", init_bias=-2.19, final_kernel=3),
                 init_cfg=None, **kwargs):
        assert init_cfg is None
        super().__init__()
        _common_init(self, in_channels, num_query, hidden_dim, depth_num, norm_bbox, downsample_scale, scalar,
                     noise_scale, noise_trans, dn_weight, split, train_cfg, test_cfg, common_heads,
                     tasks if tasks is not None else copy.deepcopy(_DEFAULT_TASKS), transformer, bbox_coder,
                     loss_cls, loss_bbox, loss_heatmap, separate_head)

    def init_weights(self):
        _common_init_weights(self)

    @property
    def coords_bev(self):
        """cmt_head.py:324-337 (returned on the reference_points device)."""
        cfg = self.train_cfg if self.train_cfg else self.test_cfg
        x_size = cfg["grid_size"][1] // self.downsample_scale
        y_size = cfg["grid_size"][0] // self.downsample_scale
        batch_y, batch_x = torch.meshgrid(torch.arange(x_size, dtype=torch.float32),
                                          torch.arange(y_size, dtype=torch.float32), indexing="ij")
        batch_x = (batch_x + 0.5) / x_size
        batch_y = (batch_y + 0.5) / y_size
        return torch.cat([batch_x[None], batch_y[None]], dim=0).view(2, -1).transpose(1, 0)

    def _forward_agents(self, agents, img_metas, B, meta_fns=None, shard=None):
        """Run the decoder for each (x, x_img, metas) agent, max-fusing into one
        [L, B*Nq, C] buffer, then the task heads.  ``meta_fns[i]`` maps the
        frame's img_metas to agent i's metas (identity by default); the ones of
        the agents with cameras are kept for stage_metas.

        ``shard`` = (rank, world, group): agent sharding over the ranks of a
        process group (SURVEY 8(e)'s optional second axis, configs[4]).  Rank r
        decodes agents r, r + world, ... into its own buffer, and ONE
        all_reduce(MAX) of the post-normed [L, B*Nq, C] outputs replaces the
        in-process max over agents -- torch.max(torch.stack(...), 0) of
        cmt_head_coop.py:383-389.  Max is exact and order-free, so every rank
        then holds the single-process fused outputs bit for bit and runs the
        task heads on them."""
        self._check_eval()
        fns = meta_fns if meta_fns is not None else [lambda m: m] * len(agents)
        mine = list(range(len(agents)))
        if shard is not None:
            rank, world, _ = shard
            mine = [i for i in mine if i % world == rank]
        self._meta_plan = [fns[i] for i in mine if agents[i][1] is not None and self.variant != "lidar"]
        prec = get_precision()
        check_f16_range(prec, [t for i in mine for t in agents[i][:2]])
        L = self.transformer.decoder.num_layers
        outs = torch.empty((L, B * self.num_query, self.hidden_dim), dtype=torch.float32,
                           device=self.reference_points.weight.device)
        outs16 = None
        if prec.gemm != torch.float32:
            outs16 = op_empty(B * self.num_query, self.hidden_dim, prec.gemm, outs.device, lead=(L,))
        self._h2d_seq = 0    # staging-buffer slot of each camera-matrix upload in this forward (engine._h2d)
        if not mine:
            outs.fill_(-float("inf"))   # a rank without an agent: the identity of the MAX all-reduce
        for j, i in enumerate(mine):
            x, x_img, metas = agents[i]
            flags = native.LN_NAN_TO_NUM | (native.LN_MAX_INTO if j > 0 else 0)
            self._decode_agent(x, x_img, metas, B, outs, flags, self.variant, prec, out16=outs16)
        if shard is not None:
            import torch.distributed as dist
            dist.all_reduce(outs, op=dist.ReduceOp.MAX, group=shard[2])
            if outs16 is not None:   # the compute-dtype copy of the fused outputs (task-head GEMM operand)
                if is_split(outs16):
                    native.split_rows(outs.view(-1, self.hidden_dim), outs16.view(-1, 2, self.hidden_dim))
                else:
                    native.cast(outs, outs16)
        return self._task_outputs(outs, B, prec, outs16)

    def forward_single(self, x, x_img, img_metas):
        B = x.shape[0] if x is not None else len(img_metas)
        if self.variant == "lidar":
            assert x_img is None
        if self.variant == "image":
            assert x is None
        if self.training:
            return self.forward_train([(x, x_img, img_metas)], img_metas, *gt_from_metas(img_metas))
        return self._forward_agents([(x, x_img, img_metas)], img_metas, B)

    def stage_metas(self, img_metas):
        """Write a new frame's camera matrices (lidar2img and its fp64 host
        inverse, cmt_head.py:428, 441-444) into the pinned staging buffers a
        captured forward reads, so ``graph.replay()`` computes the frame with
        THESE metas (the graph's copy nodes re-read the buffers).  Call it after
        the previous replay has consumed its buffers (e.g. after synchronising
        that replay's stream) and before the next one.  The agents and camera
        counts must be those of the captured forward."""
        plan = getattr(self, "_meta_plan", None)
        pool = self.__dict__.get("_pinned_meta")
        if plan is None or pool is None:
            raise RuntimeError("stage_metas needs one eager forward (and the graph capture) first")
        for seq, fn in enumerate(plan):
            l2i, i2l = _inv_lidar2img(fn(img_metas))
            t = torch.from_numpy(np.ascontiguousarray(np.stack([l2i, i2l]))).float()
            key = ("cams", tuple(t.shape), seq)
            if key not in pool:
                raise RuntimeError(f"stage_metas: camera layout {tuple(t.shape)} of agent {seq} differs from the "
                                   "captured forward's")
            pool[key].copy_(t)

    def forward(self, pts_feats, img_feats=None, img_metas=None):
        """list([bs, c, h, w]) per level -> multi_apply layout (cmt_head.py:549-554)."""
        if img_feats is None:
            img_feats = [None for _ in range(len(pts_feats))]
        img_metas = [img_metas for _ in range(len(pts_feats))]
        return multi_apply(self.forward_single, pts_feats, img_feats, img_metas)

    def get_bboxes(self, preds_dicts, img_metas, img=None, rescale=False):
        """cmt_head.py:905-919 (box_type_3d wrapping applied when the meta has it)."""
        preds = self.bbox_coder.decode(preds_dicts)
        ret = []
        for i, p in enumerate(preds):
            bboxes = p["bboxes"]
            bboxes[:, 2] = bboxes[:, 2] - bboxes[:, 5] * 0.5
            box_type = img_metas[i].get("box_type_3d") if isinstance(img_metas[i], dict) else None
            if box_type is not None:
                bboxes = box_type(bboxes, bboxes.size(-1))
            ret.append([bboxes, p["scores"], p["labels"]])
        return ret


@HEADS.register_module()
class CmtImageHead(CmtHead):
    """cmt_head.py:922-999 (no shared_conv, image memory only)."""
    variant = "image"

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.shared_conv = None


@HEADS.register_module()
class CmtLidarHead(CmtHead):
    """cmt_head.py:1002-1085 (no rv_embedding, BEV memory only)."""
    variant = "lidar"

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.rv_embedding = None
