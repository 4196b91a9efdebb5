"""Training forward and loss of CmtHead / CmtHeadCoop on the native training
kernels (BASELINE.json configs[3]).

Reference: projects/mmdet3d_plugin/models/dense_heads/cmt_head.py
  prepare_for_dn 339-415 (DN query groups, attention mask 386-398),
  forward_single 475-547 (training branch: dn_* outputs split off the front),
  _get_targets_single / get_targets 556-675 (HungarianAssigner3D,
  core/bbox/assigners/hungarian_assigner_3d.py:68-156, scipy on the host),
  _loss_single_task / loss_single 677-758, _dn_loss_single_task /
  dn_loss_single 760-813 (reduce_mean all-reduce of num_tgt), loss 815-903;
and cmt_head_coop.py:205-275, 362-437, 686 for the two-agent head.

Every matrix product, attention core, LayerNorm, BatchNorm, conv weight
gradient and loss runs in train.hip / attn_train.hip through
models/utils/train_ops.py (autograd Functions with native forward AND
backward); the glue here is index/reshape work on [B, Nq]-sized tensors,
residual adds, ReLU, dropout masks and the sin/cos / camera geometry of the
query embedding (a few thousand elements), all on the device.  The Hungarian
assignment copies the [Nq, n_gt] cost matrix to the host and runs scipy's
linear_sum_assignment, exactly as the reference does.
"""
import math

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F
from scipy.optimize import linear_sum_assignment

from ... import native
from ... import native_train as T
from ...runtime import OPTIONS
from ..utils import train_ops as ops

__all__ = ["HeadTrainMixin", "Boxes3D", "inverse_sigmoid"]


def _to_dev_async(t, dev):
    """host tensor -> device without a stream sync (pinned staging, non-blocking copy; the caching
    host allocator keeps the staging block until the copy has run)"""
    if t.device.type != "cpu" or torch.device(dev).type == "cpu":
        return t.to(dev)
    return t.pin_memory().to(dev, non_blocking=True)


class _DecoderStep(torch.nn.Module):
    """One agent's decoder training walk with its static switches, as a module whose parameters
    are the decoder's (the callable torch.cuda.make_graphed_callables captures)."""

    def __init__(self, decoder, n_agents=0, **opts):
        super().__init__()
        self.decoder = decoder
        self.n_agents = n_agents   # > 0: the inputs are tgt, qpos, the agents' mem rows, their pos rows
        self.opts = opts

    def forward(self, tgt, qpos, *rest):
        *rows, seed = rest
        n = self.n_agents
        mem, pos = (list(rows[:n]), list(rows[n:])) if n else (rows[0], rows[1])
        return self.decoder.train_rows(tgt, qpos, mem, pos, seed_dev=seed, **self.opts)


def inverse_sigmoid(x, eps=1e-5):
    """mmdet 2.28.2 inverse_sigmoid."""
    x = x.clamp(min=0, max=1)
    return torch.log(x.clamp(min=eps) / (1 - x).clamp(min=eps))


class Boxes3D:
    """The part of mmdet3d LiDARInstance3DBoxes the head reads: ``tensor``
    [n, 9] (x, y, z_bottom, w, l, h, yaw, vx, vy) and ``gravity_center``."""

    def __init__(self, tensor):
        self.tensor = tensor

    @property
    def gravity_center(self):
        t = self.tensor
        return torch.cat([t[:, :2], t[:, 2:3] + t[:, 5:6] * 0.5], 1)


def _gravity_boxes(g):
    """GT boxes [n, 9] with gravity centres: LiDARInstance3DBoxes-like objects
    (anything with ``gravity_center`` and ``tensor``, cmt_head.py:571-573) are
    converted; plain tensors are taken as gravity-centre boxes already."""
    if hasattr(g, "gravity_center") and hasattr(g, "tensor"):
        return torch.cat([g.gravity_center, g.tensor[:, 3:]], 1)
    return g


def _normalize_bbox(b):
    """core/bbox/util.py:8-34."""
    return torch.cat([b[..., 0:3], b[..., 3:6].log(), b[..., 6:7].sin(), b[..., 6:7].cos(), b[..., 7:9]], -1)


def _pos2embed(pos, F_):
    """cmt_head.py:40-50 as differentiable tensor ops (reference points carry
    a gradient into reference_points.weight)."""
    pos = pos * (2 * math.pi)
    dim_t = torch.arange(F_, dtype=pos.dtype, device=pos.device)
    dim_t = 2 * torch.div(dim_t, 2, rounding_mode="floor") / F_ + 1
    px = pos[..., 0, None] / dim_t
    py = pos[..., 1, None] / dim_t
    px = torch.stack((px[..., 0::2].sin(), px[..., 1::2].cos()), -1).flatten(-2)
    py = torch.stack((py[..., 0::2].sin(), py[..., 1::2].cos()), -1).flatten(-2)
    return torch.cat((py, px), -1)


class HeadTrainMixin:
    """Mixed into CmtHead (and through it CmtHeadCoop and the LiDAR / image
    variants)."""

    train_dropout = True   # the reference trains with dropout 0.1 (attn_drop of the self-attention core and
    #                        the dropout_layer after both attentions); parity tests switch it off
    train_cross_fp16 = True   # the flash-attn fp16 cross core (reference numerics); off = exact f32 core

    # ------------------------------------------------------------------ DN queries
    def prepare_for_dn_train(self, B, gt_boxes, gt_labels, rand_prob=None, generator=None):
        """prepare_for_dn training branch (cmt_head.py:339-415).  gt_boxes[b]:
        [n_b, 9] gravity-centre boxes on the device; gt_labels[b] [n_b].
        rand_prob: the U(-1, 1) centre noise (drawn here when None)."""
        ref = self.reference_points.weight
        dev = ref.device
        known_num = [int(t.shape[0]) for t in gt_boxes]
        if max(known_num, default=0) == 0:
            return ref.unsqueeze(0).repeat(B, 1, 1), None
        labels = torch.cat(gt_labels).long()
        boxes = torch.cat(gt_boxes).float()
        # built on the device (a pageable host -> device copy waits for the stream: the previous
        # step's backward would have to drain before this step's forward could be issued)
        batch_idx = torch.cat([torch.full((n,), i, dtype=torch.long, device=dev) for i, n in enumerate(known_num)])
        groups = min(self.scalar, self.num_query // max(known_num))
        known_indice = torch.arange(labels.numel(), device=dev).repeat(groups)
        known_labels = labels.repeat(groups)
        known_bid = batch_idx.repeat(groups)
        known_bboxs = boxes.repeat(groups, 1)
        center = known_bboxs[:, :3].clone()
        scale = known_bboxs[:, 3:6]
        if self.bbox_noise_scale > 0:
            if rand_prob is None:
                rand_prob = _to_dev_async(torch.rand(center.shape, generator=generator), dev) * 2 - 1.0
            rand_prob = _to_dev_async(rand_prob, dev)
            center = center + rand_prob * (scale / 2 + self.bbox_noise_trans) * self.bbox_noise_scale
            pcr = self.pc_range
            center = torch.stack([(center[:, 0] - pcr[0]) / (pcr[3] - pcr[0]),
                                  (center[:, 1] - pcr[1]) / (pcr[4] - pcr[1]),
                                  (center[:, 2] - pcr[2]) / (pcr[5] - pcr[2])], -1).clamp(0.0, 1.0)
            mask = torch.norm(rand_prob, 2, 1) > self.split
            known_labels = torch.where(mask, torch.full_like(known_labels, sum(self.num_classes)), known_labels)
        single_pad = int(max(known_num))
        pad = single_pad * groups
        padded = torch.cat([ref.new_zeros(pad, 3), ref], 0).unsqueeze(0).repeat(B, 1, 1)
        map_known = torch.cat([torch.arange(n, device=dev) for n in known_num])
        map_known = torch.cat([map_known + single_pad * i for i in range(groups)]).long()
        padded = padded.index_put((known_bid, map_known), center.to(padded.dtype))
        mask_dict = dict(known_indice=known_indice, batch_idx=batch_idx, map_known_indice=map_known,
                         known_lbs_bboxes=(known_labels, known_bboxs), known_labels_raw=labels.repeat(groups),
                         pad_size=pad, single_pad=single_pad, groups=groups)
        return padded, mask_dict

    # ------------------------------------------------------------------ pieces
    def _mlp_t(self, x, seq):
        h = torch.relu(ops.linear(x, seq[0].weight, seq[0].bias))
        return ops.linear(h, seq[2].weight, seq[2].bias)

    def _drop(self, x):
        return F.dropout(x, 0.1, True) if self.train_dropout else x

    def _rv_query_embed_t(self, rp, metas):
        """cmt_head.py:439-467 (geometry as device tensor ops, differentiable in rp)."""
        pad_h, pad_w, _ = metas[0]["pad_shape"][0]
        dev, dt = rp.device, rp.dtype
        l2i = _to_dev_async(torch.from_numpy(np.stack([np.asarray(m["lidar2img"], dtype=np.float64)
                                                       for m in metas])).to(dt), dev)
        i2l = _to_dev_async(torch.from_numpy(np.stack([np.linalg.inv(np.asarray(m["lidar2img"], dtype=np.float64))
                                                       for m in metas])).to(dt), dev)
        pcr = _to_dev_async(torch.tensor(self.pc_range, dtype=dt), dev)
        pts = rp * (pcr[3:] - pcr[:3]) + pcr[:3]
        proj = torch.einsum("bnd,bvcd->bvnc", torch.cat([pts, torch.ones_like(pts[..., :1])], -1), l2i)
        zm = proj[..., 2:3] > 0
        den = proj[..., 2:3] + zm * 1e-6 - (~zm) * 1e-6
        proj = torch.cat([proj[..., :3] / den, proj[..., 3:]], -1)
        mask = (proj[..., 0] < pad_w) & (proj[..., 0] >= 0) & (proj[..., 1] < pad_h) & (proj[..., 1] >= 0) & zm[..., 0]
        D = self.depth_num
        cd = 1 + torch.arange(D, dtype=dt, device=dev) * (self.pc_range[3] - 1) / D
        p3 = torch.einsum("bvnc,d->bvndc", proj, cd)
        p3 = torch.cat([p3[..., :3], torch.ones_like(p3[..., :1])], -1)
        back = torch.einsum("bvndo,bvco->bvndc", p3, i2l)
        back = (back[..., :3] - pcr[:3]) / (pcr[3:] - pcr[:3])
        rv = self._mlp_t(back.reshape(*back.shape[:-2], -1), self.rv_embedding)
        return (rv * mask.unsqueeze(-1)).sum(1)

    def _memory_t(self, x, x_img, metas, B):
        """memory / pos rows [B, Nk, C] of one agent (shared_conv with batch
        statistics, bev / rv position MLPs)."""
        C = self.hidden_dim
        mems, poss = [], []
        if x is not None and self.shared_conv is not None:
            _, Cin, H, W = x.shape
            xr = ops.nchw_rows(x, B, range_flag=self._range_flag(x.device))   # the split conv's operand
            conv = self.shared_conv.conv
            w = conv.weight.permute(0, 2, 3, 1).reshape(conv.weight.shape[0], -1)
            y = ops.bn_relu(ops.conv3x3(xr, w, (B, H, W, Cin)), self.shared_conv.bn)
            mems.append(y.view(B, H * W, C))
            cfg = self.train_cfg if self.train_cfg else self.test_cfg
            xs, ys = cfg["grid_size"][1] // self.downsample_scale, cfg["grid_size"][0] // self.downsample_scale
            pe = torch.empty((H * W, 2 * C), dtype=torch.float32, device=x.device)
            native.pos2embed(None, pe, n=H * W, F=C, grid=(xs, ys))
            poss.append(self._mlp_t(pe, self.bev_embedding).unsqueeze(0).expand(B, H * W, C))
        if x_img is not None:
            BV, _, h, w_ = x_img.shape
            V = BV // B
            mems.append(ops.nchw_rows(x_img, B).view(B, V * h * w_, C))
            pad_h, pad_w, _ = metas[0]["pad_shape"][0]
            i2l = _to_dev_async(torch.from_numpy(np.stack([np.linalg.inv(np.asarray(m["lidar2img"], dtype=np.float64))
                                                           for m in metas])).float(), x_img.device)
            D = self.depth_num
            coords = torch.empty((BV * h * w_, 3 * D), dtype=torch.float32, device=x_img.device)
            native.rv_pe_coords(i2l, coords, BV=BV, h=h, w=w_, D=D, pad_h=float(pad_h), pad_w=float(pad_w),
                                depth_max=float(self.pc_range[3]), pc_range=self.pc_range)
            poss.append(self._mlp_t(coords, self.rv_embedding).view(B, V * h * w_, C))
        return torch.cat(mems, 1), torch.cat(poss, 1)

    def _decoder_t(self, tgt, qpos, mem, pos, mask_dict):
        """PETRTransformerDecoder with the training op walk (post-norm,
        petr_transformer.py:324-487; mmcv BaseTransformerLayer): the decoder's
        own train_rows, with this head's DN padding and dropout switches.
        mem / pos may be lists (one per agent: every agent's decoder in one walk).
        With OPTIONS.train_graph (CMT_TRAIN_GRAPH=1; off by default) the walk's
        forward and backward are HIP graphs (torch.cuda.make_graphed_callables)
        captured once per shape, the attention dropout seed drawn on the device
        each step (profiles/r5_experiments.txt r5ai, r5at).  Limits of the graph
        mode: the key holds the DN padding, which follows the batch's GT count, so
        real data with a varying GT count re-captures often (the cache keeps 8
        shapes); a forward whose previous replay's backward has not run yet takes
        the eager walk."""
        pad = mask_dict["pad_size"] if mask_dict else 0
        group = mask_dict["single_pad"] if mask_dict else 0
        dec = self.transformer.decoder
        if not (OPTIONS.train_graph and tgt.is_cuda and torch.is_grad_enabled()
                and not torch.cuda.is_current_stream_capturing()):
            return dec.train_rows(tgt, qpos, mem, pos, pad=pad, group=group, dropout=self.train_dropout,
                                  cross_fp16=self.train_cross_fp16)
        agents = isinstance(mem, (list, tuple))
        ins = (tgt, qpos) + (tuple(mem) + tuple(pos) if agents else (mem, pos))
        # a graph reads its inputs, parameters and outputs at fixed addresses: one per shape, DN
        # geometry and parameter storage
        key = (pad, group, self.train_dropout, self.train_cross_fp16,
               tuple((tuple(t.shape), t.requires_grad) for t in ins),
               tuple(p.data_ptr() for p in dec.parameters()))
        cache = self.__dict__.setdefault("_dec_graphs", {})
        fn = cache.get(key)
        seed = torch.randint(0, 2 ** 31 - 1, (1,), dtype=torch.int32, device=tgt.device)
        if fn is None:
            if len(cache) >= 8:          # shapes follow the GT count: keep the cache bounded
                cache.clear()
            step = _DecoderStep(dec, len(mem) if agents else 0, pad=pad, group=group, dropout=self.train_dropout,
                                cross_fp16=self.train_cross_fp16)
            samples = tuple(t.detach().clone().requires_grad_(t.requires_grad) for t in ins) + (seed.clone(),)
            fn = cache[key] = torch.cuda.make_graphed_callables(step, samples, allow_unused_input=True)
        # a graphed callable replays into static output / saved buffers: a second forward of the same
        # key before the first one's backward would overwrite what that backward reads -- take the
        # eager walk for it instead (gradient accumulation, a second head pass)
        pending = self.__dict__.setdefault("_dec_graph_pending", set())
        if key in pending:
            return dec.train_rows(tgt, qpos, mem, pos, pad=pad, group=group, dropout=self.train_dropout,
                                  cross_fp16=self.train_cross_fp16)
        out = fn(*ins, seed)
        first = out[0] if isinstance(out, (tuple, list)) else out
        if first.requires_grad:
            pending.add(key)
            first.register_hook(lambda g, k=key: pending.discard(k))
        return out

    def _task_head_t(self, task, x, reference):
        """SeparateTaskHead (cmt_head.py:136-203) + box epilogue (501-513).
        x [L, B, Nq, C] -> dict of [L, B, Nq, k]."""
        L, B, Nq, C = x.shape
        k = task.final_kernel
        if k == 3:   # conv along queries, zero padded per (layer, sample): taps q-1, q, q+1
            xin = ops.taps3(x)                                                          # [L, B, Nq, 3C]
        else:
            xin = x
        out = {}
        for name in task.heads:
            seq = getattr(task, name)
            c1, gln, c2 = seq[0], seq[1], seq[3]
            hc = c1.weight.shape[0] // L
            w1 = c1.weight.view(L, hc, C, k).permute(0, 1, 3, 2).reshape(L, hc, k * C)
            h = ops.linear_batched(xin, w1)                                              # [L, B, Nq, hc]
            h = ops.group_layer_norm(h.reshape(L, B * Nq, hc), gln.weight, gln.bias, gln.eps).view(L, B, Nq, hc)
            h = torch.relu(h)
            if k == 3:
                h = ops.taps3(h)
            on = c2.weight.shape[0] // L
            w2 = c2.weight.view(L, on, hc, k).permute(0, 1, 3, 2).reshape(L, on, k * hc)
            b2 = c2.bias.view(L, on)
            out[name] = ops.linear_batched(h, w2, b2)
        pcr = self.pc_range
        c = (out["center"] + reference[None, :, :, :2]).sigmoid()
        z = (out["height"] + reference[None, :, :, 2:3]).sigmoid()
        # x / y scaled by their pc_range spans in one op (per-column slices would each backward as a
        # zero fill + copy)
        sc = self.__dict__.get("_xy_affine")
        if sc is None or sc[0].device != c.device:
            sc = (torch.tensor([pcr[3] - pcr[0], pcr[4] - pcr[1]], dtype=torch.float32, device=c.device),
                  torch.tensor([pcr[0], pcr[1]], dtype=torch.float32, device=c.device))
            self.__dict__["_xy_affine"] = sc
        out["center"] = torch.addcmul(sc[1], c, sc[0])
        out["height"] = z * (pcr[5] - pcr[2]) + pcr[2]
        return out

    # ------------------------------------------------------------------ forward
    def forward_train(self, agents, img_metas, gt_boxes, gt_labels, rand_prob=None):
        """Training forward: ``agents`` = list of (x [B,512,H,W] or None, x_img or
        None, agent metas); gt_boxes[b] [n_b, 9] gravity-centre boxes, gt_labels[b].
        Returns (preds: list over tasks of dicts incl. dn_* and dn_mask_dict, as
        cmt_head.py:515-545)."""
        B = len(img_metas)
        C = self.hidden_dim
        self._stash_gt_labels(list(gt_labels))
        ref, mask_dict = self.prepare_for_dn_train(B, gt_boxes, gt_labels, rand_prob)
        rp = inverse_sigmoid(ref.clone()).sigmoid()
        qpos = self._mlp_t(_pos2embed(rp, C), self.bev_embedding)
        qs, mems, poss = [], [], []
        for x, x_img, metas in agents:
            q = qpos
            if x_img is not None and self.rv_embedding is not None:
                q = q + self._rv_query_embed_t(rp, metas)
            mem, pos = self._memory_t(x, x_img, metas, B)
            qs.append(q)
            mems.append(mem)
            poss.append(pos)
        if len(agents) > 1:
            # the agents' decoders as one walk: the query side of every layer on all agents' rows at
            # once (half the launches of two walks), the cross-attention per agent: 28.0-29.2 ->
            # 31.8-32.5 steps/s (profiles/r5_experiments.txt r5as)
            qa = torch.cat(qs, 0)
            decs = list(self._decoder_t(torch.zeros_like(qa), qa, mems, poss, mask_dict).split(B, dim=1))
        else:
            decs = [self._decoder_t(torch.zeros_like(qs[0]), qs[0], mems[0], poss[0], mask_dict)]
        # coop max fusion as the reference writes it (cmt_head_coop.py:388-389): torch.max over the
        # stacked agents routes each element's gradient to ONE agent (the max index), also on ties
        dec = decs[0] if len(decs) == 1 else torch.max(torch.stack(decs), 0).values
        reference = inverse_sigmoid(ref.clone())
        preds = []
        flag = 0
        pad = mask_dict["pad_size"] if mask_dict else 0
        for t, task in enumerate(self.task_heads):
            outs = self._task_head_t(task, dec, reference)
            if pad:
                names = self.class_names[t]
                kl, kb = mask_dict["known_lbs_bboxes"]
                raw = mask_dict["known_labels_raw"]
                n = len(names)
                # labels of this task's classes relative to it, the others n (no boolean-mask writes:
                # each was a device -> host sync)
                new_kl = torch.where((kl >= flag) & (kl < flag + n), kl - flag, torch.full_like(kl, n))
                new_raw = torch.where((raw >= flag) & (raw < flag + n), raw - flag, torch.full_like(raw, n))
                tmd = dict(mask_dict, known_lbs_bboxes=(new_kl, kb), known_labels_raw=new_raw)
                for key in list(outs):
                    # split, not two slices: one cat in the backward instead of two zero-filled copies + add
                    outs["dn_" + key], outs[key] = outs[key].split([pad, outs[key].shape[2] - pad], 2)
                outs["dn_mask_dict"] = tmd
            flag += len(self.class_names[t])
            preds.append(outs)
        return preds

    # ------------------------------------------------------------------ loss
    def _loss_cfg(self):
        lc, lb = self.loss_cls_cfg or {}, self.loss_bbox_cfg or {}
        tc = (self.train_cfg or {}).get("pts", self.train_cfg or {}) if self.train_cfg else {}
        asg = tc.get("assigner", {}) if tc else {}
        cw = tc.get("code_weights", [2.0, 2.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 0.2, 0.2]) if tc else \
            [2.0, 2.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 0.2, 0.2]
        return dict(gamma=float(lc.get("gamma", 2.0)), alpha=float(lc.get("alpha", 0.25)),
                    cls_weight=float(lc.get("loss_weight", 1.0)), box_weight=float(lb.get("loss_weight", 0.25)),
                    match_cls_weight=float(asg.get("cls_cost", {}).get("weight", 2.0)),
                    match_reg_weight=float(asg.get("reg_cost", {}).get("weight", 0.25)), code_weights=cw)

    def _stash_gt_labels(self, gt_labels):
        """Starts the device -> host copy of the GT labels before this step's forward kernels are
        queued (pinned, non-blocking, with an event): loss() selects each task's GT and the DN
        rows on the host from it, without a stream sync behind the whole forward."""
        self.__dict__["_gt_host"] = None
        if not gt_labels or any(l.device.type == "cpu" for l in gt_labels):
            return
        key = tuple((l.data_ptr(), l.numel()) for l in gt_labels)
        cat = torch.cat([l.reshape(-1).long() for l in gt_labels])
        host = torch.empty(cat.shape, dtype=torch.long, pin_memory=True)
        host.copy_(cat, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.__dict__["_gt_host"] = (key, [l.numel() for l in gt_labels], host, ev)

    def _gt_labels_host(self, gt_labels):
        """Per sample the GT labels as host int64 arrays: from forward_train's stashed copy when
        these are the tensors it saw (waits only for that copy), else copied here (a sync)."""
        self.__dict__["_gt_host_hit"] = False
        if all(l.device.type == "cpu" for l in gt_labels):
            return [l.reshape(-1).long().numpy() for l in gt_labels]
        st = self.__dict__.get("_gt_host")
        if st is not None and st[0] == tuple((l.data_ptr(), l.numel()) for l in gt_labels):
            st[3].synchronize()
            flat, counts = st[2].numpy(), st[1]
            self.__dict__["_gt_host_hit"] = True
        else:
            flat = torch.cat([l.reshape(-1).long() for l in gt_labels]).cpu().numpy()
            counts = [l.numel() for l in gt_labels]
        return list(np.split(flat, np.cumsum(counts)[:-1]))

    def _gt_split(self, gtb, gtl, lab_host):
        """{(task, sample): (boxes, labels relative to the task)}: the GT of each task's classes,
        selected once per step by index lists built on the host (lab_host: _gt_labels_host) --
        a boolean-mask selection on the device is a device -> host sync each."""
        out, flag = {}, 0
        for t, ncls in enumerate(self.num_classes):
            for b in range(len(gtl)):
                lh = lab_host[b]
                idx = np.nonzero((lh >= flag) & (lh < flag + ncls))[0]
                if len(idx) == len(lh):
                    out[(t, b)] = (gtb[b], gtl[b] - flag)
                elif len(idx) == 0:
                    out[(t, b)] = (gtb[b][:0], gtl[b][:0])
                else:
                    it = _to_dev_async(torch.from_numpy(idx), gtb[b].device)
                    out[(t, b)] = (gtb[b].index_select(0, it), gtl[b].index_select(0, it) - flag)
            flag += ncls
        return out

    def _assign_all(self, preds, gts, cfg, code_w, between=None):
        """HungarianAssigner3D (hungarian_assigner_3d.py:68-156) for every
        (layer, task, sample): the [Nq, n_gt] cost matrices are built on the
        device (cmt_match_cost, each sample's normalised GT built once for all
        layers), copied to the host in ONE non-blocking transfer and solved by
        scipy's linear_sum_assignment as the reference does; ``between()`` (host
        work that does not need the matches) runs while that copy waits for the
        forward's kernels.  Returns {(l, t, b): (rows, cols) host int64 arrays}
        (absent: no GT)."""
        L, B = preds[0]["center"].shape[:2]
        jobs, costs = [], []
        gnorm = {key: (_normalize_bbox(g).contiguous(), gl.int().contiguous())
                 for key, (g, gl) in gts.items() if g.shape[0] > 0}
        for t, d in enumerate(preds):
            pb_all = torch.cat([d[k].detach() for k in ("center", "height", "dim", "rot", "vel")], -1)  # [L, B, Nq, 10]
            pl_all = d["cls_logits"].detach()
            for l in range(L):
                pb, pl = pb_all[l], pl_all[l]
                for b in range(B):
                    if (t, b) not in gnorm:
                        continue
                    gn, gli = gnorm[(t, b)]
                    cost = T.match_cost(pl[b].contiguous(), pb[b].contiguous(), gn, gli, code_w,
                                        gamma=cfg["gamma"], alpha=cfg["alpha"], cls_weight=cfg["match_cls_weight"],
                                        reg_weight=cfg["match_reg_weight"])
                    jobs.append(((l, t, b), cost.shape))
                    costs.append(cost.reshape(-1))
        out = {}
        if not jobs:
            if between is not None:
                between()
            return out
        cat = torch.cat(costs)                                    # the one device -> host copy
        if cat.is_cuda:
            host_t = torch.empty(cat.shape, dtype=cat.dtype, pin_memory=True)
            host_t.copy_(cat, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host_t, ev = cat, None
        if between is not None:
            between()
        if ev is not None:
            ev.synchronize()
        host = host_t.numpy()
        off = 0
        for key, shape in jobs:
            n = shape[0] * shape[1]
            r, c = linear_sum_assignment(host[off:off + n].reshape(shape))
            off += n
            out[key] = (np.asarray(r, dtype=np.int64), np.asarray(c, dtype=np.int64))
        return out

    def _targets_all(self, L, B, Nq, ncls, t, gts, matches, dev):
        """_get_targets_single of every (layer, sample) of task t at once: labels [L B Nq] (ncls =
        background), gravity-centre targets [L B Nq, 9], box weights [L B Nq, 10], and #pos per
        layer -- three index writes from ONE host -> device copy of the matched (row, GT) pairs
        (rows flattened over layers and samples), instead of three per (layer, sample)."""
        R = L * B * Nq
        labels = torch.full((R,), ncls, dtype=torch.int32, device=dev)
        tgt = torch.zeros((R, 9), dtype=torch.float32, device=dev)
        bw = torch.zeros((R, 10), dtype=torch.float32, device=dev)
        npos = [0] * L
        goff, gb_l, gl_l, g0 = {}, [], [], 0
        for b in range(B):
            g_b, gl_b = gts[(t, b)]
            goff[b] = g0
            gb_l.append(g_b)
            gl_l.append(gl_b)
            g0 += g_b.shape[0]
        rows, cols = [], []
        for l in range(L):
            for b in range(B):
                m = matches.get((l, t, b))
                if m is None:
                    continue
                r, c = m
                rows.append(r + (l * B + b) * Nq)
                cols.append(c + goff[b])
                npos[l] += len(r)
        if rows:
            idx = _to_dev_async(torch.from_numpy(np.stack([np.concatenate(rows), np.concatenate(cols)])), dev)
            gb_t = gb_l[0] if B == 1 else torch.cat(gb_l)
            gl_t = gl_l[0] if B == 1 else torch.cat(gl_l)
            labels[idx[0]] = gl_t[idx[1]].int()
            tgt[idx[0]] = gb_t[idx[1]].float()
            bw.index_fill_(0, idx[0], 1.0)   # (an index_put of a Python scalar copies it to the device: a sync)
        return labels, tgt, bw, npos

    def _box_terms(self, tgt, bw, code_w):
        """normalize the targets, drop non-finite rows (isnotnan), code weights."""
        nt = _normalize_bbox(tgt)
        ok = torch.isfinite(nt).all(-1)
        nt = torch.where(ok[:, None], nt, torch.zeros_like(nt))
        w = bw * code_w[None] * ok[:, None].float()
        return nt.contiguous(), w.contiguous()

    def loss(self, gt_bboxes_3d, gt_labels_3d, preds_dicts, **kwargs):
        """cmt_head.py:815-903 on the native loss / cost kernels.  preds_dicts:
        the multi_apply layout (tuple over tasks of [dict]) or a list of dicts.
        Returns the reference's loss dict."""
        preds = [p[0] if isinstance(p, (list, tuple)) else p for p in preds_dicts]
        cfg = self._loss_cfg()
        dev = preds[0]["center"].device
        code_w = _to_dev_async(torch.tensor(cfg["code_weights"], dtype=torch.float32), dev)
        gtb = [_gravity_boxes(g).to(dev).float() for g in gt_bboxes_3d]
        gtl = [l.to(dev).long() for l in gt_labels_3d]
        L, B = preds[0]["center"].shape[:2]
        eps = float(torch.finfo(torch.float32).eps)   # mmdet weight_reduce_loss avg_factor + eps
        lab_host = self._gt_labels_host(list(gt_labels_3d))
        gts = self._gt_split(gtb, gtl, lab_host)
        # the per-task work that does not need the matches is issued while the cost matrices' copy
        # to the host waits for the forward's kernels (_assign_all's between)
        pre = {}

        def between():
            flag = 0
            for t, d in enumerate(preds):
                ncls = self.num_classes[t]
                pbs = torch.cat([d[k] for k in ("center", "height", "dim", "rot", "vel")], -1).unbind(0)
                pls = d["cls_logits"].unbind(0)
                md = d.get("dn_mask_dict")
                dn = (self._dn_prep(d, md, ncls, code_w, self._dn_rows_host(md, lab_host, flag, ncls))
                      if md is not None and md["pad_size"] > 0 else None)
                pre[t] = (pbs, pls, dn)
                flag += ncls
        matches = self._assign_all(preds, gts, cfg, code_w, between=between)
        # reduce_mean of the DN target count (cmt_head_coop.py:686): the same for every layer and task, so
        # one all-reduce per step -- issued on EVERY rank, also when its frames carry no GT (a rank that
        # skipped it would pair the next collective, the gradient all-reduce, with this one)
        md0 = next((d.get("dn_mask_dict") for d in preds if d.get("dn_mask_dict") is not None), None)
        num_tgt = float(md0["known_indice"].numel()) if md0 is not None else 0.0
        if dist.is_available() and dist.is_initialized():
            nt_t = torch.tensor([num_tgt], device=dev)
            dist.all_reduce(nt_t)
            num_tgt = float(nt_t.item()) / dist.get_world_size()
        num_tgt = max(num_tgt, 1.0)
        losses = {}
        # per task, once: the layers' box / logit views (one unbind each, so the backward writes every
        # layer's gradient into one buffer instead of a zero-filled full copy per selected layer), the
        # layer-invariant DN terms and every layer's matching targets; then per layer ONE autograd
        # node (ops.layer_loss: the matching and DN focal / L1 terms, nan_to_num, dn_weight)
        tot = None
        for t, d in enumerate(preds):
            ncls = self.num_classes[t]
            Nq = d["cls_logits"].shape[2]
            pbs, pls, dn = pre[t]
            labels, tgt, bw, npos = self._targets_all(L, B, Nq, ncls, t, gts, matches, dev)
            nt, w = self._box_terms(tgt, bw, code_w)
            lw = torch.ones(B * Nq, dtype=torch.float32, device=dev)
            R = B * Nq
            per_layer = []
            for l in range(L):
                nn_ = R - npos[l]
                lcfg = dict(gamma=cfg["gamma"], alpha=cfg["alpha"], cls_weight=cfg["cls_weight"],
                            box_weight=cfg["box_weight"], cls_avg=max(npos[l] + 0.1 * nn_, 1.0) + eps,
                            box_avg=float(npos[l]) + eps)
                if dn is not None:
                    # mmdet's loss weights times dn_weight; the box term only when the task has DN rows
                    dcfg = dict(gamma=cfg["gamma"], alpha=cfg["alpha"], cls_weight=cfg["cls_weight"] * self.dn_weight,
                                box_weight=cfg["box_weight"] * self.dn_weight * (1.0 if dn["any_task"] else 0.0),
                                cls_avg=dn["cls_avg"] + eps, box_avg=num_tgt + eps)
                    v = ops.layer_loss(pls[l].reshape(-1, ncls), pbs[l].reshape(-1, 10), labels[l * R:(l + 1) * R],
                                       lw, nt[l * R:(l + 1) * R], w[l * R:(l + 1) * R], lcfg,
                                       dn["pls"][l], dn["pbs"][l], dn["kl"], dn["lw"], dn["ntg"], dn["w"], dcfg)
                else:
                    v = ops.layer_loss(pls[l].reshape(-1, ncls), pbs[l].reshape(-1, 10), labels[l * R:(l + 1) * R],
                                       lw, nt[l * R:(l + 1) * R], w[l * R:(l + 1) * R], lcfg)
                per_layer.append(v)
            tot = per_layer if tot is None else [[a + b_ for a, b_ in zip(x, y)] for x, y in zip(tot, per_layer)]
        for l in range(L):
            key = "" if l == L - 1 else f"d{l}."
            v = tot[l]
            losses[key + "loss_cls"] = v[0]
            losses[key + "loss_bbox"] = v[1]
            if len(v) > 2:
                losses[key + "dn_loss_cls"] = v[2]
                losses[key + "dn_loss_bbox"] = v[3]
        return losses

    def _dn_rows_host(self, md, lab_host, flag, ncls):
        """The DN rows of one task (known_labels_raw of its classes, cmt_head.py:790-792) from the
        host labels: (any row of the task, the rows to keep -- all when none), or None when
        forward_train's stashed labels are not the ones given to loss (then _dn_prep selects on the
        device)."""
        if md is None or not self.__dict__.get("_gt_host_hit", False):
            return None
        if sum(len(x) for x in lab_host) * md["groups"] != md["known_labels_raw"].numel():
            return None
        rep = np.tile(np.concatenate(lab_host), md["groups"])
        tm = (rep >= flag) & (rep < flag + ncls)
        anyt = bool(tm.any())
        return anyt, (np.nonzero(tm)[0] if anyt else np.arange(len(rep)))

    def _dn_prep(self, d, md, ncls, code_w, rows_host=None):
        """The layer-invariant part of _dn_loss_single_task (cmt_head.py:760-806): the known
        queries' logits / boxes of every layer (one gather), targets, weights and averages.
        rows_host: _dn_rows_host's (any_task, rows) -- without it the rows are selected on the
        device (two syncs)."""
        kl, kb = md["known_lbs_bboxes"]
        raw = md["known_labels_raw"]
        bid = md["batch_idx"][md["known_indice"]]
        mk = md["map_known_indice"]
        pl = d["dn_cls_logits"][:, bid, mk]                                         # [L, nk, ncls]
        pb = torch.cat([d["dn_" + k] for k in ("center", "height", "dim", "rot", "vel")], -1)[:, bid, mk]
        num_tgt = md["known_indice"].numel()
        if rows_host is not None:
            any_task = rows_host[0]
            rows = _to_dev_async(torch.from_numpy(rows_host[1].astype(np.int64)), pl.device)
        else:
            task_mask = raw != ncls
            any_task = bool(task_mask.any())
            rows = (task_mask if any_task else torch.ones_like(task_mask)).nonzero().squeeze(1)
        ntg, w = self._box_terms(kb[rows].float(), torch.ones((rows.numel(), 10), device=pl.device), code_w)
        return dict(pls=pl.unbind(0), pbs=pb[:, rows].unbind(0), kl=kl.int(), ntg=ntg, w=w, any_task=any_task,
                    cls_avg=max(num_tgt * 3.14159 / 6 * self.split ** 3, 1),
                    lw=torch.ones(pl.shape[1], dtype=torch.float32, device=pl.device))
