"""PETR decoder building blocks with the reference's registry names, kwargs
and state_dict layout, executed by the gfx950 kernels.

Reference: projects/mmdet3d_plugin/models/utils/petr_transformer.py
  PETRMultiheadFlashAttention 182-321, PETRTransformerDecoder 324-371,
  PETRTransformerDecoderLayer 374-487,
and the mmcv 1.6.2 classes the configs instantiate through it
(MultiheadAttention, FFN, BaseTransformerLayer, TransformerLayerSequence;
not vendored -- restated from the pinned version).

Two execution paths:
  * module-level ``forward`` methods: the reference's per-module API on
    sequence-first [N, B, C] tensors (each op one or more native launches);
  * ``PETRTransformerDecoder.run_rows``: the fused decoder used by the heads --
    the K/V projections of all layers are hoisted into ONE GEMM over the
    memory (memory and key_pos are layer-invariant, cmt_transformer.py:84-127),
    positional adds are fused into GEMM prologues, residual adds into GEMM
    epilogues, and each layer's norms.2 LayerNorm is fused with the shared
    post_norm (+ nan_to_num / coop max) in one wavefront-reduction kernel.
"""
import copy
import math
import warnings

import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import native
from ...registry import (ATTENTION, FEEDFORWARD_NETWORK, TRANSFORMER_LAYER, TRANSFORMER_LAYER_SEQUENCE,
                         build_from_cfg)
from ...profiling import timed
from ...runtime import OPTIONS, SPLIT, get_precision, op_empty
from .attention import FlashMHA, project_attend_project
from .packing import PackCache, to_dtype

__all__ = ["FFN", "MultiheadAttention", "PETRMultiheadFlashAttention", "PETRMultiheadAttention",
           "PETRTransformerDecoderLayer", "PETRTransformerDecoder"]


def _wo(lw):
    """Chain A's out_proj weights: fragment-major when packed (registers), else row-major (LDS ring)."""
    return lw["sa_owp"] if lw.get("sa_owp") is not None else lw["sa_ow"]


def _b1w(lw):
    """Chain B1's out_proj and fc1 weights: row-major (f16 / bf16 chains) or fragment-major pair
    packs (the split chains)."""
    if lw.get("ca_owp") is not None:
        return lw["ca_owp"], lw["f1_wp"]
    return lw["ca_ow"], lw["f1_w"]


def _rows(x):
    """[N, B, C] -> contiguous fp32 [N*B, C]."""
    return x.reshape(-1, x.shape[-1]).contiguous().float()


def _grad_mode(module):
    """Training forward on the differentiable native ops (train_ops) instead of
    the fused inference kernels."""
    return module.training and torch.is_grad_enabled()


def dn_mask_params(mask):
    """(pad_size, single_pad) of the DN self-attention mask of prepare_for_dn
    (cmt_head.py:386-398: True = hidden; the matching queries never see the DN
    queries, DN group i sees only itself among the DN queries) -- the structure
    the native kernels apply from these two numbers.  Any other mask raises."""
    m = mask.bool()
    if m.dim() != 2 or m.shape[0] != m.shape[1]:
        raise NotImplementedError("only [T, T] DN self-attention masks are supported natively")
    T = m.shape[0]
    pad = int(m[-1].sum().item())
    if pad == 0:
        if bool(m.any()):
            raise NotImplementedError("only the DN query mask of prepare_for_dn is supported natively")
        return 0, 0
    single = int((~m[0]).sum().item()) - (T - pad)
    if single <= 0 or pad % single:
        raise NotImplementedError("only the DN query mask of prepare_for_dn is supported natively")
    idx = torch.arange(T, device=m.device)
    q, k = idx[:, None], idx[None, :]
    want = (k < pad) & ((q >= pad) | (k // single != q // single))
    if not torch.equal(want, m):
        raise NotImplementedError("only the DN query mask of prepare_for_dn is supported natively")
    return pad, single


def train_layer(lay, tgt, qpos, memk, mem, *, pad=0, group=0, dropout=True, cross_fp16=True, seed=0, seed_dev=None,
                kv=None, li=0):
    """One PETRTransformerDecoderLayer in training (petr_transformer.py:374-487,
    mmcv BaseTransformerLayer post-norm walk) on the differentiable native ops:
    rows batch-first [B, N, C]; memk = memory + key_pos.  The self-attention
    core applies the DN mask (pad, group) and attn_drop, both attentions the
    dropout_layer after their out-projection (mmcv's deprecated ``dropout``
    kwarg sets both, 0.1 in every config); the cross core emulates flash-attn's
    fp16 inputs when cross_fp16.  memk / mem may be lists, one [B, Nk_a, C] pair
    per agent whose queries are the consecutive B-row blocks of tgt / qpos: the
    query-side products run once for all agents, the cross-attention per agent.  kv: per agent
    the (holder, token) of train_ops.kv_all -- every layer's K / V projected up front -- and li
    this layer's index in them (then memk / mem are not read here)."""
    from . import train_ops as ops
    sa, ca, ffn, nm = lay.attentions[0], lay.attentions[1], lay.ffns[0], lay.norms
    H = sa.num_heads

    def drop(x, p):
        return F.dropout(x, p, True) if dropout and p > 0 else x
    w = sa.attn
    wq, wk, wv = w.in_proj_weight.chunk(3)
    bq, bk, bv = w.in_proj_bias.chunk(3) if w.in_proj_bias is not None else (None, None, None)
    qi = tgt + qpos
    o = ops.attention(ops.linear(qi, wq, bq), ops.linear(qi, wk, bk), ops.linear(tgt, wv, bv), H, dn_pad=pad,
                      dn_group=group, dropout_p=sa.attn_drop_p if dropout else 0.0, seed=seed, seed_dev=seed_dev)
    tgt = ops.layer_norm(tgt + drop(ops.linear(o, w.out_proj.weight, w.out_proj.bias), sa.drop_prob),
                         nm[0].weight, nm[0].bias, nm[0].eps)
    w = ca.attn
    wq, wk, wv = w.in_proj_weight.chunk(3)
    bq, bk, bv = w.in_proj_bias.chunk(3) if w.in_proj_bias is not None else (None, None, None)
    qx = ops.linear(tgt + qpos, wq, bq)
    if kv is not None:
        qxs = qx.split(qx.shape[0] // len(kv), 0) if len(kv) > 1 else (qx,)
        o = [ops.cross_attention(qxs[i], tok, hol, li, H, fp16=cross_fp16) for i, (hol, tok) in enumerate(kv)]
        o = torch.cat(o, 0) if len(o) > 1 else o[0]
    elif isinstance(mem, (list, tuple)):
        # split, not slicing: its backward is one cat where each slice's is a zero fill + copy + add
        qxs = qx.split(qx.shape[0] // len(mem), 0)
        o = torch.cat([ops.attention(qxs[i], ops.linear(mk, wk, bk), ops.linear(m, wv, bv), H,
                                     fp16=cross_fp16) for i, (mk, m) in enumerate(zip(memk, mem))], 0)
    else:
        o = ops.attention(qx, ops.linear(memk, wk, bk), ops.linear(mem, wv, bv), H, fp16=cross_fp16)
    tgt = ops.layer_norm(tgt + drop(ops.linear(o, w.out_proj.weight, w.out_proj.bias), ca.drop_prob),
                         nm[1].weight, nm[1].bias, nm[1].eps)
    l1, l2 = ffn.layers[0][0], ffn.layers[1]
    h = torch.relu(ops.linear(tgt, l1.weight, l1.bias))
    return ops.layer_norm(tgt + ops.linear(h, l2.weight, l2.bias), nm[2].weight, nm[2].bias, nm[2].eps)


@FEEDFORWARD_NETWORK.register_module()
class FFN(nn.Module):
    """mmcv 1.6.2 FFN: layers = Sequential(Sequential(Linear, act, Dropout) x (num_fcs-1),
    Linear, Dropout); out = identity + layers(x) when add_identity."""

    def __init__(self, embed_dims=256, feedforward_channels=1024, num_fcs=2, act_cfg=dict(type="ReLU", inplace=True),
                 ffn_drop=0.0, dropout_layer=None, add_identity=True, init_cfg=None, **kwargs):
        super().__init__()
        assert num_fcs >= 2
        if act_cfg.get("type", "ReLU") != "ReLU":
            raise NotImplementedError("only ReLU FFNs are used by CMT configs")
        self.embed_dims = embed_dims
        self.feedforward_channels = feedforward_channels
        self.num_fcs = num_fcs
        layers = []
        c_in = embed_dims
        for _ in range(num_fcs - 1):
            layers.append(nn.Sequential(nn.Linear(c_in, feedforward_channels), nn.ReLU(inplace=True),
                                        nn.Dropout(ffn_drop)))
            c_in = feedforward_channels
        layers.append(nn.Linear(feedforward_channels, embed_dims))
        layers.append(nn.Dropout(ffn_drop))
        self.layers = nn.Sequential(*layers)
        self.dropout_layer = nn.Identity()
        self.add_identity = add_identity
        self._pack = PackCache()

    def packed(self, prec):
        lins = [m[0] for m in self.layers[:-2]] + [self.layers[-2]]
        return self._pack.get("w", [l.weight for l in lins], prec.name,
                              lambda: [to_dtype(l.weight, prec.gemm) for l in lins])

    def forward(self, x, identity=None):
        if _grad_mode(self):
            from . import train_ops as ops
            h = x
            lins = [m[0] for m in self.layers[:-2]] + [self.layers[-2]]
            for i, lin in enumerate(lins):
                h = ops.linear(h, lin.weight, lin.bias)
                if i < len(lins) - 1:
                    h = F.dropout(torch.relu(h), self.layers[i][2].p, True)
            return (identity if identity is not None else x) + F.dropout(h, self.layers[-1].p, True)
        prec = get_precision()
        ws = self.packed(prec)
        shape = x.shape
        h = _rows(x)
        lins = [m[0] for m in self.layers[:-2]] + [self.layers[-2]]
        for i, (lin, w) in enumerate(zip(lins, ws)):
            last = i == len(lins) - 1
            R = None
            if last and self.add_identity:
                R = _rows(identity if identity is not None else x)
            h = native.linear(h, w, lin.bias, relu=not last, R=R)
        return h.view(*shape[:-1], self.embed_dims)


class _MHABase(nn.Module):
    """Shared forward of mmcv MultiheadAttention / PETRMultiheadFlashAttention
    (sequence-first tensors, identity connection, positional encodings added
    to query and key: petr_transformer.py:282-321)."""
    fp16_core = False   # True for the flash-attn based wrapper

    def _weights(self):
        raise NotImplementedError

    drop_prob = 0.0     # dropout_layer after the out-projection (training)
    attn_drop_p = 0.0   # attention-probability dropout of the core (training; nn.MultiheadAttention only)

    def forward(self, query, key=None, value=None, identity=None, query_pos=None, key_pos=None, attn_mask=None,
                key_padding_mask=None, **kwargs):
        if attn_mask is not None or _grad_mode(self):
            return self._forward_t(query, key, value, identity, query_pos, key_pos, attn_mask)
        if key_padding_mask is not None and bool(key_padding_mask.any()):
            raise NotImplementedError("non-trivial key_padding_mask is not used by CMT configs")
        if key is None:
            key = query
        if value is None:
            value = key
        if identity is None:
            identity = query
        if key_pos is None and query_pos is not None:
            if query_pos.shape == key.shape:
                key_pos = query_pos
            else:
                warnings.warn(f"position encoding of key is missing in {self.__class__.__name__}.")
        if self.batch_first:   # [B, N, C] -> sequence-first rows
            query, key, value, identity = (t.transpose(0, 1) for t in (query, key, value, identity))
            query_pos = query_pos.transpose(0, 1) if query_pos is not None else None
            key_pos = key_pos.transpose(0, 1) if key_pos is not None else None
        Nq, B, C = query.shape
        Nk = key.shape[0]
        prec = get_precision()
        w_in, b_in, w_out, b_out = self._weights(prec)
        adt, rnd = (prec.attn, prec.round_cross_out) if self.fp16_core else (prec.self_attn, False)
        if adt == SPLIT:   # the split core takes head-split pair rows (fused decoder); rows here: exact f32
            adt = torch.float32
        out = project_attend_project(_rows(query), _rows(key), _rows(value),
                                     _rows(query_pos) if query_pos is not None else None,
                                     _rows(key_pos) if key_pos is not None else None,
                                     w_in, b_in, w_out, b_out, _rows(identity), adt, rnd, B=B, Nq=Nq, Nk=Nk,
                                     H=self.num_heads, layout="seq_first")
        out = out.view(Nq, B, C)
        return out.transpose(0, 1) if self.batch_first else out


    def _forward_t(self, query, key, value, identity, query_pos, key_pos, attn_mask):
        """Training (or DN-masked) forward on the differentiable native ops: the
        DN mask goes to the attention kernel as (pad, group) (dn_mask_params)."""
        from . import train_ops as ops
        key = query if key is None else key
        value = key if value is None else value
        identity = query if identity is None else identity
        if key_pos is None and query_pos is not None and query_pos.shape == key.shape:
            key_pos = query_pos
        pad, grp = dn_mask_params(attn_mask) if attn_mask is not None else (0, 0)
        bf = self.batch_first
        t = (lambda x: x) if bf else (lambda x: None if x is None else x.transpose(0, 1))
        q, k, v, idn, qp, kp = (t(x) for x in (query, key, value, identity, query_pos, key_pos))
        qi = q + qp if qp is not None else q
        ki = k + kp if kp is not None else k
        w = self.attn
        wq, wk, wv = w.in_proj_weight.chunk(3)
        bq, bk, bv = w.in_proj_bias.chunk(3) if w.in_proj_bias is not None else (None, None, None)
        training = self.training
        o = ops.attention(ops.linear(qi, wq, bq), ops.linear(ki, wk, bk), ops.linear(v, wv, bv), self.num_heads,
                          dn_pad=pad, dn_group=grp, fp16=self.fp16_core,
                          dropout_p=self.attn_drop_p if training else 0.0,
                          seed=int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if training and self.attn_drop_p else 0)
        y = ops.linear(o, w.out_proj.weight, w.out_proj.bias)
        out = idn + (F.dropout(y, self.drop_prob, True) if training and self.drop_prob > 0 else y)
        return out if bf else out.transpose(0, 1)


@ATTENTION.register_module()
class MultiheadAttention(_MHABase):
    """mmcv 1.6.2 MultiheadAttention wrapper around ``nn.MultiheadAttention``
    (self-attention, attn_cfgs[0] of every config).  ``self.attn`` keeps the
    torch module only as the parameter container (state_dict keys
    ``attn.in_proj_weight`` etc.); the math runs natively.  The reference core
    runs in fp32; here it runs in the policy's attention dtype."""

    def __init__(self, embed_dims, num_heads, attn_drop=0.0, proj_drop=0.0,
                 dropout_layer=dict(type="Dropout", drop_prob=0.0), init_cfg=None, batch_first=False, **kwargs):
        super().__init__()
        if "dropout" in kwargs:   # mmcv 1.6.2: the deprecated kwarg sets attn_drop AND dropout_layer's drop_prob
            attn_drop = kwargs.pop("dropout")
            self.drop_prob = float(attn_drop)
        else:
            self.drop_prob = float((dropout_layer or {}).get("drop_prob", 0.0))
        self.attn_drop_p = float(attn_drop)
        self.embed_dims = embed_dims
        self.num_heads = num_heads
        self.batch_first = batch_first
        self.attn = nn.MultiheadAttention(embed_dims, num_heads, attn_drop, **kwargs)
        self.proj_drop = nn.Dropout(proj_drop)
        self.dropout_layer = nn.Identity()
        self._pack = PackCache()

    def _weights(self, prec):
        a = self.attn
        pk = self._pack.get("w", [a.in_proj_weight, a.out_proj.weight], prec.name, lambda: dict(
            w_in=to_dtype(a.in_proj_weight, prec.gemm), w_out=to_dtype(a.out_proj.weight, prec.gemm)))
        return pk["w_in"], a.in_proj_bias, pk["w_out"], a.out_proj.bias


@ATTENTION.register_module()
class PETRMultiheadFlashAttention(_MHABase):
    """petr_transformer.py:182-321 (FlashMHA inside, batch_first forced True
    at 224 -- the wrapper transposes; here the sequence-first rows are fed to
    the kernel directly through its stride arguments)."""
    fp16_core = True

    def __init__(self, embed_dims, num_heads, attn_drop=0.0, proj_drop=0.0,
                 dropout_layer=dict(type="Dropout", drop_prob=0.0), init_cfg=None, batch_first=True, **kwargs):
        super().__init__()
        if "dropout" in kwargs:   # petr_transformer.py:211-218: attn_drop (FlashMHA's `bias`) and dropout_layer
            attn_drop = kwargs["dropout"]
            self.drop_prob = float(kwargs.pop("dropout"))
        else:
            self.drop_prob = float((dropout_layer or {}).get("drop_prob", 0.0))
        self.attn_drop_p = 0.0   # FlashAttention's attention_dropout keeps its default 0 (attention.py:36)
        self.embed_dims = embed_dims
        self.num_heads = num_heads
        self.batch_first = False   # forward() receives sequence-first tensors (mmcv layer convention)
        self.attn = FlashMHA(embed_dims, num_heads, attn_drop, **kwargs)
        self.proj_drop = nn.Dropout(proj_drop)
        self.dropout_layer = nn.Identity()

    def _weights(self, prec):
        pk = self.attn.packed(prec)
        return pk["w_in"], self.attn.in_proj_bias, pk["w_out"], self.attn.out_proj.bias


@ATTENTION.register_module()
class PETRMultiheadAttention(MultiheadAttention):
    """petr_transformer.py:37-177 (registered, unused by the configs): the
    mmcv MultiheadAttention contract with ``batch_first`` honoured."""


@TRANSFORMER_LAYER.register_module()
class PETRTransformerDecoderLayer(nn.Module):
    """petr_transformer.py:374-487 over mmcv 1.6.2 BaseTransformerLayer
    (post-norm op walk; deprecated ``feedforward_channels``/``ffn_dropout``/
    ``ffn_num_fcs`` kwargs override ``ffn_cfgs`` as in mmcv)."""

    SUPPORTED_ORDER = ("self_attn", "norm", "cross_attn", "norm", "ffn", "norm")

    def __init__(self, attn_cfgs, feedforward_channels=None, ffn_dropout=0.0, operation_order=None,
                 act_cfg=dict(type="ReLU", inplace=True), norm_cfg=dict(type="LN"), ffn_num_fcs=2, with_cp=True,
                 ffn_cfgs=None, batch_first=False, init_cfg=None, **kwargs):
        super().__init__()
        assert len(operation_order) == 6
        assert set(operation_order) == {"self_attn", "norm", "cross_attn", "ffn"}
        self.operation_order = tuple(operation_order)
        self.pre_norm = operation_order[0] == "norm"
        self.use_checkpoint = with_cp
        self.batch_first = batch_first
        num_attn = sum(op in ("self_attn", "cross_attn") for op in operation_order)
        if isinstance(attn_cfgs, dict):
            attn_cfgs = [copy.deepcopy(attn_cfgs) for _ in range(num_attn)]
        assert len(attn_cfgs) == num_attn
        self.attentions = nn.ModuleList(build_from_cfg(c, ATTENTION) for c in attn_cfgs)
        self.embed_dims = self.attentions[0].embed_dims
        ffn_cfgs = copy.deepcopy(ffn_cfgs) if ffn_cfgs is not None else dict(
            type="FFN", embed_dims=self.embed_dims, feedforward_channels=1024, num_fcs=2, ffn_drop=0.0,
            act_cfg=dict(type="ReLU", inplace=True))
        if feedforward_channels is not None:
            ffn_cfgs["feedforward_channels"] = feedforward_channels
        ffn_cfgs["ffn_drop"] = ffn_dropout
        ffn_cfgs["num_fcs"] = ffn_num_fcs
        ffn_cfgs.setdefault("embed_dims", self.embed_dims)
        num_ffns = operation_order.count("ffn")
        self.ffns = nn.ModuleList(build_from_cfg(copy.deepcopy(ffn_cfgs), FEEDFORWARD_NETWORK)
                                  for _ in range(num_ffns))
        if norm_cfg.get("type", "LN") != "LN":
            raise NotImplementedError("only LN norms are used by CMT configs")
        self.norms = nn.ModuleList(nn.LayerNorm(self.embed_dims) for _ in range(operation_order.count("norm")))

    def _norm(self, i, x):
        n = self.norms[i]
        if _grad_mode(self):
            from . import train_ops as ops
            return ops.layer_norm(x, n.weight, n.bias, n.eps)
        rows = _rows(x)
        y = torch.empty_like(rows)
        native.layernorm(rows, n.weight, n.bias, y, rows=rows.shape[0], C=rows.shape[1], ldx=rows.shape[1],
                         ldy=rows.shape[1], eps=n.eps)
        return y.view(x.shape)

    def forward(self, query, key=None, value=None, query_pos=None, key_pos=None, attn_masks=None,
                query_key_padding_mask=None, key_padding_mask=None, **kwargs):
        """mmcv BaseTransformerLayer.forward op walk (post-norm).  In training
        every op runs on the differentiable native ops (with_cp, the
        reference's gradient checkpointing, only trades memory for recompute:
        the step's values and gradients are the same without it)."""
        num_attn = 2
        if attn_masks is None or isinstance(attn_masks, torch.Tensor):
            attn_masks = [attn_masks for _ in range(num_attn)]
        attn_i = norm_i = ffn_i = 0
        identity = query
        for op in self.operation_order:
            if op == "self_attn":
                query = self.attentions[attn_i](query, query, query, identity if self.pre_norm else None,
                                                query_pos=query_pos, key_pos=query_pos,
                                                attn_mask=attn_masks[attn_i], key_padding_mask=query_key_padding_mask)
                attn_i += 1
                identity = query
            elif op == "norm":
                query = self._norm(norm_i, query)
                norm_i += 1
            elif op == "cross_attn":
                query = self.attentions[attn_i](query, key, value, identity if self.pre_norm else None,
                                                query_pos=query_pos, key_pos=key_pos,
                                                attn_mask=attn_masks[attn_i], key_padding_mask=None)
                attn_i += 1
                identity = query
            elif op == "ffn":
                query = self.ffns[ffn_i](query, identity if self.pre_norm else None)
                ffn_i += 1
        return query


@TRANSFORMER_LAYER_SEQUENCE.register_module()
class PETRTransformerDecoder(nn.Module):
    """petr_transformer.py:324-371 over mmcv TransformerLayerSequence."""

    def __init__(self, transformerlayers=None, num_layers=None, post_norm_cfg=dict(type="LN"),
                 return_intermediate=False, init_cfg=None, **kwargs):
        super().__init__()
        if isinstance(transformerlayers, dict):
            transformerlayers = [copy.deepcopy(transformerlayers) for _ in range(num_layers)]
        assert len(transformerlayers) == num_layers
        self.num_layers = num_layers
        self.layers = nn.ModuleList(build_from_cfg(c, TRANSFORMER_LAYER) for c in transformerlayers)
        self.embed_dims = self.layers[0].embed_dims
        self.pre_norm = self.layers[0].pre_norm
        self.return_intermediate = return_intermediate
        self.post_norm = nn.LayerNorm(self.embed_dims) if post_norm_cfg is not None else None
        self._pack = PackCache()

    # ------------------------------------------------------------------
    def forward(self, query, key=None, value=None, query_pos=None, key_pos=None, attn_masks=None,
                query_key_padding_mask=None, key_padding_mask=None, reg_branch=None, **kwargs):
        """Sequence-first API (query [Nq,B,C], key [Nk,B,C]) ->
        [L, Nq, B, C] (return_intermediate) or [1, Nq, B, C]."""
        masked = attn_masks is not None and any(m is not None for m in (attn_masks if isinstance(attn_masks, list)
                                                                       else [attn_masks]))
        if masked or _grad_mode(self):
            # training-time DN queries / gradients: the layer walk on the differentiable native ops
            return self._forward_layers(query, key, value, query_pos, key_pos, attn_masks)
        if value is not None and value is not key and not torch.equal(value, key):
            # the fused path assumes value == key (true for every CMT transformer)
            return self._forward_layers(query, key, value, query_pos, key_pos)
        Nq, B, C = query.shape
        Nk = key.shape[0]
        if not self.fused_supported() or key_pos is None or query_pos is None:
            return self._forward_layers(query, key, value, query_pos, key_pos)
        mem = key.transpose(0, 1).reshape(B * Nk, C).contiguous().float()
        pos = key_pos.transpose(0, 1).reshape(B * Nk, C).contiguous().float()
        qpos = query_pos.transpose(0, 1).reshape(B * Nq, C).contiguous().float()
        tgt0 = query.transpose(0, 1).reshape(B * Nq, C).contiguous().float()
        out = self.run_rows(mem, pos, qpos, B=B, Nk=Nk, Nq=Nq, post_flags=0, tgt0=tgt0)
        out = out.view(self.num_layers, B, Nq, C).transpose(1, 2)
        return out if self.return_intermediate else out[-1:]

    def _forward_layers(self, query, key, value, query_pos, key_pos, attn_masks=None):
        inter = []
        for layer in self.layers:
            query = layer(query, key, value, query_pos=query_pos, key_pos=key_pos, attn_masks=attn_masks)
            if self.return_intermediate:
                inter.append(self._post(query) if self.post_norm is not None else query)
        if not self.return_intermediate:
            return (self._post(query) if self.post_norm is not None else query)[None]
        return torch.stack(inter)

    def train_rows(self, tgt, qpos, mem, pos, *, pad=0, group=0, dropout=True, cross_fp16=True, seed_dev=None):
        """The decoder in training on batch-first rows (tgt / qpos [B, Nq, C],
        mem / pos [B, Nk, C]): every layer (train_layer) and its post_norm
        (petr_transformer.py:347-371), nan_to_num (cmt_head.py:499) ->
        [L, B, Nq, C], differentiable in every input and parameter.
        seed_dev: int32 device tensor [1], the attention dropout seed read on the device
        (no host draw: the graph-captured form, train_engine._decoder_t).  mem / pos may be
        lists (one per agent, train_layer): every agent's decoder in one walk."""
        from . import train_ops as ops
        memk = [m + p for m, p in zip(mem, pos)] if isinstance(mem, (list, tuple)) else mem + pos
        # every layer's cross-attention K / V of each agent in two Linears of width L C (train_ops.kv_all)
        C = self.embed_dims
        lkv = []
        for lay in self.layers:
            w = lay.attentions[1].attn
            _, wk, wv = w.in_proj_weight.chunk(3)
            _, bk, bv = w.in_proj_bias.chunk(3) if w.in_proj_bias is not None else (None, None, None)
            lkv.append((wk, bk, wv, bv))
        agents = list(zip(memk, mem)) if isinstance(mem, (list, tuple)) else [(memk, mem)]
        kv = [ops.kv_all(mk, m, lkv) for mk, m in agents]
        outs = []
        if seed_dev is not None:
            seed0 = 0
        else:
            seed0 = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if dropout else 0
        for li, lay in enumerate(self.layers):
            tgt = train_layer(lay, tgt, qpos, memk, mem, pad=pad, group=group, dropout=dropout,
                              cross_fp16=cross_fp16, seed=seed0 + li, seed_dev=seed_dev, kv=kv, li=li)
            outs.append(ops.layer_norm(tgt, self.post_norm.weight, self.post_norm.bias, self.post_norm.eps))
        return torch.nan_to_num(torch.stack(outs))

    def _post(self, x):
        if _grad_mode(self):
            from . import train_ops as ops
            n = self.post_norm
            return ops.layer_norm(x, n.weight, n.bias, n.eps)
        rows = _rows(x)
        y = torch.empty_like(rows)
        n = self.post_norm
        native.layernorm(rows, n.weight, n.bias, y, rows=rows.shape[0], C=rows.shape[1], ldx=rows.shape[1],
                         ldy=rows.shape[1], eps=n.eps)
        return y.view(x.shape)

    def fused_supported(self):
        l0 = self.layers[0]
        return (l0.operation_order == PETRTransformerDecoderLayer.SUPPORTED_ORDER and self.post_norm is not None
                and self.embed_dims == 256 and all(len(l.ffns) == 1 and l.ffns[0].num_fcs == 2 for l in self.layers)
                and all(a.num_heads * 32 == self.embed_dims for l in self.layers for a in l.attentions))

    # ------------------------------------------------------------------
    def _chain_ok(self):
        """Row-block chains (cmt_chain) need C = 256, FFN 1024 and one LN eps."""
        if self.embed_dims != 256 or self.post_norm is None:
            return False
        eps = {n.eps for l in self.layers for n in l.norms} | {self.post_norm.eps}
        return len(eps) == 1 and all(l.ffns[0].feedforward_channels == 1024 for l in self.layers)

    def _chain_pack(self, prec):
        """Per layer the fp32 parameter blocks of chains A and B (cmt_hip.h cmt_chain_args.prm)."""
        params = [p for p in self.parameters()]

        def build():
            C, L = self.embed_dims, self.num_layers
            dev = self.post_norm.weight.device

            def vec(t, n):
                return t.detach().float().reshape(-1) if t is not None else torch.zeros(n, device=dev)

            A, Bk = [], []
            for l, lay in enumerate(self.layers):
                sa, ca, ffn, nm = lay.attentions[0].attn, lay.attentions[1].attn, lay.ffns[0], lay.norms
                cbq = ca.in_proj_bias[:C] if ca.in_proj_bias is not None else None
                A.append(torch.cat([vec(sa.out_proj.bias, C), vec(nm[0].weight, C), vec(nm[0].bias, C),
                                    vec(cbq, C)]).contiguous())
                nxt = self.layers[l + 1].attentions[0].attn.in_proj_bias if l + 1 < L else None
                Bk.append(torch.cat([vec(ca.out_proj.bias, C), vec(nm[1].weight, C), vec(nm[1].bias, C),
                                     vec(ffn.layers[0][0].bias, 4 * C), vec(ffn.layers[1].bias, C),
                                     vec(nm[2].weight, C), vec(nm[2].bias, C), vec(self.post_norm.weight, C),
                                     vec(self.post_norm.bias, C), vec(nxt, 3 * C)]).contiguous())
            return dict(A=A, B=Bk)
        return self._pack.get("chain", params, prec.name, build)

    def packed(self, prec):
        params = [p for p in self.parameters()]

        def build():
            L, C = self.num_layers, self.embed_dims
            g = prec.gemm
            layers = []
            kw, kb, vw, vb = [], [], [], []
            for lay in self.layers:
                sa = lay.attentions[0].attn
                ca = lay.attentions[1].attn
                ffn = lay.ffns[0]
                chain = g in (torch.float16, torch.bfloat16)   # the row-block chains' fragment-major copies
                # the split chains (rowchain_x3.hip): every chain weight as a fragment-major pair pack
                sp = g == SPLIT and self._chain_ok() and tuple(ffn.layers[1].weight.shape) == (256, 1024)
                layers.append(dict(
                    sa_w=to_dtype(sa.in_proj_weight, g), sa_b=sa.in_proj_bias.detach().contiguous(),
                    # chain B2's copy of the in_proj weights, fragment-major (cmt_hip.h cmt_chain_args.Wn)
                    sa_wp=(native.pack_chain_wn(to_dtype(sa.in_proj_weight, g))
                           if chain and tuple(sa.in_proj_weight.shape) == (768, 256) else None),
                    sa_ow=to_dtype(sa.out_proj.weight, g), sa_ob=sa.out_proj.bias.detach().contiguous(),
                    # chain A's copy of the self-attn out_proj weights, fragment-major (cmt_hip.h wo_frag)
                    sa_owp=(native.pack_chain_wn(to_dtype(sa.out_proj.weight, g))
                            if chain and C == 256 else None),
                    ca_wq=to_dtype(ca.in_proj_weight[:C], g),
                    ca_wqp=(native.pack_chain_wn(to_dtype(ca.in_proj_weight[:C], g))
                            if chain and C == 256 else None),
                    ca_bq=ca.in_proj_bias[:C].detach().contiguous() if ca.in_proj_bias is not None else None,
                    ca_ow=to_dtype(ca.out_proj.weight, g),
                    ca_ob=ca.out_proj.bias.detach().contiguous() if ca.out_proj.bias is not None else None,
                    f1_w=to_dtype(ffn.layers[0][0].weight, g), f1_b=ffn.layers[0][0].bias.detach().contiguous(),
                    f2_w=to_dtype(ffn.layers[1].weight, g), f2_b=ffn.layers[1].bias.detach().contiguous(),
                    f2_wp=(native.pack_chain_fc2(to_dtype(ffn.layers[1].weight, g))
                           if chain and tuple(ffn.layers[1].weight.shape) == (256, 1024) else None),
                    norms=[(n.weight.detach().contiguous(), n.bias.detach().contiguous(), n.eps)
                           for n in lay.norms]))
                if sp:
                    lw = layers[-1]
                    lw.update(sa_wp=native.pack_chain_pair(lw["sa_w"].view(3 * C, 2, C)),
                              sa_owp=native.pack_chain_pair(lw["sa_ow"].view(C, 2, C)),
                              ca_wqp=native.pack_chain_pair(lw["ca_wq"].view(C, 2, C)),
                              ca_owp=native.pack_chain_pair(lw["ca_ow"].view(C, 2, C)),
                              f1_wp=native.pack_chain_pair(lw["f1_w"].view(4 * C, 2, C)),
                              f2_wp=native.pack_chain_fc2_pair(lw["f2_w"].view(C, 2, 4 * C)))
                kw.append(ca.in_proj_weight[C:2 * C])
                vw.append(ca.in_proj_weight[2 * C:])
                if ca.in_proj_bias is not None:
                    kb.append(ca.in_proj_bias[C:2 * C])
                    vb.append(ca.in_proj_bias[2 * C:])
            kv_w = to_dtype(torch.cat(kw + vw, 0), g)
            kv_b = torch.cat(kb + vb, 0).detach().contiguous() if kb else None
            kv_wp = None
            if C == 256 and kv_w.dtype in (torch.float16, torch.bfloat16):
                kv_wp = native.kv_pack(kv_w)
            elif C == 256 and kv_w.dtype == SPLIT:
                # split pairs: the fragment-packed hi halves, then the lo halves (cmt_kv_proj's split form)
                b = kv_w.view(torch.float16)
                kv_wp = torch.cat([native.kv_pack(b[:, 0].contiguous()),
                                   native.kv_pack(b[:, 1].contiguous())]).view(SPLIT)
            return dict(layers=layers, kv_w=kv_w, kv_wp=kv_wp, kv_b=kv_b,
                        post=(self.post_norm.weight.detach().contiguous(),
                              self.post_norm.bias.detach().contiguous(), self.post_norm.eps))
        return self._pack.get("decoder", params, prec.name, build)

    def run_rows(self, mem, pos, qpos, *, B, Nk, Nq, out=None, post_flags=native.LN_NAN_TO_NUM, prec=None,
                 tgt0=None, kv_operands=None, out16=None, state=None):
        """Fused decoder.  mem/pos: [B*Nk, C] fp32 batch-major rows, qpos:
        [B*Nq, C] fp32.  Writes the post-normed layer outputs to
        out [L, B*Nq, C] (fp32) with ``post_flags`` (nan_to_num / max-into).
        Under an f16/bf16 policy the producers may hand over the K/V GEMM
        operands already in the compute dtype: kv_operands = (lowp(mem),
        lowp(mem + pos)); mem/pos are then unused.  ``out16`` (f16/bf16 policy
        only): a compute-dtype copy of ``out`` for the task-head GEMM."""
        if not self.fused_supported():
            raise NotImplementedError("fused decoder supports the CMT post-norm layout (C=256, 8x32 heads)")
        prec = get_precision(prec)
        if prec.gemm != torch.float32:
            return self._run_rows_lowp(mem, pos, qpos, B=B, Nk=Nk, Nq=Nq, out=out, post_flags=post_flags, prec=prec,
                                       tgt0=tgt0, kv_operands=kv_operands, out16=out16, state=state)
        pk = self.packed(prec)
        L, C, H = self.num_layers, self.embed_dims, self.embed_dims // 32
        dev = mem.device
        adt = prec.attn
        f32 = torch.float32
        rows = B * Nq
        if out is None:
            out = torch.empty((L, rows, C), dtype=f32, device=dev)
        scale = 1.0 / math.sqrt(32.0)
        # K/V of every layer in one GEMM: head-split [B][2L*H][Nk][32]
        kv = torch.empty((B * 2 * L * C * Nk,), dtype=adt, device=dev)
        native.gemm(mem, pk["kv_w"], kv, M=B * Nk, N=2 * L * C, K=C, lda=C, ldw=C, ldc=0, bias=pk["kv_b"],
                    A2=pos, lda2=C, a2_cols=L * C, headsplit_rows=Nk)
        # target = zeros_like(query_embed) in every CMT transformer (cmt_transformer.py:114)
        tgt = tgt0.clone() if tgt0 is not None else torch.zeros((rows, C), dtype=f32, device=dev)
        qkv = torch.empty((B * 3 * C * Nq,), dtype=prec.self_attn, device=dev)
        qc = torch.empty((B * C * Nq,), dtype=adt, device=dev)
        o = torch.empty((rows, C), dtype=f32, device=dev)
        t1 = torch.empty_like(o)
        t1n = torch.empty_like(o)
        hf = torch.empty((rows, pk["layers"][0]["f1_w"].shape[0]), dtype=f32, device=dev)
        ws_bytes = max(native.attn_workspace_bytes(B=B, H=H, Nq=Nq, Nk=Nk),
                       native.attn_workspace_bytes(B=B, H=H, Nq=Nq, Nk=Nq))
        ws = torch.empty((max(ws_bytes, 1),), dtype=torch.uint8, device=dev)
        FF = hf.shape[1]
        for l, lw in enumerate(pk["layers"]):
            # --- self attention (mmcv MultiheadAttention): q=k=tgt+qpos, v=tgt
            native.gemm(tgt, lw["sa_w"], qkv, M=rows, N=3 * C, K=C, lda=C, ldw=C, ldc=0, bias=lw["sa_b"],
                        A2=qpos, lda2=C, a2_cols=2 * C, headsplit_rows=Nq)
            native.attention(qkv, qkv, qkv, o, B=B, H=H, Nq=Nq, Nk=Nq,
                             q_strides=(3 * C * Nq, 32 * Nq, 32), k_strides=(3 * C * Nq, 32 * Nq, 32),
                             v_strides=(3 * C * Nq, 32 * Nq, 32), k_offset=C * Nq, v_offset=2 * C * Nq,
                             o_strides=(Nq * C, C), scale=scale, workspace=ws)
            native.gemm(o, lw["sa_ow"], t1, M=rows, N=C, K=C, lda=C, ldw=C, ldc=C, bias=lw["sa_ob"], R=tgt, ldr=C)
            w0, b0, e0 = lw["norms"][0]
            native.layernorm(t1, w0, b0, t1n, rows=rows, C=C, ldx=C, ldy=C, eps=e0)
            # --- cross attention (PETRMultiheadFlashAttention): q=x+qpos, k=mem+pos, v=mem
            native.gemm(t1n, lw["ca_wq"], qc, M=rows, N=C, K=C, lda=C, ldw=C, ldc=0, bias=lw["ca_bq"],
                        A2=qpos, lda2=C, a2_cols=C, headsplit_rows=Nq)
            with timed("cross_attn"):
                native.attention(qc, kv, kv, o, B=B, H=H, Nq=Nq, Nk=Nk,
                                 q_strides=(C * Nq, 32 * Nq, 32), k_strides=(2 * L * C * Nk, 32 * Nk, 32),
                                 v_strides=(2 * L * C * Nk, 32 * Nk, 32), k_offset=l * C * Nk,
                                     v_offset=(L + l) * C * Nk, o_strides=(Nq * C, C), scale=scale, workspace=ws,
                                 round_output=prec.round_cross_out)
            native.gemm(o, lw["ca_ow"], t1, M=rows, N=C, K=C, lda=C, ldw=C, ldc=C, bias=lw["ca_ob"], R=t1n, ldr=C)
            w1, b1, e1 = lw["norms"][1]
            native.layernorm(t1, w1, b1, o, rows=rows, C=C, ldx=C, ldy=C, eps=e1)   # o <- LN1 output
            # --- FFN
            native.gemm(o, lw["f1_w"], hf, M=rows, N=FF, K=C, lda=C, ldw=C, ldc=FF, bias=lw["f1_b"], relu=True)
            native.gemm(hf, lw["f2_w"], t1, M=rows, N=C, K=FF, lda=FF, ldw=FF, ldc=C, bias=lw["f2_b"], R=o, ldr=C)
            # --- norms.2 -> next query, fused with post_norm -> out[l]
            w2, b2, e2 = lw["norms"][2]
            pw, pb, _pe = pk["post"]
            native.layernorm(t1, w2, b2, tgt, rows=rows, C=C, ldx=C, ldy=C, eps=e2, W2=pw, B2=pb, Y2=out,
                             ldy2=C, flags2=post_flags, y2_offset=l * rows * C)
        return out

    def _use_chain(self, prec):
        """Row-block chains (f16 / bf16 policies, and their split-f16 form under the 'ref'
        policy; CMT_CHAIN=0: separate launches)."""
        return self._chain_ok() and get_precision(prec).gemm != torch.float32 and OPTIONS.chain

    def prologue_ok(self, prec):
        """Whether run_rows takes a lowp_state whose layer 0 up to the
        cross-attention core (it reads only the query embedding) may be queued
        beforehand on another stream, beside the memory-side work (every f16 /
        bf16 / split policy of the fused decoder)."""
        prec = get_precision(prec)
        return prec.gemm != torch.float32 and self.fused_supported()

    def lowp_state(self, *, B, Nk, Nq, prec, device):
        """Working buffers of one lowp decoder run with a zero target
        (allocated on the current stream; lowp_layer0 may then run on another
        one)."""
        prec = get_precision(prec)
        # every packed weight the run reads is built HERE, on the current stream: a pack first
        # built inside lowp_layer0 on the second stream would be read by the main stream's
        # K/V projection with nothing ordering the two
        pk = self.packed(prec)
        chain = self._use_chain(prec)
        if chain:
            self._chain_pack(prec)
        C, H = self.embed_dims, self.embed_dims // 32
        lp, f32, rows = prec.gemm, torch.float32, B * Nq
        FF = pk["layers"][0]["f1_w"].shape[0]
        ws_bytes = max(native.attn_workspace_bytes(B=B, H=H, Nq=Nq, Nk=Nk),
                       native.attn_workspace_bytes(B=B, H=H, Nq=Nq, Nk=Nq))
        # self-attention Q|K|V head-split; a split self-attention core (the 'ref' policy) takes
        # them as f16 pairs, 64 16-bit elements per (head, row): hi 32 | lo 32
        sps = 2 if prec.self_attn == SPLIT else 1
        st = dict(
            chain=chain,
            tgt=torch.empty((rows, C), dtype=f32, device=device),
            tl=op_empty(rows, C, lp, device),                            # lowp(tgt)
            tp=op_empty(rows, C, lp, device),                            # lowp(tgt + qpos)
            qkv=torch.empty((B * 3 * C * Nq * sps,), dtype=prec.self_attn, device=device),
            qc=torch.empty((B * C * Nq,), dtype=prec.attn, device=device),
            ob=op_empty(rows, C, lp, device),                            # attention output (out-proj operand)
            t1n=torch.empty((rows, C), dtype=f32, device=device),
            hf=op_empty(rows, FF, lp, device),
            ws=torch.empty((max(ws_bytes, 1),), dtype=torch.uint8, device=device),
            layer0_done=False, stream=None)
        if chain:
            st["cws"] = torch.empty(native.chain_ws_numel(rows), dtype=f32, device=device)
        else:
            # the N = C out-projection / fc2 GEMMs of the split policy run split-K into KSP fp32
            # partial blocks of t1 (their 64 x 64 tile grid alone covers under a quarter of the
            # CUs); the LayerNorm after each sums the blocks
            st["ksp"] = 4 if lp == SPLIT else 1
            st["t1"] = torch.empty((st["ksp"], rows, C), dtype=f32, device=device)
            st["o"] = torch.empty((rows, C), dtype=f32, device=device)
            # (cmt_gemm_ln on pairs -- out-projection + LayerNorm in one launch, 32 full rows per
            # workgroup -- measured slower in the frame: 572 vs 590 frames/s alternating A/B; its
            # 29 workgroups each stream the 256 KB of pair weights, profiles/r3f_fused_ln_ab.txt)
        return st

    def lowp_layer0(self, st, qpos, *, B, Nq, prec, first_ops_ready=False):
        """Layer 0 up to the cross-attention core: the zero target's operands
        (add_cast), the self-attention in_proj and core, out_proj + norms[0]
        and the cross-attention Q projection (chain A on the chain path).  None
        of it reads the memory side, so the head runs it on a second stream
        beside shared_conv / the encodings / the K/V projection (the stream it
        runs on is recorded and joined before the first cross-attention)."""
        prec = get_precision(prec)
        pk = self.packed(prec)
        C, H, rows = self.embed_dims, self.embed_dims // 32, B * Nq
        l0 = pk["layers"][0]
        if not first_ops_ready:   # else written by the query embedding's last kernel (masked_view_sum_ex)
            native.add_cast(None, rows=rows, C=C, Yl=st["tl"], Yp=st["tp"], P=qpos)
        native.gemm(st["tl"], l0["sa_w"], st["qkv"], M=rows, N=3 * C, K=C, lda=C, ldw=C, ldc=0, bias=l0["sa_b"],
                    A2=st["tp"], lda2=C, a2_cols=2 * C, headsplit_rows=Nq)
        self._self_attn(st, B=B, H=H, Nq=Nq, C=C)
        if st["chain"]:
            ch = self._chain_pack(prec)
            native.chain(0, st["ob"], qpos, ch["A"][0], _wo(l0), l0["ca_wqp"], st["t1n"], rows=rows, Nq=Nq,
                         eps=self.post_norm.eps, R=None, Q=st["qc"])
        else:
            self._self_out_q(st, l0, qpos, None, rows=rows, Nq=Nq, C=C)   # layer 0: zero residual
        st["layer0_done"] = True
        st["stream"] = torch.cuda.current_stream()

    def _self_attn(self, st, *, B, H, Nq, C):
        qkv = st["qkv"]
        sps = 2 if qkv.dtype == SPLIT else 1
        hs = (3 * C * Nq * sps, 32 * sps * Nq, 32 * sps)
        native.attention(qkv, qkv, qkv, st["ob"], B=B, H=H, Nq=Nq, Nk=Nq, q_strides=hs, k_strides=hs, v_strides=hs,
                         k_offset=C * Nq * sps, v_offset=2 * C * Nq * sps, o_strides=(Nq * C, C),
                         scale=1.0 / math.sqrt(32.0), workspace=st["ws"], fold_scale=True)

    def _self_out_q(self, st, lw, qpos, R, *, rows, Nq, C):
        """Separate-launch path: self-attn out_proj (+ residual R; None = zero
        target), norms[0] -> t1n and lowp(t1n + qpos), cross-attention Q."""
        t1, ksp = st["t1"], st["ksp"]
        w0, b0, e0 = lw["norms"][0]
        native.gemm(st["ob"], lw["sa_ow"], t1, M=rows, N=C, K=C, lda=C, ldw=C, ldc=C, bias=lw["sa_ob"], R=R,
                    ldr=C if R is not None else 0, k_splits=ksp)
        native.layernorm_ex(t1, w0, b0, rows=rows, C=C, ldx=C, eps=e0, Y=st["t1n"], ldy=C, Yp=st["tp"], P=qpos,
                            nparts=ksp)
        native.gemm(st["tp"], lw["ca_wq"], st["qc"], M=rows, N=C, K=C, lda=C, ldw=C, ldc=0, bias=lw["ca_bq"],
                    headsplit_rows=Nq)

    def _project_kv(self, pk, memb, mposb, *, B, Nk, prec):
        """Cross-attention K / V of every layer from lowp(mem) / lowp(mem + pos)
        in one launch, into [B][K_0..K_L-1 | V_0..V_L-1][H][Nk][32].  Returns
        (kv, one dict per layer: k / v element offsets and the key-norm maxima).

        (One launch per layer on a second stream, each joined by an event
        before its layer's cross-attention, was measured: the later layers'
        launches took the whole chip ahead of layer 0's cross-attention instead
        of filling the latency-bound query-side gaps, and a per-layer launch
        re-stages the token tile for 2 of the 12 projections -- 68-71 us each
        against 288 / 6; profiles/r3s_kv_per_layer.txt.)"""
        L, C, H = self.num_layers, self.embed_dims, self.embed_dims // 32
        dev = memb.device
        kv = torch.empty((B * 2 * L * C * Nk,), dtype=prec.attn, device=dev)
        # f16 / bf16 K: the per-64-row max |k|^2 (epilogue by-product) bounds every score,
        # so the cross-attention kernel needs no running max (cmt_hip.h kmax2)
        kmax2 = None
        if prec.attn in (torch.bfloat16, torch.float16):
            kmax2 = torch.empty((-(-B * Nk // native.PLANE_MAX_ROWS), L * H), dtype=torch.float32, device=dev)
        if pk["kv_wp"] is not None and memb.dtype == pk["kv_wp"].dtype:
            native.kv_proj(memb, pk["kv_wp"], kv, M=B * Nk, N=2 * L * C, bias=pk["kv_b"], A2=mposb,
                           headsplit_rows=Nk, plane_max2=kmax2, plane_max_cols=L * C)
        else:
            native.gemm(memb, pk["kv_w"], kv, M=B * Nk, N=2 * L * C, K=C, lda=C, ldw=C, ldc=0, bias=pk["kv_b"],
                        A2=mposb, lda2=C, a2_cols=L * C, headsplit_rows=Nk, plane_max2=kmax2, plane_max_cols=L * C)
        return kv, [dict(k=l * C * Nk, v=(L + l) * C * Nk, kmax=kmax2, ld=L * H, p0=l * H) for l in range(L)]

    def _cross_attn(self, qc, kv, ent, ob, *, B, Nq, Nk, ws, prec, keep=False):
        """Cross-attention core of one layer.  keep: a split launch may leave its
        partials in ``ws`` for chain B1 (ABI 19) -- returns their count, 0 when
        ``ob`` was written."""
        L, C, H = self.num_layers, self.embed_dims, self.embed_dims // 32
        with timed("cross_attn"):
            return native.attention(qc, kv, kv, ob, B=B, H=H, Nq=Nq, Nk=Nk,
                                    q_strides=(C * Nq, 32 * Nq, 32), k_strides=(2 * L * C * Nk, 32 * Nk, 32),
                                    v_strides=(2 * L * C * Nk, 32 * Nk, 32), k_offset=ent["k"], v_offset=ent["v"],
                                    o_strides=(Nq * C, C), scale=1.0 / math.sqrt(32.0), workspace=ws,
                                    round_output=prec.round_cross_out, fold_scale=prec.fold_q, kmax2=ent["kmax"],
                                    kmax_ld=ent["ld"], kmax_plane0=ent["p0"], keep_partials=keep)

    def _run_rows_lowp(self, mem, pos, qpos, *, B, Nk, Nq, out, post_flags, prec, tgt0, kv_operands, out16=None,
                       state=None):
        """run_rows under an f16/bf16/split policy: every GEMM operand is
        produced in the compute format by the kernel before it (LayerNorm
        writes lowp(y) and lowp(y + query_pos) beside the fp32 residual stream,
        attention writes its output in it, FFN fc1 writes its activation in
        it), so every GEMM stages A and W by LDS-DMA.  The residual stream, the
        LayerNorm statistics and the decoder outputs stay fp32.  ``state``
        (zero target, tgt0 None): buffers from lowp_state whose layer 0 up to
        the cross-attention core may already be queued (lowp_layer0)."""
        pk = self.packed(prec)
        L, C, H = self.num_layers, self.embed_dims, self.embed_dims // 32
        lp = prec.gemm
        dev = qpos.device
        f32 = torch.float32
        rows = B * Nq
        if out is None:
            out = torch.empty((L, rows, C), dtype=f32, device=dev)
        if kv_operands is None:
            memb = op_empty(B * Nk, C, lp, dev)
            mposb = torch.empty_like(memb)
            native.add_cast(mem, rows=B * Nk, C=C, Yl=memb, Yp=mposb, P=pos)
        else:
            memb, mposb = kv_operands
        # K columns read lowp(mem + pos), V columns lowp(mem)
        kv, kvl = self._project_kv(pk, memb, mposb, B=B, Nk=Nk, prec=prec)
        use_chain = self._use_chain(prec)
        if tgt0 is None:
            # target = zeros_like(query_embed) in every CMT transformer (cmt_transformer.py:114):
            # layer 0's residual is None and its first operands come from add_cast's zeros
            st = state if state is not None else self.lowp_state(B=B, Nk=Nk, Nq=Nq, prec=prec, device=dev)
            if not st["layer0_done"]:
                self.lowp_layer0(st, qpos, B=B, Nq=Nq, prec=prec)
            elif st["stream"] is not None and st["stream"] != torch.cuda.current_stream():
                torch.cuda.current_stream().wait_stream(st["stream"])   # join the layer-0 side stream
            if use_chain:
                return self._chain_layers(st, qpos, kv, kvl, B=B, Nk=Nk, Nq=Nq, out=out, post_flags=post_flags,
                                          prec=prec, out16=out16)
            return self._sep_layers(st, qpos, kv, kvl, B=B, Nk=Nk, Nq=Nq, out=out, post_flags=post_flags,
                                    prec=prec, out16=out16, l0_done=True)
        if state is not None:
            raise ValueError("run_rows: a lowp_state applies to a zero target only")
        st = self.lowp_state(B=B, Nk=Nk, Nq=Nq, prec=prec, device=dev)
        tgt = st["tgt"]
        tgt.copy_(tgt0)
        native.add_cast(tgt, rows=rows, C=C, Yl=st["tl"], Yp=st["tp"], P=qpos)
        if use_chain:
            # per layer: self-attn core, chain A (out_proj + norms[0] + cross Q proj),
            # cross-attn core, chain B1 (out_proj + norms[1] + FFN quarter -> fp32 partials),
            # chain B2 (partials -> norms[2] + post_norm + next layer's in_proj) -- see rowchain.hip
            ch = self._chain_pack(prec)
            eps = self.post_norm.eps
            l0 = pk["layers"][0]
            native.gemm(st["tl"], l0["sa_w"], st["qkv"], M=rows, N=3 * C, K=C, lda=C, ldw=C, ldc=0,
                        bias=l0["sa_b"], A2=st["tp"], lda2=C, a2_cols=2 * C, headsplit_rows=Nq)
            for l, lw in enumerate(pk["layers"]):
                self._self_attn(st, B=B, H=H, Nq=Nq, C=C)
                native.chain(0, st["ob"], qpos, ch["A"][l], lw["sa_ow"], lw["ca_wqp"], st["t1n"], rows=rows, Nq=Nq,
                             eps=eps, R=tgt, Q=st["qc"])
                xs = self._cross_attn(st["qc"], kv, kvl[l], st["ob"], B=B, Nq=Nq, Nk=Nk, ws=st["ws"], prec=prec,
                                      keep=self._keep_partials(prec))
                nxt = pk["layers"][l + 1]["sa_wp"] if l + 1 < L else None
                native.chain(1, st["ob"], None, ch["B"][l], *_b1w(lw), tgt, rows=rows, Nq=Nq, eps=eps,
                             R=st["t1n"], W2=lw["f2_wp"], WS=st["cws"], **self._xpart(st["ws"], xs, prec))
                native.chain(2, None, qpos if nxt is not None else None, ch["B"][l], None, None, tgt, rows=rows,
                             Nq=Nq, eps=eps, Wn=nxt, OUT=out, out_offset=l * rows * C, out_flags=post_flags,
                             Q=st["qkv"] if nxt is not None else None, WS=st["cws"], OUT16=out16)
            return out
        return self._sep_layers(st, qpos, kv, kvl, B=B, Nk=Nk, Nq=Nq, out=out, post_flags=post_flags, prec=prec,
                                out16=out16, l0_done=False)

    def _sep_layers(self, st, qpos, kv, kvl, *, B, Nk, Nq, out, post_flags, prec, out16, l0_done):
        """Separate-launch decoder layers (the split policy, or CMT_CHAIN=0).
        ``l0_done``: layer 0 up to its cross-attention core already queued
        (lowp_layer0, zero target)."""
        pk = self.packed(prec)
        L, C, H = self.num_layers, self.embed_dims, self.embed_dims // 32
        rows = B * Nq
        lp = prec.gemm
        tgt, tl, tp, qkv, ob, t1n, hf, t1, o, ws, ksp = (st[k] for k in ("tgt", "tl", "tp", "qkv", "ob", "t1n", "hf",
                                                                         "t1", "o", "ws", "ksp"))
        FF = hf.shape[-1]
        pw, pb, _pe = pk["post"]
        for l, lw in enumerate(pk["layers"]):
            if l > 0 or not l0_done:
                # --- self attention: Q|K columns read lowp(tgt + qpos), V columns lowp(tgt)
                native.gemm(tl, lw["sa_w"], qkv, M=rows, N=3 * C, K=C, lda=C, ldw=C, ldc=0, bias=lw["sa_b"],
                            A2=tp, lda2=C, a2_cols=2 * C, headsplit_rows=Nq)
                self._self_attn(st, B=B, H=H, Nq=Nq, C=C)
                self._self_out_q(st, lw, qpos, tgt, rows=rows, Nq=Nq, C=C)
            # --- cross attention: q = lowp(x + qpos); K/V from _project_kv
            self._cross_attn(st["qc"], kv, kvl[l], ob, B=B, Nq=Nq, Nk=Nk, ws=ws, prec=prec)
            w1, b1, e1 = lw["norms"][1]
            native.gemm(ob, lw["ca_ow"], t1, M=rows, N=C, K=C, lda=C, ldw=C, ldc=C, bias=lw["ca_ob"], R=t1n,
                        ldr=C, k_splits=ksp)
            native.layernorm_ex(t1, w1, b1, rows=rows, C=C, ldx=C, eps=e1, Y=o, ldy=C, Yl=tl, nparts=ksp)
            # --- FFN (fc1 activation written in the compute dtype)
            native.gemm(tl, lw["f1_w"], hf, M=rows, N=FF, K=C, lda=C, ldw=C, ldc=FF, bias=lw["f1_b"], relu=True)
            # --- fc2 + residual + norms.2 -> next query (fp32 + both lowp operands), + post_norm -> out[l]
            w2, b2, e2 = lw["norms"][2]
            native.gemm(hf, lw["f2_w"], t1, M=rows, N=C, K=FF, lda=FF, ldw=FF, ldc=C, bias=lw["f2_b"], R=o,
                        ldr=C, k_splits=ksp)
            native.layernorm_ex(t1, w2, b2, rows=rows, C=C, ldx=C, eps=e2, Y=tgt, ldy=C, Yl=tl, Yp=tp, P=qpos,
                                W2=pw, B2=pb, Y2=out, ldy2=C, flags2=post_flags, y2_offset=l * rows * C,
                                nparts=ksp)
        if out16 is not None:
            if lp == SPLIT:
                native.split_rows(out.view(-1, C), out16.view(-1, 2, C))
            else:
                native.cast(out, out16)
        return out

    @staticmethod
    def _keep_partials(prec):
        """Split chains ('ref'): chain B1 combines the cross-attention's split partials itself
        (ABI 19) -- one launch and one pair-row round trip fewer per layer."""
        return prec.gemm == SPLIT and OPTIONS.chain_combine

    @staticmethod
    def _xpart(ws, kept, prec):
        if not kept:
            return {}
        return dict(xpart=ws.view(torch.float32), xsplits=kept, xround=prec.round_cross_out)

    def _chain_layers(self, st, qpos, kv, kvl, *, B, Nk, Nq, out, post_flags, prec, out16):
        """Chain path from layer 0's cross-attention core on (layer 0's self
        block already queued by lowp_layer0): per layer the cross-attention
        core, chain B1, chain B2 (which also runs the next layer's in_proj),
        then the next layer's self-attention core and chain A."""
        pk = self.packed(prec)
        ch = self._chain_pack(prec)
        L, C, H = self.num_layers, self.embed_dims, self.embed_dims // 32
        rows = B * Nq
        eps = self.post_norm.eps
        tgt, qkv, qc, ob, t1n, ws, cws = (st[k] for k in ("tgt", "qkv", "qc", "ob", "t1n", "ws", "cws"))
        for l, lw in enumerate(pk["layers"]):
            if l > 0:
                self._self_attn(st, B=B, H=H, Nq=Nq, C=C)
                native.chain(0, ob, qpos, ch["A"][l], _wo(lw), lw["ca_wqp"], t1n, rows=rows, Nq=Nq, eps=eps,
                             R=tgt, Q=qc)
            xs = self._cross_attn(qc, kv, kvl[l], ob, B=B, Nq=Nq, Nk=Nk, ws=ws, prec=prec,
                                  keep=self._keep_partials(prec))
            nxt = pk["layers"][l + 1]["sa_wp"] if l + 1 < L else None
            native.chain(1, ob, None, ch["B"][l], *_b1w(lw), tgt, rows=rows, Nq=Nq, eps=eps,
                         R=t1n, W2=lw["f2_wp"], WS=cws, **self._xpart(ws, xs, prec))
            native.chain(2, None, qpos if nxt is not None else None, ch["B"][l], None, None, tgt, rows=rows,
                         Nq=Nq, eps=eps, Wn=nxt, OUT=out, out_offset=l * rows * C, out_flags=post_flags,
                         Q=qkv if nxt is not None else None, WS=cws, OUT16=out16)
        return out
