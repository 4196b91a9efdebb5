"""CmtTransformer / CmtLidarTransformer / CmtImageTransformer with the
reference's registry names and forward signatures, on the fused native
decoder.

Reference: projects/mmdet3d_plugin/models/utils/cmt_transformer.py
  CmtTransformer 48-127, CmtLidarTransformer 130-204, CmtImageTransformer 207-282.
Memory = cat(BEV tokens "(h w)", image tokens "(v h w)") and pos likewise
(:104-112), target = 0 (:114), output [L, B, Nq, C] (:125).  In training (or
with the DN attention mask of prepare_for_dn in attn_masks[0]) the decoder runs
on the differentiable native ops (PETRTransformerDecoder.train_rows).  Here memory
and pos are assembled directly in batch-major row layout by the layout kernel
(no rearrange/cat copies of the reference), and the decoder hoists every
layer's K/V projection into one GEMM (PETRTransformerDecoder.run_rows).
"""
import torch
import torch.nn as nn

from ... import native
from ...registry import TRANSFORMER, TRANSFORMER_LAYER_SEQUENCE, build_from_cfg

__all__ = ["CmtTransformer", "CmtLidarTransformer", "CmtImageTransformer"]


class _CmtTransformerBase(nn.Module):
    def __init__(self, encoder=None, decoder=None, init_cfg=None, cross=False):
        super().__init__()
        if encoder is not None:
            raise NotImplementedError("CMT configs use no transformer encoder")
        self.encoder = None
        self.decoder = build_from_cfg(decoder, TRANSFORMER_LAYER_SEQUENCE)
        self.embed_dims = self.decoder.embed_dims
        self.cross = cross

    def init_weights(self):
        """DETR init (cmt_transformer.py:77-82): xavier-uniform every module
        weight with dim > 1 (mmcv xavier_init also zeroes that module's bias)."""
        for m in self.modules():
            if hasattr(m, "weight") and isinstance(m.weight, torch.Tensor) and m.weight.dim() > 1:
                nn.init.xavier_uniform_(m.weight)
                if getattr(m, "bias", None) is not None:
                    nn.init.zeros_(m.bias)
        self._is_init = True

    def _train_mode(self, attn_masks):
        masked = attn_masks is not None and any(m is not None for m in attn_masks)
        return masked or (self.training and torch.is_grad_enabled())

    def _run_train(self, mem, pos, query_embed, attn_masks):
        """Training / DN-masked forward (cmt_transformer.py:84-127 with
        attn_masks=[dn_mask, None]): memory / pos rows [B, Nk, C] built
        differentiably, target = 0, the decoder on the native training ops."""
        from .petr_transformer import dn_mask_params
        m0 = attn_masks[0] if attn_masks is not None else None
        pad, grp = dn_mask_params(m0) if m0 is not None else (0, 0)
        qpos = query_embed.float()
        dec = self.decoder
        # train_cross_fp16 (default True): flash-attn's fp16 cross core, as the reference trains
        out = dec.train_rows(torch.zeros_like(qpos), qpos, mem, pos, pad=pad, group=grp,
                             dropout=self.training, cross_fp16=getattr(self, "train_cross_fp16", True))
        if not dec.return_intermediate:
            out = out[-1:]
        return out, mem.transpose(0, 1)

    def _run(self, B, Nk, Nq, fill_mem, fill_pos, query_embed):
        C = self.embed_dims
        dev = query_embed.device
        mem = torch.empty((B * Nk, C), dtype=torch.float32, device=dev)
        pos = torch.empty((B * Nk, C), dtype=torch.float32, device=dev)
        fill_mem(mem)
        fill_pos(pos)
        qpos = query_embed.reshape(B * Nq, C).contiguous().float()
        out = self.decoder.run_rows(mem, pos, qpos, B=B, Nk=Nk, Nq=Nq, post_flags=0)
        L = out.shape[0]
        out_dec = out.view(L, B, Nq, C)
        if not self.decoder.return_intermediate:
            out_dec = out_dec[-1:]
        return out_dec, mem.view(B, Nk, C).transpose(0, 1)


@TRANSFORMER.register_module()
class CmtTransformer(_CmtTransformerBase):
    def forward(self, x, x_img, query_embed, bev_pos_embed, rv_pos_embed, attn_masks=None, reg_branch=None):
        """x [bs, C, h, w]; x_img [bs*v, C, h', w']; query_embed [bs, Nq, C];
        bev_pos_embed [h*w, C]; rv_pos_embed [bs*v, h', w', C] ->
        (out_dec [L, bs, Nq, C], memory [Nk, bs, C])."""
        bs, C, h, w = x.shape
        BV, _, hi, wi = x_img.shape
        v = BV // bs
        HW, hwi = h * w, hi * wi
        Nk = HW + v * hwi
        Nq = query_embed.shape[1]
        if self._train_mode(attn_masks):
            from .train_ops import nchw_rows
            mem = torch.cat([nchw_rows(x, bs).view(bs, HW, C), nchw_rows(x_img, bs).view(bs, v * hwi, C)], 1)
            pos = torch.cat([bev_pos_embed.float().unsqueeze(0).expand(bs, HW, C),
                             rv_pos_embed.reshape(bs, v * hwi, C).float()], 1)
            return self._run_train(mem, pos, query_embed, attn_masks)

        def fill_mem(mem):
            native.nchw_to_rows(x.contiguous().float(), mem, nb=bs, nv=1, C=C, HW=HW, ldy=C, rows_per_batch=Nk)
            native.nchw_to_rows(x_img.contiguous().float(), mem, nb=bs, nv=v, C=C, HW=hwi, ldy=C,
                                rows_per_batch=Nk, row_offset=HW)

        def fill_pos(pos):
            p = pos.view(bs, Nk, C)
            p[:, :HW] = bev_pos_embed.float()
            p[:, HW:] = rv_pos_embed.reshape(bs, v * hwi, C).float()

        return self._run(bs, Nk, Nq, fill_mem, fill_pos, query_embed)


@TRANSFORMER.register_module()
class CmtLidarTransformer(_CmtTransformerBase):
    def forward(self, x, mask, query_embed, pos_embed, attn_masks=None, reg_branch=None):
        """x [bs, C, h, w]; mask [bs, h, w] (all zero in CMT); pos_embed [h*w, C]."""
        bs, C, h, w = x.shape
        Nk = h * w
        Nq = query_embed.shape[1]
        if self._train_mode(attn_masks):
            from .train_ops import nchw_rows
            mem = nchw_rows(x, bs).view(bs, Nk, C)
            return self._run_train(mem, pos_embed.float().unsqueeze(0).expand(bs, Nk, C), query_embed, attn_masks)

        def fill_mem(mem):
            native.nchw_to_rows(x.contiguous().float(), mem, nb=bs, nv=1, C=C, HW=Nk, ldy=C, rows_per_batch=Nk)

        def fill_pos(pos):
            pos.view(bs, Nk, C)[:] = pos_embed.float()

        return self._run(bs, Nk, Nq, fill_mem, fill_pos, query_embed)


@TRANSFORMER.register_module()
class CmtImageTransformer(_CmtTransformerBase):
    def forward(self, x_img, query_embed, rv_pos_embed, attn_masks=None, reg_branch=None, bs=2):
        """x_img [bs*v, C, h, w]; rv_pos_embed [bs*v, h, w, C]."""
        BV, C, h, w = x_img.shape
        v = BV // bs
        Nk = v * h * w
        Nq = query_embed.shape[1]
        if self._train_mode(attn_masks):
            from .train_ops import nchw_rows
            mem = nchw_rows(x_img, bs).view(bs, Nk, C)
            return self._run_train(mem, rv_pos_embed.reshape(bs, Nk, C).float(), query_embed, attn_masks)

        def fill_mem(mem):
            native.nchw_to_rows(x_img.contiguous().float(), mem, nb=bs, nv=v, C=C, HW=h * w, ldy=C,
                                rows_per_batch=Nk)

        def fill_pos(pos):
            pos.view(bs, Nk, C)[:] = rv_pos_embed.reshape(bs, Nk, C).float()

        return self._run(bs, Nk, Nq, fill_mem, fill_pos, query_embed)
