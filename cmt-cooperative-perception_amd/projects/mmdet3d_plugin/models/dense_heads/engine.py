"""Native execution of one CMT head forward (per agent and for the task heads).

This is the hot path of SURVEY.md section 8(a), rows a1-a16, executed as a
fixed sequence of gfx950 kernels over HBM-resident buffers:

  shared_conv     NCHW->NHWC layout kernel + implicit-GEMM 3x3 conv (BN folded, ReLU)
                  written straight into the memory rows (cmt_head.py:280-287, 481)
  bev pos         pos2embed(coords_bev) fused kernel -> 2 GEMMs (bias/ReLU fused)
                  written straight into the pos rows (cmt_head.py:324-337, 489)
  image memory    layout kernel "(bs v) c h w -> bs (v h w) c" into the memory rows
  rv pos          frustum geometry kernel (fp64 host inverse) -> 2 GEMMs into pos rows
                  (cmt_head.py:417-433)
  query embed     pos2embed(sigmoid(inverse_sigmoid(ref))) -> 2 GEMMs, plus the
                  projected-view geometry kernel -> 2 GEMMs -> masked view sum
                  (cmt_head.py:435-473)
  decoder         PETRTransformerDecoder.run_rows (K/V of all layers in one GEMM,
                  per layer 7 GEMMs + 2 attention + 3 LayerNorm launches)
  coop max        fused into the post_norm kernel (cmt_head_coop.py:383-389)
  task heads      grouped Conv1d as one batched (implicit conv1d) GEMM over the
                  decoder layers, then GroupLayerNorm1d+ReLU, conv #2 and the
                  box epilogue (cmt_head.py:136-203, 501-513)

The reference computes the BEV positional encoding, the coordinate encodings
and every layer's K/V projection again on each forward; so does this engine
(no output caching across frames).
"""

import numpy as np
import torch

from ... import native
from ...runtime import OPTIONS, SPLIT, get_precision, op_empty
from ..utils.packing import to_dtype

__all__ = ["HeadEngineMixin"]


def _inv_lidar2img(metas):
    """np.linalg.inv of every lidar2img in fp64 (cmt_head.py:428, 441-444)."""
    l2i = np.stack([np.asarray(m["lidar2img"], dtype=np.float64) for m in metas])   # [B, V, 4, 4]
    i2l = np.linalg.inv(l2i)
    return l2i, i2l


class HeadEngineMixin:
    """Mixed into CmtHead / CmtHeadCoop and their LiDAR / image variants."""

    # ------------------------------------------------------------------ packing
    def _engine_pack(self, prec):
        params = [p for p in self.parameters()] + [b for b in self.buffers()]

        def build():
            g = prec.gemm
            pk = {}
            if getattr(self, "shared_conv", None) is not None:
                conv, bn = self.shared_conv.conv, self.shared_conv.bn
                s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
                w = conv.weight * s[:, None, None, None]                   # [Cout, Cin, 3, 3]
                pk["conv_w"] = to_dtype(w.permute(0, 2, 3, 1).reshape(w.shape[0], -1), g)   # [Cout, 9*Cin]
                b = bn.bias - bn.running_mean * s
                if conv.bias is not None:
                    b = b + conv.bias * s
                pk["conv_b"] = b.detach().float().contiguous()
            be = self.bev_embedding
            pk["bev"] = (to_dtype(be[0].weight, g), be[0].bias.detach().contiguous(),
                         to_dtype(be[2].weight, g), be[2].bias.detach().contiguous())
            if getattr(self, "rv_embedding", None) is not None:
                re = self.rv_embedding
                pk["rv"] = (to_dtype(re[0].weight, g), re[0].bias.detach().contiguous(),
                            to_dtype(re[2].weight, g), re[2].bias.detach().contiguous())
                w0, _, w2, _ = pk["rv"]
                if (g == SPLIT and w2.shape[0] == 256 and w0.shape[0] % 32 == 0 and w0.shape[-1] % 16 == 0
                        and w0.shape[-1] <= 192):
                    # fragment packs of the one-launch MLP (cmt_mlp2_x3)
                    pk["rv_fused"] = native.mlp2_pack(w0, w2)
            return pk
        return self._pack.get("engine", params, prec.name, build)

    # ------------------------------------------------------------------ pieces
    def _mlp(self, x, w, out=None, *, batch=1, a_bstride=0, c_bstride=0, c_offset=0, M=None, R=None, r_offset=0):
        """Linear-ReLU-Linear with the second GEMM optionally scattering rows
        into a larger buffer (batched) and adding a residual R laid out like
        ``out``.  The hidden activation is kept in x's dtype when that is the
        compute dtype (LDS-DMA operand for the second GEMM)."""
        w0, b0, w2, b2 = w
        hdt = x.dtype if x.dtype == w0.dtype else torch.float32
        h = native.linear(x, w0, b0, relu=True, out_dtype=hdt)
        if out is None:
            return native.linear(h, w2, b2)
        M = M if M is not None else h.shape[0]
        native.gemm(h, w2, out, M=M, N=w2.shape[0], K=w2.shape[-1], lda=h.shape[-1], ldw=w2.shape[-1],
                    ldc=out.shape[-1], bias=b2, batch=batch, a_bstride=a_bstride * h.shape[-1] if batch > 1 else 0,
                    c_bstride=c_bstride, c_offset=c_offset, R=R, ldr=out.shape[-1] if R is not None else 0,
                    r_bstride=c_bstride if R is not None else 0, r_offset=r_offset)
        return out

    def _conv_halo_ok(self, x, pk, prec):
        _, Cin, _, W = x.shape
        # 'ref': three f16 passes on split pixels / weights; f16 / bf16 policies: one pass (round 6)
        return (prec.gemm in (SPLIT, torch.float16, torch.bfloat16) and OPTIONS.conv_halo and Cin % 16 == 0
                and W <= 180 and pk["conv_w"].shape[0] % 128 == 0 and pk["conv_w"].dtype == prec.gemm)

    def _range_flag(self, dev):
        """The head's f16-operand range flag: an int32 device word the kernels that read the
        external feature maps (the NCHW shared_conv's epilogue, the camera-row layout pass) set
        when a value falls outside the f16 / f16-pair operand format (cmt_hip.h ABI 18).  Made on
        the first (eager) forward, so a captured graph writes the same word on every replay."""
        f = self.__dict__.get("_range_flag_t")
        if f is None or f.device != dev:
            f = torch.zeros(1, dtype=torch.int32, device=dev)
            self.__dict__["_range_flag_t"] = f
        return f

    def check_input_range(self):
        """Raise ValueError if a forward since the last call -- eager or a replayed HIP
        graph, where the host-side check_f16_range cannot run -- met a feature-map value
        the f16-operand policies cannot carry (non-finite or |x| >= 65520), and clear the
        flag.  One 4-byte device read (it waits for the work queued before it); call it
        after consuming a replay's outputs."""
        f = self.__dict__.get("_range_flag_t")
        if f is None:
            return
        if int(f.item()):
            f.zero_()
            raise ValueError("an input feature map held a value outside the f16 operand range (non-finite or "
                             "|x| >= 65520) of the current precision policy; the outputs of that forward are "
                             "not valid -- use set_precision('exact') for such inputs")

    def _shared_conv_into(self, x, mem, Nk, pk, prec, pos=None, P=None):
        """shared_conv into the memory rows; with ``P`` (the weight-only BEV
        position rows, fp32 [H*W, C]) the NCHW conv also writes lowp(memory + pos)
        into ``pos`` -- the BEV position MLP's second GEMM is then not run."""
        B, Cin, H, W = x.shape
        Cout = pk["conv_w"].shape[0]
        if self._conv_halo_ok(x, pk, prec):
            # reference numerics: the conv reads the NCHW fp32 map itself, splitting each input
            # pixel into f16 hi / lo once per workgroup for all nine taps (cmt_hip.h
            # CMT_A_CONV3X3_NCHW) -- no NCHW -> pair-rows pass
            native.gemm(x.contiguous().float(), pk["conv_w"], mem, M=H * W, N=Cout, K=9 * Cin, lda=H * W,
                        ldw=9 * Cin, ldc=Cout, bias=pk["conv_b"], relu=True, a_mode=native.A_CONV3X3_NCHW,
                        conv=(H, W, Cin), batch=B, a_bstride=Cin * H * W, c_bstride=Nk * Cout,
                        A2=P, lda2=Cout if P is not None else 0, c2=pos if P is not None else None,
                        range_flag=self._range_flag(x.device) if prec.gemm != torch.bfloat16 else None)
            return
        assert P is None
        xin = op_empty(B * H * W, Cin, prec.gemm, x.device)
        native.nchw_to_rows(x.contiguous().float(), xin, nb=B, nv=1, C=Cin, HW=H * W, ldy=Cin, rows_per_batch=H * W,
                            range_flag=self._range_flag(x.device))
        native.gemm(xin, pk["conv_w"], mem, M=H * W, N=Cout, K=9 * Cin, lda=Cin, ldw=9 * Cin, ldc=Cout,
                    bias=pk["conv_b"], relu=True, a_mode=native.A_CONV3X3, conv=(H, W, Cin), batch=B,
                    a_bstride=H * W * Cin, c_bstride=Nk * Cout)

    def _h2d(self, arr, dev, tag):
        """Host camera matrices (fp64 inverse on the host, as the reference) ->
        fp32 device tensor.  Every eager call also sets up a pinned staging
        buffer per (tag, shape, upload index in the forward); under HIP-graph capture the values go through
        that buffer, so the graph holds a host->device copy node that re-reads
        it on each replay (pinned allocation itself is not capturable, hence
        the eager warm-up torch's graph capture needs anyway)."""
        t = torch.from_numpy(np.ascontiguousarray(arr)).float()
        pool = self.__dict__.setdefault("_pinned_meta", {})
        seq = self.__dict__.get("_h2d_seq", 0)
        self._h2d_seq = seq + 1
        key = (tag, tuple(t.shape), seq)
        if torch.cuda.is_current_stream_capturing():
            if key not in pool:
                raise RuntimeError("camera metas of this shape were never seen eagerly: run one eager forward "
                                   "before capturing the head in a HIP graph")
            pool[key].copy_(t)
            d = torch.empty(t.shape, dtype=t.dtype, device=dev)
            d.copy_(pool[key], non_blocking=True)
            return d
        if key not in pool and dev.type == "cuda":
            pool[key] = torch.empty(t.shape, dtype=t.dtype).pin_memory()
        return t.to(dev)

    def _bev_pos_hidden(self, H, W, pk):
        """First half of bev_pos_embed (cmt_head.py:324-337, 489): pos2embed of
        the BEV grid and bev_embedding[0] + ReLU -- input-independent."""
        C = self.hidden_dim
        cfg = self.train_cfg if self.train_cfg else self.test_cfg
        x_size = cfg["grid_size"][1] // self.downsample_scale
        y_size = cfg["grid_size"][0] // self.downsample_scale
        if x_size * y_size != H * W:
            raise ValueError(f"BEV map {H}x{W} does not match grid_size/downsample ({x_size}x{y_size})")
        w0, b0, _, _ = pk["bev"]

        def build():
            pe = op_empty(H * W, 2 * C, w0.dtype, w0.device)
            native.pos2embed(None, pe, n=H * W, F=C, grid=(x_size, y_size))
            hdt = pe.dtype if pe.dtype == w0.dtype else torch.float32
            return native.linear(pe, w0, b0, relu=True, out_dtype=hdt)
        # A function of the weights and the grid only: kept like a weight pack (rebuilt when
        # bev_embedding[0] changes, Tensor._version / storage tracked) unless CMT_BEV_POS_CACHE=0.
        # Never built inside a graph capture (its buffer must outlive the graph).
        if not OPTIONS.bev_pos_cache:
            return build()
        key = (H, W, x_size, y_size, str(w0.dtype))
        name = f"bev_hidden_{H}x{W}_{w0.dtype}"
        src = [self.bev_embedding[0].weight, self.bev_embedding[0].bias]   # the parameters themselves
        if torch.cuda.is_current_stream_capturing() and not self._pack.has(name, src, key):
            return build()
        return self._pack.get(name, src, key, build)

    def _bev_pos_rows(self, H, W, pk):
        """The whole BEV position encoding bev_embedding(pos2embed(coords_bev))
        (cmt_head.py:324-337, 489) as fp32 rows [H*W, C]: like the hidden rows, a
        function of the weights and the grid only, kept like a weight pack
        (bev_embedding tracked); the NCHW conv adds it to the memory rows in its
        epilogue (``_shared_conv_into(P=...)``)."""
        _, _, w2, b2 = pk["bev"]
        C = self.hidden_dim

        def build():
            hid = self._bev_pos_hidden(H, W, pk)
            rows = torch.empty((H * W, C), dtype=torch.float32, device=w2.device)
            native.gemm(hid, w2, rows, M=H * W, N=C, K=w2.shape[-1], lda=hid.shape[-1], ldw=w2.shape[-1], ldc=C,
                        bias=b2)
            return rows
        key = (H, W, str(w2.dtype))
        name = f"bev_pos_rows_{H}x{W}_{w2.dtype}"
        be = self.bev_embedding
        src = [be[0].weight, be[0].bias, be[2].weight, be[2].bias]
        if torch.cuda.is_current_stream_capturing() and not self._pack.has(name, src, key):
            return build()
        return self._pack.get(name, src, key, build)

    def _bev_pos_out(self, hid, pos, B, Nk, pk, R=None):
        """Second half: bev_embedding[2] into the pos rows of every batch
        element; with R (the memory rows in the compute dtype) the output is
        lowp(memory + pos) -- the K-projection operand."""
        _, _, w2, b2 = pk["bev"]
        C, M = self.hidden_dim, hid.shape[0]
        native.gemm(hid, w2, pos, M=M, N=w2.shape[0], K=w2.shape[-1], lda=hid.shape[-1], ldw=w2.shape[-1], ldc=C,
                    bias=b2, batch=B, a_bstride=0, c_bstride=Nk * C, R=R, ldr=C if R is not None else 0,
                    r_bstride=Nk * C if R is not None else 0)

    def _bev_pos_into(self, pos, B, Nk, H, W, pk, R=None):
        """bev_pos_embed (cmt_head.py:324-337, 489) into the pos rows (both halves)."""
        self._bev_pos_out(self._bev_pos_hidden(H, W, pk), pos, B, Nk, pk, R=R)

    def _cams(self, metas, dev):
        """(lidar2img, inv(lidar2img)) of every camera as [B, V, 4, 4] fp32 device
        views of ONE upload (fp64 host inverse, cmt_head.py:428, 441-444)."""
        l2i, i2l = _inv_lidar2img(metas)
        both = self._h2d(np.stack([l2i, i2l]), dev, "cams")
        return both[0], both[1]

    def _rv_fused(self, pk):
        """The fragment packs of the one-launch rv_embedding (cmt_mlp2_x3) when
        that path applies (split policy, CMT_MLP_FUSED), else None."""
        return pk.get("rv_fused") if OPTIONS.mlp_fused else None

    def _rv_pe_hidden(self, x_img, metas, B, pk, cams=None):
        """First half of _rv_pe + rv_embedding (cmt_head.py:417-433, 297-301):
        the frustum coordinates and rv_embedding[0] + ReLU -- they read only
        the camera matrices and the feature-map shape.  With the one-launch MLP
        (_rv_fused) this returns the coordinates and _rv_pe_out runs both layers."""
        BV, _, h, w = x_img.shape
        pad_h, pad_w, _ = metas[0]["pad_shape"][0]
        dev = x_img.device
        i2l = (cams if cams is not None else self._cams(metas, dev))[1]
        D = self.depth_num
        w0, b0, _, _ = pk["rv"]
        cdt = w0.dtype if (3 * D) % 64 == 0 else torch.float32
        coords = op_empty(BV * h * w, 3 * D, cdt, dev)
        native.rv_pe_coords(i2l, coords, BV=BV, h=h, w=w, D=D, pad_h=float(pad_h), pad_w=float(pad_w),
                            depth_max=float(self.pc_range[3]), pc_range=self.pc_range)
        if self._rv_fused(pk) is not None and cdt == SPLIT:
            return coords                                                    # [BV*h*w, 2, 3D]
        hdt = cdt if cdt == w0.dtype else torch.float32
        return native.linear(coords, w0, b0, relu=True, out_dtype=hdt)       # [BV*h*w, 4C]

    def _rv_pe_out(self, hid, pos, B, Nk, offset, pk, R=None):
        """Second half: rv_embedding[2] into the camera pos rows (+ R as in _bev_pos_out)."""
        C = self.hidden_dim
        _, b0, w2, b2 = pk["rv"]
        M = hid.shape[0] // B   # V * h * w rows per batch element
        fused = self._rv_fused(pk)
        if fused is not None and hid.shape[-1] != w2.shape[-1]:
            # hid holds the coordinates: both layers in one launch, the hidden rows stay on chip
            native.mlp2(hid, fused[0], b0, fused[1], b2, pos, M=M, K=native.width(hid), Hd=w2.shape[-1], R=R,
                        batch=B, a_bstride=M * native.width(hid), c_offset=offset * C, c_bstride=Nk * C,
                        r_offset=offset * C, r_bstride=Nk * C)
            return
        native.gemm(hid, w2, pos, M=M, N=C, K=w2.shape[-1], lda=hid.shape[-1], ldw=w2.shape[-1], ldc=C,
                    bias=b2, batch=B, a_bstride=M * hid.shape[-1], c_bstride=Nk * C, c_offset=offset * C,
                    R=R, ldr=C if R is not None else 0, r_bstride=Nk * C if R is not None else 0,
                    r_offset=offset * C)

    def _rv_geo_ok(self, x_img, pk, prec):
        """The camera memory rows in one launch (cmt_mlp2_x3's fused form, ABI 20): the one-launch
        MLP with the reference's depth_num = 64 (K = 192) at the split policy."""
        return (OPTIONS.rv_geo and self._rv_fused(pk) is not None and prec.gemm == SPLIT
                and 3 * self.depth_num == 192 and x_img.shape[1] == self.hidden_dim)

    def _rv_rows_geo(self, x_img, metas, B, Nk, offset, pk, mem, pos, cams):
        """rv_embedding over the frustum coordinates (cmt_head.py:417-433, 297-301) and the
        camera memory rows "(bs v) c h w -> bs (v h w) c" (cmt_transformer.py:104-105) in ONE
        launch: the coordinates are generated in the MLP's prologue from the inverse camera
        matrices, the image features read as NCHW in its epilogue, where they become the memory
        rows (mem) and the residual of lowp(memory + pos) (pos)."""
        C = self.hidden_dim
        BV, _, h, w = x_img.shape
        pad_h, pad_w, _ = metas[0]["pad_shape"][0]
        _, b0, w2, b2 = pk["rv"]
        fused = self._rv_fused(pk)
        M = BV // B * h * w
        geo = dict(i2l=cams[1], h=h, w=w, D=self.depth_num, pad_h=float(pad_h), pad_w=float(pad_w),
                   depth_max=float(self.pc_range[3]), pc_range=self.pc_range)
        native.mlp2(None, fused[0], b0, fused[1], b2, pos, M=M, K=3 * self.depth_num, Hd=w2.shape[-1], batch=B,
                    c_offset=offset * C, c_bstride=Nk * C, geo=geo, rx=x_img.contiguous().float(), C2=mem,
                    c2_offset=offset * C, c2_bstride=Nk * C, range_flag=self._range_flag(x_img.device))

    def _rv_pe_into(self, pos, x_img, metas, B, Nk, offset, pk, R=None, cams=None):
        self._rv_pe_out(self._rv_pe_hidden(x_img, metas, B, pk, cams=cams), pos, B, Nk, offset, pk, R=R)

    def _query_bev_pos(self, pk):
        """bev_embedding(pos2embed(sigmoid(inverse_sigmoid(reference_points))))
        (cmt_head.py:469-473): [Nq, C] fp32, a function of the weights only --
        kept like a weight pack (reference_points and bev_embedding tracked),
        never built inside a graph capture; CMT_BEV_POS_CACHE=0 recomputes it."""
        C = self.hidden_dim
        ref = self.reference_points.weight.detach().contiguous()
        Nq = ref.shape[0]

        def build():
            pe = op_empty(Nq, 2 * C, pk["bev"][0].dtype, ref.device)
            native.pos2embed(ref, pe, n=Nq, F=C, mode=1, pos_stride=3)
            qb = torch.empty((Nq, C), dtype=torch.float32, device=ref.device)
            self._mlp(pe, pk["bev"], qb, M=Nq)
            return qb
        if not OPTIONS.bev_pos_cache:
            return build()
        be = self.bev_embedding
        src = [self.reference_points.weight, be[0].weight, be[0].bias, be[2].weight, be[2].bias]
        key = str(pk["bev"][0].dtype)
        name = f"query_bev_pos_{key}"
        if torch.cuda.is_current_stream_capturing() and not self._pack.has(name, src, key):
            return build()
        return self._pack.get(name, src, key, build)

    def _query_pos(self, B, metas, with_rv, pk, cams=None, first_ops=None):
        """query_embed (+ _rv_query_embed) -> [B*Nq, C] fp32.  ``first_ops``
        (tl, tp) f16/bf16 [B*Nq, C]: with the RV term the final sum also writes
        the decoder's first operands lowp(0) and lowp(0 + query_pos) (the
        add_cast of layer 0); returns (qpos, written)."""
        C = self.hidden_dim
        ref = self.reference_points.weight.detach().contiguous()
        Nq = ref.shape[0]
        dev = ref.device
        qb = self._query_bev_pos(pk)
        if not with_rv:
            return qb.repeat(B, 1), False
        qpos = torch.empty((B * Nq, C), dtype=torch.float32, device=dev)
        V = len(metas[0]["lidar2img"])
        pad_h, pad_w, _ = metas[0]["pad_shape"][0]
        l2i, i2l = cams if cams is not None else self._cams(metas, dev)
        refB = ref.unsqueeze(0).expand(B, Nq, 3).contiguous()
        D = self.depth_num
        mask = torch.empty((B * V * Nq,), dtype=torch.float32, device=dev)
        w0 = pk["rv"][0]
        if w0.dtype != torch.float32 and (3 * D) % 64 == 0:
            # compute-dtype operand written by the geometry kernel (the same RNE rounding the
            # GEMM would apply on load): both MLP GEMMs then run on the LDS-DMA path
            coords = op_empty(B * V * Nq, 3 * D, w0.dtype, dev)
            native.rv_query_coords_lowp(refB, l2i, i2l, coords, mask, B=B, V=V, Nq=Nq, D=D, pad_h=float(pad_h),
                                        pad_w=float(pad_w), pc_range=self.pc_range)
        else:
            coords = torch.empty((B * V * Nq, 3 * D), dtype=torch.float32, device=dev)
            native.rv_query_coords(refB, l2i, i2l, coords, mask, B=B, V=V, Nq=Nq, D=D, pad_h=float(pad_h),
                                   pad_w=float(pad_w), pc_range=self.pc_range)
        fused = self._rv_fused(pk)
        # the one-launch MLP also for the queries' 900 x 6 view rows (43 workgroups): alone the two
        # GEMMs' finer tiles finish sooner, but this runs on the second stream beside the K/V
        # side of the frame, where fewer, longer workgroups take fewer CUs from it (661.1 vs 658.3
        # frames/s alternating, profiles/r4z10_query_mlp_fused.txt)
        if fused is not None and coords.dtype == SPLIT:
            r = torch.empty((coords.shape[0], C), dtype=torch.float32, device=dev)
            _, b0, w2, b2 = pk["rv"]
            native.mlp2(coords, fused[0], b0, fused[1], b2, r, M=coords.shape[0], K=native.width(coords),
                        Hd=w2.shape[-1])
        else:
            r = self._mlp(coords, pk["rv"])
        tl, tp = first_ops if first_ops is not None else (None, None)
        native.masked_view_sum(r, mask, qpos, B=B, V=V, Nq=Nq, C=C, base=qb, Yl=tl, Yp=tp)
        return qpos, first_ops is not None

    # ------------------------------------------------------------------ per agent
    def _decode_agent(self, x, x_img, metas, B, out, post_flags, variant, prec, out16=None):
        """One get_outs_dec (cmt_head_coop.py:341-360) / the decoder part of
        forward_single (cmt_head.py:481-499); writes post-normed, nan_to_num'ed
        decoder outputs [L, B*Nq, C] into ``out`` (max-merged when post_flags
        has LN_MAX_INTO); ``out16`` receives the same values in the compute
        dtype (f16/bf16 policy)."""
        pk = self._engine_pack(prec)
        C = self.hidden_dim
        dev = self.reference_points.weight.device
        use_bev = variant != "image"
        use_img = variant != "lidar"
        HW = V = hw = 0
        if use_bev:
            _, _, H, W = x.shape
            HW = H * W
        if use_img:
            BV, _, hi, wi = x_img.shape
            V, hw = BV // B, hi * wi
        Nk = HW + V * hw
        lowp = prec.gemm != torch.float32
        # fp32 policy: memory / pos rows in fp32.  f16/bf16 policy: the K/V
        # GEMM operands lowp(memory) and lowp(memory + pos) are written
        # directly by the conv / layout epilogues and the pos-MLP epilogues.
        mdt = prec.gemm if lowp else torch.float32
        mem = op_empty(B * Nk, C, mdt, dev)
        pos = op_empty(B * Nk, C, mdt, dev)
        R = mem if lowp else None
        # reference numerics with the NCHW conv: lowp(memory + pos) of the BEV rows comes from the
        # conv epilogue plus the kept BEV position rows (CMT_BEV_POS_CACHE=0: the MLP runs per call)
        fuse_bev = use_bev and OPTIONS.bev_pos_cache and self._conv_halo_ok(x, pk, prec)
        dec = self.transformer.decoder
        Nq = self.num_query
        state = None
        side = self._side_stream(dev) if dec.prologue_ok(prec) else None
        # with the one-launch camera rows the camera matrices are first read after the conv: their
        # upload goes on the second stream, so the conv is the frame's first node (675.1 vs 672.8
        # frames/s, 3 alternating pairs; the main stream's wait for it before the camera rows costs
        # ~6 us of the ~10 it saves -- profiles/r5_experiments.txt r5am)
        late_cams = side is not None and use_img and use_bev and fuse_bev and self._rv_geo_ok(x_img, pk, prec)
        cams = self._cams(metas, dev) if use_img and not late_cams else None
        if side is not None:
            # A second stream runs everything that does not read the conv output: the
            # input-independent first halves of the BEV / RV position MLPs and the camera
            # memory rows (joined by an event before their second GEMMs, which add the
            # memory rows), then the query embedding and layer 0 up to the
            # cross-attention core (joined by run_rows before the first cross-attention).
            # With the NCHW conv (reference numerics) the RV half runs on the main stream
            # ahead of the conv instead (585.5 vs 582.2 frames/s A/B).
            # Buffers that outlive the side stream's work are allocated here, on the main
            # stream, or recorded on it.
            main = torch.cuda.current_stream()
            state = dec.lowp_state(B=B, Nk=Nk, Nq=Nq, prec=prec, device=dev)
            # the BEV position rows (weight-only, kept) folded into the conv epilogue
            P = self._bev_pos_rows(H, W, pk) if fuse_bev else None
            hb = hr = None
            # RV encoder's first half on the main stream, ahead of the conv: on the second stream
            # its kernels share the chip with the conv's and RV fc2 waits for them
            rv_main = use_img and fuse_bev
            # the camera memory rows in one launch after the conv (ABI 20): no coordinates or
            # layout launches ahead of the conv, no cross-stream wait before the RV MLP; the
            # second stream forks before the conv but is captured after it, so the conv takes the
            # chip first (profiles/r5_experiments.txt r5k / r5l)
            geo = rv_main and self._rv_geo_ok(x_img, pk, prec)
            if rv_main and not geo:
                hr = self._rv_pe_hidden(x_img, metas, B, pk, cams=cams)
            side.wait_stream(main)
            if geo:
                self._shared_conv_into(x, mem, Nk, pk, prec, pos=pos, P=P)
            ready = torch.cuda.Event()
            bev_ready = torch.cuda.Event()
            cams_ready = torch.cuda.Event()
            with torch.cuda.stream(side):
                if late_cams:
                    cams = self._cams(metas, dev)
                    cams_ready.record(side)
                if use_bev and not fuse_bev:
                    hb = self._bev_pos_hidden(H, W, pk)
                # the BEV position MLP's second GEMM waits only for its own hidden rows (usually a
                # kept pack: no kernel), not for the RV encoder's first half -- whose kernels
                # cannot start until shared_conv's workgroups leave the CUs
                bev_ready.record(side)
                if use_img and not geo:
                    native.nchw_to_rows(x_img.contiguous().float(), mem, nb=B, nv=V, C=C, HW=hw, ldy=C,
                                        range_flag=self._range_flag(x_img.device),
                                        rows_per_batch=Nk, row_offset=HW)
                    if not rv_main:
                        hr = self._rv_pe_hidden(x_img, metas, B, pk, cams=cams)
                ready.record(side)
                qpos, firsts = self._query_pos(B, metas, use_img, pk, cams=cams,
                                               first_ops=(state["tl"], state["tp"]))
                dec.lowp_layer0(state, qpos, B=B, Nq=Nq, prec=prec, first_ops_ready=firsts)
            for t in (qpos, hb, hr) + (tuple(cams) if late_cams else ()):
                if t is not None:
                    t.record_stream(main)
            if geo:
                if late_cams:
                    main.wait_event(cams_ready)
                self._rv_rows_geo(x_img, metas, B, Nk, HW, pk, mem, pos, cams)
            else:
                if use_bev and fuse_bev:
                    self._shared_conv_into(x, mem, Nk, pk, prec, pos=pos, P=P)
                elif use_bev:
                    self._shared_conv_into(x, mem, Nk, pk, prec)
                    main.wait_event(bev_ready)
                    self._bev_pos_out(hb, pos, B, Nk, pk, R=R)
                main.wait_event(ready)
                if use_img:
                    self._rv_pe_out(hr, pos, B, Nk, HW, pk, R=R)
        else:
            if use_bev and fuse_bev:
                self._shared_conv_into(x, mem, Nk, pk, prec, pos=pos, P=self._bev_pos_rows(H, W, pk))
            elif use_bev:
                self._shared_conv_into(x, mem, Nk, pk, prec)
                self._bev_pos_into(pos, B, Nk, H, W, pk, R=R)
            if use_img:
                native.nchw_to_rows(x_img.contiguous().float(), mem, nb=B, nv=V, C=C, HW=hw, ldy=C,
                                    range_flag=self._range_flag(x_img.device),
                                    rows_per_batch=Nk, row_offset=HW)
                self._rv_pe_into(pos, x_img, metas, B, Nk, HW, pk, R=R, cams=cams)
        if side is None:
            qpos, _ = self._query_pos(B, metas, use_img, pk, cams=cams)
        dec.run_rows(mem, pos, qpos, B=B, Nk=Nk, Nq=Nq, out=out, post_flags=post_flags, prec=prec,
                     kv_operands=(mem, pos) if lowp else None, out16=out16 if lowp else None, state=state)
        return out

    def _side_stream(self, dev):
        """The head's second HIP stream on ``dev`` (CMT_SIDE_STREAM=0: none)."""
        if dev.type != "cuda" or not OPTIONS.side_stream:
            return None
        pool = self.__dict__.setdefault("_side_streams", {})
        if dev not in pool:
            pool[dev] = torch.cuda.Stream(device=dev)
        return pool[dev]

    # ------------------------------------------------------------------ task heads
    def _task_outputs(self, outs_dec, B, prec, outs16=None):
        """SeparateTaskHead for every task + box epilogue.  outs_dec [L, B*Nq, C]
        fp32; ``outs16`` (optional) the same in the compute dtype, read by the
        first grouped conv's GEMM directly (LDS-DMA path) instead of
        converting fp32 on load -- the same bf16/f16 rounding either way."""
        plan = self._task_plan(outs_dec, B, prec, outs16)
        self._task_run(plan, 0, outs_dec.shape[0])
        return plan["ret"]

    def _task_plan(self, outs_dec, B, prec, outs16=None):
        """Output buffers of the task heads (allocated on the current stream)
        and the per-task packed weights; _task_run fills layers [l0, l1)."""
        L = outs_dec.shape[0]
        Nq = self.num_query
        ref = self.reference_points.weight.detach()
        tasks, ret = [], []
        for task in self.task_heads:
            tp = task.packed(prec)
            width = len(tp["names"]) * 64
            H1 = torch.empty((L, B * Nq, width), dtype=torch.float32, device=outs_dec.device)
            A = outs16 if outs16 is not None and outs16.dtype == tp["w1"].dtype else outs_dec
            OUT = torch.empty((L, B, Nq, tp["out_total"]), dtype=torch.float32, device=outs_dec.device)
            tasks.append((tp, A, H1, OUT))
            outs = {}
            start = 0
            for name, n in zip(tp["names"], tp["head_out"]):
                outs[name] = OUT[..., start:start + n]
                start += n
            ret.append(outs)
        refB = ref.unsqueeze(0).expand(B, Nq, 3).contiguous()
        return dict(tasks=tasks, ret=ret, refB=refB, B=B)

    def _task_run(self, plan, l0, l1):
        """Task heads of decoder layers [l0, l1): the grouped conv as one GEMM
        batched over the layers, then GroupLayerNorm1d + ReLU, conv #2 and the
        box epilogue (cmt_head.py:136-203, 501-513)."""
        B, Nq, C, n = plan["B"], self.num_query, self.hidden_dim, l1 - l0
        for tp, A, H1, OUT in plan["tasks"]:
            nh, k = len(tp["names"]), tp["k"]
            width = nh * 64
            # the grouped conv's groups are the decoder layers: weights of groups [l0, l1)
            native.gemm(A[l0:l1], tp["w1"][l0:l1], H1[l0:l1], M=B * Nq, N=width, K=k * C, lda=C, ldw=k * C, ldc=width,
                        batch=n, a_bstride=B * Nq * C, w_bstride=width * k * C, c_bstride=B * Nq * width,
                        a_mode=native.A_CONV1D3 if k == 3 else native.A_ROWS, seg_len=Nq)
            # box_epilogue = False (diagnostics / parity at the logit level): center and height
            # come out as the raw task-head logits, before + inverse_sigmoid(ref) and sigmoid
            epi = getattr(self, "box_epilogue", True)
            native.task_head_tail(H1[l0:l1], tp["gw"][l0:l1], tp["gb"][l0:l1], tp["w2"][l0:l1], tp["b2"][l0:l1],
                                  plan["refB"], OUT[l0:l1], L=n,
                                  B=B, Nq=Nq, nheads=nh, hc=64, head_out=tp["head_out"], k=k,
                                  center_col=tp["center_col"] if epi else -1,
                                  height_col=tp["height_col"] if epi else -1, pc_range=self.pc_range)

    def _check_eval(self):
        if self.training:
            raise RuntimeError("the fused inference path was reached in training mode: training goes through "
                               "forward_train (forward / forward_single / forward_agents route there)")
