"""Native box decode (cmt_box_decode via MultiTaskBBoxCoder / get_bboxes)
vs the oracle's restatement of MultiTaskBBoxCoder.decode + get_bboxes
(oracle/cmt_oracle.py decode)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ("center", "height", "dim", "rot", "vel")
WIDTH = {"center": 2, "height": 1, "dim": 3, "rot": 2, "vel": 2}


def _preds(B, Nq, class_split, seed, ties=False):
    g = torch.Generator().manual_seed(seed)
    preds = []
    for n in class_split:
        d = {k: torch.randn(6, B, Nq, w, generator=g) * (30 if k == "center" else 1) for k, w in WIDTH.items()}
        d["cls_logits"] = torch.randn(6, B, Nq, n, generator=g) * 2
        if ties:   # a block of equal logits straddling the k-th value
            d["cls_logits"][-1, :, :40, 0] = 0.25
        preds.append(d)
    return preds


@pytest.mark.parametrize("B,Nq,split,max_num,thr,ties", [(1, 900, [10], 300, None, False),
                                                        (2, 300, [3, 4], 100, 0.3, False),
                                                        (1, 200, [10], 150, None, True),
                                                        (3, 400, [7], 350, 0.05, False)])
def test_native_decode_matches_oracle(dev, B, Nq, split, max_num, thr, ties):
    from oracle import cmt_oracle as O
    from projects.mmdet3d_plugin.core.bbox.coders import MultiTaskBBoxCoder
    preds = _preds(B, Nq, split, seed=B * 100 + Nq, ties=ties)
    ncls = sum(split)
    pcr = [-61.2, -61.2, -10.0, 61.2, 61.2, 10.0]
    ref = O.decode(preds, ncls, max_num=max_num, post_center_range=pcr, score_threshold=thr)
    coder = MultiTaskBBoxCoder(pc_range=[-54, -54, -5, 54, 54, 3], post_center_range=pcr, max_num=max_num,
                               score_threshold=thr, num_classes=ncls)
    got = coder.decode([[{k: v.to(dev) for k, v in d.items()}] for d in preds])
    for b in range(B):
        r, g = ref[b], got[b]
        gb = g["bboxes"].cpu().clone()
        gb[:, 2] = gb[:, 2] - gb[:, 5] * 0.5          # the z-shift get_bboxes applies (oracle.decode includes it)
        assert g["scores"].shape == r["scores"].shape
        assert torch.allclose(g["scores"].cpu(), r["scores"], atol=1e-6)
        assert torch.equal(g["labels"].cpu(), r["labels"].long())
        assert torch.allclose(gb, r["bboxes"], atol=1e-4, rtol=1e-5)
        if len(g["scores"]) > 1:
            assert (g["scores"][:-1] >= g["scores"][1:]).all()
