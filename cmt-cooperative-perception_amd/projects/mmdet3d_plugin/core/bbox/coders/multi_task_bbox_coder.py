"""MultiTaskBBoxCoder (NMS-free decode) with the reference's API.

Reference: projects/mmdet3d_plugin/core/bbox/coders/multi_task_bbox_coder.py:15-142,
denormalize_bbox core/bbox/util.py:37-68.  Decode
runs as ONE native launch for the whole batch (cmt_box_decode: sigmoid,
top-k over Nq*classes by LDS radix select, gather, exp/atan2 denormalisation,
post-center-range / score mask, in-order compaction); the host only slices
each sample's [:count] rows.
"""
import torch

from .... import native
from ....registry import BBOX_CODERS

__all__ = ["MultiTaskBBoxCoder", "denormalize_bbox"]


def denormalize_bbox(nb, pc_range=None):
    """core/bbox/util.py:37-68."""
    cx, cy, cz = nb[..., 0:1], nb[..., 1:2], nb[..., 2:3]
    w, l, h = nb[..., 3:4].exp(), nb[..., 4:5].exp(), nb[..., 5:6].exp()
    rot = torch.atan2(nb[..., 6:7], nb[..., 7:8])
    if nb.size(-1) > 8:
        return torch.cat([cx, cy, cz, w, l, h, rot, nb[..., 8:9], nb[..., 9:10]], dim=-1)
    return torch.cat([cx, cy, cz, w, l, h, rot], dim=-1)


@BBOX_CODERS.register_module()
class MultiTaskBBoxCoder:
    def __init__(self, pc_range, voxel_size=None, post_center_range=None, max_num=100, score_threshold=None,
                 num_classes=10):
        self.pc_range = pc_range
        self.voxel_size = voxel_size
        self.post_center_range = post_center_range
        self.max_num = max_num
        self.score_threshold = score_threshold
        self.num_classes = num_classes

    def encode(self):
        pass

    def decode(self, preds_dicts):
        """multi_task_bbox_coder.py:102-142: last decoder layer, tasks'
        classes concatenated, boxes of task t at rows [t*Nq, (t+1)*Nq)."""
        if self.post_center_range is None:
            raise NotImplementedError("Need to reorganize output as a batch, only support post_center_range is "
                                      "not None for now!")
        bbox_l, logit_l, class_task = [], [], []
        for task_id in range(len(preds_dicts)):
            d = preds_dicts[task_id][0]
            bbox_l.append(torch.cat((d["center"][-1], d["height"][-1], d["dim"][-1], d["rot"][-1], d["vel"][-1]),
                                    dim=-1))
            logits = d["cls_logits"][-1]
            logit_l.append(logits)
            class_task += [task_id] * logits.shape[-1]
        all_logits = torch.cat(logit_l, dim=-1).float().contiguous()           # [B, Nq, ncls]
        all_bbox = torch.cat(bbox_l, dim=1).float().contiguous()               # [B, T*Nq, code]
        B, Nq, ncls = all_logits.shape
        ct = torch.tensor(class_task, dtype=torch.int32, device=all_logits.device)
        boxes, scores, labels, count = native.box_decode(all_logits.view(B, Nq * ncls), all_bbox, ct, Nq=Nq,
                                                         ncls=ncls, max_num=self.max_num,
                                                         post_center_range=self.post_center_range,
                                                         score_threshold=self.score_threshold)
        counts = count.tolist()
        return [{"bboxes": boxes[i, :n], "scores": scores[i, :n], "labels": labels[i, :n].long()}
                for i, n in enumerate(counts)]
