"""MultiTaskBBoxCoder (NMS-free decode) with the reference's API.

Reference: projects/mmdet3d_plugin/core/bbox/coders/multi_task_bbox_coder.py:15-142,
denormalize_bbox core/bbox/util.py:37-68.  Decode is outside the decoder-frame
hot path; it runs as device-side torch ops on the head's
outputs (sigmoid, top-k over Nq*classes, gather, exp/atan2, range mask).  A
fused top-k kernel is SURVEY.md 8(f) next #1.
"""
import torch

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

    def decode_single(self, cls_scores, bbox_preds, task_ids):
        """multi_task_bbox_coder.py:46-100."""
        max_num = self.max_num
        num_query = cls_scores.shape[0]
        cls_scores = cls_scores.sigmoid()
        scores, indexs = cls_scores.reshape(-1).topk(max_num)
        labels = indexs % self.num_classes
        bbox_index = torch.div(indexs, self.num_classes, rounding_mode="floor")
        task_index = torch.gather(task_ids, 1, labels.unsqueeze(1)).squeeze(1)
        bbox_preds = bbox_preds[task_index * num_query + bbox_index]
        final_box_preds = denormalize_bbox(bbox_preds, self.pc_range)
        if self.post_center_range is None:
            raise NotImplementedError("Need to reorganize output as a batch, only support post_center_range is "
                                      "not None for now!")
        pcr = torch.as_tensor(self.post_center_range, device=scores.device, dtype=final_box_preds.dtype)
        mask = (final_box_preds[..., :3] >= pcr[:3]).all(1)
        mask &= (final_box_preds[..., :3] <= pcr[3:]).all(1)
        if self.score_threshold:
            mask &= scores > self.score_threshold
        return {"bboxes": final_box_preds[mask], "scores": scores[mask], "labels": labels[mask]}

    def decode(self, preds_dicts):
        """multi_task_bbox_coder.py:102-142 (last decoder layer, tasks concatenated)."""
        bbox_l, logit_l, tid_l = [], [], []
        for task_id in range(len(preds_dicts)):
            d = preds_dicts[task_id][0]
            bbox_l.append(torch.cat((d["center"][-1], d["height"][-1], d["dim"][-1], d["rot"][-1], d["vel"][-1]),
                                    dim=-1))
            logits = d["cls_logits"][-1]
            logit_l.append(logits)
            tid_l.append(torch.full(logits.shape, task_id, dtype=torch.int64, device=logits.device))
        all_logits = torch.cat(logit_l, dim=-1)
        all_bbox = torch.cat(bbox_l, dim=1)
        all_tids = torch.cat(tid_l, dim=-1)
        return [self.decode_single(all_logits[i], all_bbox[i], all_tids[i]) for i in range(all_logits.shape[0])]
