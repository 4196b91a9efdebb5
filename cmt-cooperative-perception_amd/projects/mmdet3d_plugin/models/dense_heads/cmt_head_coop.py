"""Cooperative (vehicle + infrastructure) CMT heads on the gfx950 kernels.

Reference: projects/mmdet3d_plugin/models/dense_heads/cmt_head_coop.py
  filter_img_metas 41-57, CmtHeadCoop 72-809 (get_outs_dec 341-360,
  forward_single 362-437, max-fusion 383-389), CmtImageHeadCoop 812-911,
  CmtLidarHeadCoop 914-1017.
One decoder pass per agent with the shared head weights; the element-wise
max over agents is fused into the post_norm kernel of the second agent
(LN_MAX_INTO), then the task heads run once.  ``forward_agents`` generalises
the two-agent max to any number of agents (the 4-agent stress config) and can
shard the agents over the ranks of a process group (one MAX all-reduce).
"""
import torch

from ...registry import HEADS
from .cmt_head import CmtHead, gt_from_metas, multi_apply

__all__ = ["filter_img_metas", "get_vehicle_image_metas", "get_infrastructure_image_metas", "CmtHeadCoop",
           "CmtLidarHeadCoop", "CmtImageHeadCoop"]


def filter_img_metas(img_meta, prefix="", ignore=""):
    """cmt_head_coop.py:41-57."""
    out = dict()
    for k, v in img_meta.items():
        if k.startswith(prefix):
            out[k[len(prefix):]] = v
        elif not k.startswith(ignore):
            out[k] = v
    out["node"] = prefix
    return out


def get_infrastructure_image_metas(img_metas):
    return [filter_img_metas(m, prefix="infrastructure_", ignore="vehicle_") for m in img_metas]


def get_vehicle_image_metas(img_metas):
    return [filter_img_metas(m, prefix="vehicle_", ignore="infrastructure_") for m in img_metas]


@HEADS.register_module()
class CmtHeadCoop(CmtHead):
    """cmt_head_coop.py:72-809 (fusion: LiDAR BEV + camera per agent)."""
    variant = "fusion"

    def forward_single(self, x_vehicle, x_infrastructure, x_img_vehicle, x_img_infrastructure, img_metas):
        B = len(img_metas)
        agents, fns = [], []
        for x, xi, prefix in ((x_vehicle, x_img_vehicle, "vehicle_"),
                              (x_infrastructure, x_img_infrastructure, "infrastructure_")):
            if x is not None or xi is not None:
                fn = (lambda m, p=prefix: self._agent_metas(m, p))
                agents.append((x, xi, fn(img_metas)))
                fns.append(fn)
        if not agents:
            raise ValueError("CmtHeadCoop needs at least one agent's features")
        if self.training:   # cmt_head_coop.py:205-275 training branch (DN queries, shared GT)
            return self.forward_train(agents, img_metas, *gt_from_metas(img_metas))
        return self._forward_agents(agents, img_metas, B, meta_fns=fns)

    def _agent_metas(self, img_metas, prefix):
        if self.variant == "lidar":
            return img_metas
        return get_vehicle_image_metas(img_metas) if prefix == "vehicle_" else get_infrastructure_image_metas(img_metas)

    def forward(self, vehicle_pts_feats, infrastructure_pts_feats, vehicle_img_feats=None,
                infrastructure_img_feats=None, img_metas=None):
        """cmt_head_coop.py:439-444."""
        n = len(vehicle_pts_feats) if vehicle_pts_feats is not None else len(vehicle_img_feats)
        none = [None] * n
        img_metas = [img_metas for _ in range(n)]
        return multi_apply(self.forward_single, vehicle_pts_feats or none, infrastructure_pts_feats or none,
                           vehicle_img_feats or none, infrastructure_img_feats or none, img_metas)

    def forward_agents(self, agents, img_metas, group=None):
        """Any number of agents: ``agents`` = list of (prefix, pts_feat, img_feat);
        outputs max-fused over agents (the reference fuses exactly two).  Agent
        metas are selected by key prefix as filter_img_metas does for the two
        reference agents; with other prefixes (e.g. 'agent2_') every other
        agent's prefixed keys are dropped.

        ``group``: a torch.distributed process group (or True for the default
        group) over which the agents are SHARDED -- rank r decodes agents r,
        r + world, ... and one all_reduce(MAX) fuses them (configs[4] latency
        option); every rank passes the same agent list (a rank
        only reads the features of its own agents) and gets the fused outputs."""
        B = len(img_metas)
        prefixes = [p for p, _, _ in agents]
        if set(prefixes) <= {"vehicle_", "infrastructure_"}:
            fns = [(lambda m, p=p: self._agent_metas(m, p)) for p in prefixes]
        else:
            fns = [(lambda m, p=p: [self._select_metas(mm, p, prefixes) for mm in m] if self.variant != "lidar"
                    else m) for p in prefixes]
        triples = [(x, xi, fn(img_metas)) for (_, x, xi), fn in zip(agents, fns)]
        if self.training:
            return self.forward_train(triples, img_metas, *gt_from_metas(img_metas))
        shard = None
        if group is not None:
            import torch.distributed as dist
            g = None if group is True else group
            shard = (dist.get_rank(g), dist.get_world_size(g), g)
        return self._forward_agents(triples, img_metas, B, meta_fns=fns, shard=shard)

    @staticmethod
    def _select_metas(meta, prefix, prefixes):
        out = {}
        for k, v in meta.items():
            if k.startswith(prefix):
                out[k[len(prefix):]] = v
            elif not any(k.startswith(p) for p in prefixes):
                out[k] = v
        out["node"] = prefix
        return out


@HEADS.register_module()
class CmtImageHeadCoop(CmtHeadCoop):
    """cmt_head_coop.py:812-911."""
    variant = "image"

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.shared_conv = None


@HEADS.register_module()
class CmtLidarHeadCoop(CmtHeadCoop):
    """cmt_head_coop.py:914-1017."""
    variant = "lidar"

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.rv_embedding = None
