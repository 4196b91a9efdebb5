"""Checkpoint formats around the head.

* ``load_head_checkpoint``: an mmcv detector checkpoint (``{'state_dict': ...,
  'meta': ...}`` or a bare state dict) -> the head's state dict.  The head's
  parameters live under ``pts_bbox_head.`` in the detector
  (``cmt.py`` / ``cmt_coop.py`` build the head as ``self.pts_bbox_head``);
  key names inside the prefix are the reference's, so they
  load unchanged.
* ``convert_agent_checkpoint`` / ``merge_coop_checkpoints``: the key rewrite
  of ``tools/model_converters/convert_cmtcoop_checkpoints.py`` that turns
  single-agent CmtDetector checkpoints into one CmtCoopDetector checkpoint:
  ``update_ckpt`` 82-151 (delete prefixes, then insert prefixes, then permute
  5-D sparse-conv weights), ``update_ckpt_vehicle`` 155-218 /
  ``update_ckpt_infrastructure`` 222-284 (the per-agent tables), ``main``
  287-372 (lidar/camera halves merged camera-first so LiDAR keys win, then
  vehicle-first so infrastructure keys win on the shared head keys).

Files are read with ``torch.load(..., weights_only=True)`` only: nothing in a
checkpoint is executed.
"""
import os

import torch

__all__ = ["read_state_dict", "load_head_checkpoint", "convert_agent_checkpoint", "merge_coop_checkpoints",
           "AGENTS", "HEAD_PREFIX"]

HEAD_PREFIX = "pts_bbox_head."
# feature-extractor modules that move under '<agent>_model.' (convert_cmtcoop_checkpoints.py:163-170, 231-238)
_MODULES = ("img_backbone", "img_neck", "pts_voxel_encoder", "pts_middle_encoder", "pts_backbone", "pts_neck")
# spconv v1 -> v2 kernel layout of the sparse middle encoder (174-178, 241-245)
_PERMUTED = ("pts_middle_encoder.conv_input", "pts_middle_encoder.encoder_layers", "pts_middle_encoder.conv_out")
_PERM = (1, 2, 3, 4, 0)
AGENTS = ("vehicle", "infrastructure")


def read_state_dict(src):
    """Path or dict -> flat state dict (unwraps mmcv's ``{'state_dict': ...}``)."""
    if isinstance(src, (str, os.PathLike)):
        src = torch.load(src, map_location="cpu", weights_only=True)
    if isinstance(src, dict) and "state_dict" in src and isinstance(src["state_dict"], dict):
        src = src["state_dict"]
    return dict(src)


def load_head_checkpoint(head, src, strict=True):
    """Load the ``pts_bbox_head.*`` part of a detector checkpoint (or a bare
    head state dict) into ``head``.  Returns torch's (missing, unexpected)."""
    sd = read_state_dict(src)
    if any(k.startswith(HEAD_PREFIX) for k in sd):
        sd = {k[len(HEAD_PREFIX):]: v for k, v in sd.items() if k.startswith(HEAD_PREFIX)}
    return head.load_state_dict(sd, strict=strict)


def convert_agent_checkpoint(sd, agent, prefix=None, wo_trans=False):
    """``update_ckpt_vehicle`` / ``update_ckpt_infrastructure`` on one
    single-agent detector state dict.  ``prefix`` ('pts' / 'img') restricts
    the renamed modules to one modality, as for the separate lidar / camera
    checkpoints; ``wo_trans`` also drops the head's transformer."""
    if agent not in AGENTS:
        raise ValueError(f"agent must be one of {AGENTS}")
    other = AGENTS[1 - AGENTS.index(agent)]
    insert = {m: f"{agent}_model.{m}" for m in _MODULES if prefix is None or m.startswith(prefix)}
    permute = {f"{agent}_model.{p}": _PERM for p in _PERMUTED}
    delete = [f"{other}_model", HEAD_PREFIX + "task_heads"]
    if wo_trans:
        delete.append(HEAD_PREFIX + "transformer")
    out = {k: v for k, v in read_state_dict(sd).items() if not any(k.startswith(d) for d in delete)}
    renamed = {}
    for k, v in out.items():
        nk = k
        for old, new in insert.items():
            if k.startswith(old):
                nk = k.replace(old, new)   # the reference's str.replace (every occurrence)
        renamed[nk] = v
    for k, v in renamed.items():
        for p, perm in permute.items():
            if k.startswith(p) and torch.is_tensor(v) and v.dim() == len(perm):
                renamed[k] = v.permute(perm)
    return renamed


def merge_coop_checkpoints(vehicle=None, infrastructure=None, vehicle_lidar=None, vehicle_camera=None,
                           infrastructure_lidar=None, infrastructure_camera=None, wo_trans=False):
    """``main`` of convert_cmtcoop_checkpoints.py without the model build:
    whole-agent checkpoints, or per-modality halves, -> one coop state dict."""
    def agent_sd(agent, whole, lidar, camera):
        if whole is not None:
            return convert_agent_checkpoint(whole, agent, wo_trans=wo_trans)
        pts = convert_agent_checkpoint(lidar, agent, prefix="pts", wo_trans=wo_trans) if lidar is not None else {}
        img = convert_agent_checkpoint(camera, agent, prefix="img", wo_trans=wo_trans) if camera is not None else {}
        return {**img, **pts}

    v = agent_sd("vehicle", vehicle, vehicle_lidar, vehicle_camera)
    i = agent_sd("infrastructure", infrastructure, infrastructure_lidar, infrastructure_camera)
    return {**v, **i}
