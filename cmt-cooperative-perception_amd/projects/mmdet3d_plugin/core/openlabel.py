"""Detections -> OpenLABEL JSON (the output wire format).

Restates ``tools/inference_to_openlabel_coop.py``:

* ``box_corners``            -- ``get_corners`` 37-53 (BEV corners of a yawed box)
* ``Detection``              -- the ``Detection`` dataclass 56-103 (the fields the
                                exporter reads; ids count up per process as there)
* ``detections_to_openlabel``-- 167-285: one frame, objects keyed by uuid, cuboid
                                ``[x, y, z, qx, qy, qz, qw, dx, dy, dz]`` with the
                                quaternion of the xyz-Euler rotation (0, 0, yaw)
                                (scipy ``as_quat`` order: scalar last), text / num /
                                vec attributes in the reference's order
* ``boxes_to_detections``    -- the per-frame loop of ``main`` 423-502: optional
                                class / score filters, location = bottom centre
                                lifted by half the height, yaw negated, and the
                                number of points inside the box.  As there, the
                                point count uses an oriented box CENTRED at the
                                box's (bottom-centre) (x, y, z) with extent
                                (dx, dy, dz) and rotation yaw about z (open3d
                                ``OrientedBoundingBox`` built from ``bbox[:3]``);
                                the points are the xyz columns given.

open3d and scipy's Rotation are not needed: the point-in-box test and the
quaternion are closed-form numpy.  Host-side formatting only: no device code.
"""
import json
import math
import os
import uuid as _uuid
from dataclasses import dataclass, field
from typing import Any, List, Optional, Tuple

import numpy as np

__all__ = ["box_corners", "Detection", "detections_to_openlabel", "boxes_to_detections", "points_in_box",
           "yaw_quaternion", "DEFAULT_SENSOR_ID"]

DEFAULT_SENSOR_ID = "s110_lidar_ouster_south"   # inference_to_openlabel_coop.py:491
_next_detection_id = [0]


def box_corners(yaw: float, width: float, length: float, position: np.ndarray) -> np.ndarray:
    """The 4 BEV corners (get_corners 37-53): +-length/2 along the heading,
    +-width/2 across it, around ``position`` (3-vector)."""
    v1 = np.array([math.cos(yaw), math.sin(yaw), 0.0]) * (length * 0.5)
    v2 = np.array([-math.sin(yaw), math.cos(yaw), 0.0]) * (width * 0.5)
    pos = np.asarray(position, dtype=float).flatten()
    return np.array([pos + v1 + v2, pos - v1 + v2, pos - v1 - v2, pos + v1 - v2])


@dataclass
class Detection:
    """One detected road user (the fields of inference_to_openlabel_coop.py:56-103
    the exporter reads)."""
    location: np.ndarray
    dimensions: Tuple[float, float, float]
    yaw: float
    category: str
    bbox_2d: Optional[np.ndarray] = None          # [x_min, y_min, x_max, y_max]
    id: int = -1
    sensor_id: Optional[str] = ""
    uuid: str = ""
    pos_history: Optional[List[np.ndarray]] = field(default_factory=list)
    color: Optional[str] = None
    num_lidar_points: int = 0
    score: float = 0.0
    occlusion_level: Optional[str] = None
    overlap: bool = False
    extra: Optional[Any] = None

    def __post_init__(self):
        if self.id == -1:
            self.id = _next_detection_id[0]
        _next_detection_id[0] += 1

    def get_corners(self) -> np.ndarray:
        return box_corners(self.yaw, self.dimensions[1], self.dimensions[0], self.location)


def yaw_quaternion(yaw: float) -> List[float]:
    """Rotation.from_euler('xyz', [0, 0, yaw]).as_quat(): (x, y, z, w)."""
    return [0.0, 0.0, math.sin(0.5 * yaw), math.cos(0.5 * yaw)]


def _num(v):
    return float(v) if isinstance(v, (np.floating, float)) else v


def detections_to_openlabel(detection_list: List[Detection], filename: Optional[str] = None,
                            output_folder_path: Optional[str] = None, coordinate_systems=None,
                            frame_properties=None, frame_id=None, streams=None) -> dict:
    """inference_to_openlabel_coop.py:167-285.  Returns the JSON object and
    writes it (indent 4) to ``output_folder_path/filename`` when both are given."""
    out = {"openlabel": {"metadata": {"schema_version": "1.0.0"}, "coordinate_systems": {}}}
    if coordinate_systems:
        out["openlabel"]["coordinate_systems"] = coordinate_systems
    if frame_id is None:
        frame_id = "0"
    frame_id = str(frame_id)
    frame_map = {frame_id: {}}
    objects = {}
    for idx, det in enumerate(detection_list):
        pos = np.asarray(det.location, dtype=float).flatten()
        quat = yaw_quaternion(float(det.yaw))
        dims = det.dimensions
        object_id = str(det.uuid) or str(idx)
        attrs = {"text": [], "num": [], "vec": []}
        if det.color is not None:
            attrs["text"].append({"name": "body_color", "val": det.color.lower()})
        attrs["text"].append({"name": "overlap", "val": str(det.overlap)})
        if det.occlusion_level is not None:
            attrs["text"].append({"name": "occlusion_level", "val": det.occlusion_level})
        if det.sensor_id is not None:
            attrs["text"].append({"name": "sensor_id", "val": det.sensor_id})
        attrs["num"].append({"name": "num_points", "val": int(det.num_lidar_points)})
        attrs["num"].append({"name": "score", "val": float(det.score)})
        if det.bbox_2d is not None:
            b = det.bbox_2d
            w, h = float(b[2] - b[0]), float(b[3] - b[1])
            bbox_2d = [{"name": "shape", "val": [float(b[0] + w / 2.0), float(b[1] + h / 2.0), w, h]}]
        else:
            bbox_2d = []
        if det.pos_history is not None:
            hist = []
            for p in det.pos_history:
                q = np.asarray(p, dtype=float).flatten().tolist()
                hist.extend(q[:3])
            attrs["vec"].append({"name": "track_history", "val": hist})
        objects[object_id] = {
            "object_data": {
                "name": det.category.upper() + "_" + object_id.split("-")[0],
                "type": det.category.upper(),
                "cuboid": {
                    "name": "shape3D",
                    "val": [float(pos[0]), float(pos[1]), float(pos[2]), quat[0], quat[1], quat[2], quat[3],
                            _num(dims[0]), _num(dims[1]), _num(dims[2])],
                    "attributes": attrs,
                },
                "bbox": bbox_2d,
            }
        }
    frame_map[frame_id]["objects"] = objects
    if frame_properties:
        frame_map[frame_id]["frame_properties"] = frame_properties
    if streams:
        out["openlabel"]["streams"] = streams
    out["openlabel"]["frames"] = frame_map
    if filename is not None and output_folder_path is not None:
        os.makedirs(output_folder_path, exist_ok=True)
        with open(os.path.join(output_folder_path, filename), "w", encoding="utf-8") as f:
            json.dump(out, f, indent=4)
    return out


def points_in_box(points_xyz: np.ndarray, center, extent, yaw: float) -> int:
    """Points inside an oriented box (open3d ``get_point_indices_within_bounding_box``
    on an ``OrientedBoundingBox`` with R = rot_z(yaw)): |R^T (p - c)| <= extent / 2
    per axis, boundary included."""
    if points_xyz is None or len(points_xyz) == 0:
        return 0
    p = np.asarray(points_xyz, dtype=np.float64)[:, :3] - np.asarray(center, dtype=np.float64)[None, :3]
    c, s = math.cos(yaw), math.sin(yaw)
    lx = c * p[:, 0] + s * p[:, 1]
    ly = -s * p[:, 0] + c * p[:, 1]
    half = 0.5 * np.asarray(extent, dtype=np.float64)
    inside = (np.abs(lx) <= half[0]) & (np.abs(ly) <= half[1]) & (np.abs(p[:, 2]) <= half[2])
    return int(inside.sum())


def boxes_to_detections(bboxes, scores, labels, class_names, points_xyz=None, bbox_classes=None, bbox_score=None,
                        sensor_id=DEFAULT_SENSOR_ID, uuid_fn=None) -> List[Detection]:
    """The per-frame loop of inference_to_openlabel_coop.py:452-494 on decoded
    boxes ``[n, >= 7]`` (x, y, z_bottom, dx, dy, dz, yaw, ...), scores [n] and
    labels [n] (tensors or arrays).  ``uuid_fn``: uuid source (default uuid4)."""
    to_np = lambda t: t.detach().cpu().numpy() if hasattr(t, "detach") else np.asarray(t)  # noqa: E731
    b, s, lab = to_np(bboxes), to_np(scores), to_np(labels)
    if bbox_classes is not None:
        keep = np.isin(lab, bbox_classes)
        b, s, lab = b[keep], s[keep], lab[keep]
    if bbox_score is not None:
        keep = s >= bbox_score
        b, s, lab = b[keep], s[keep], lab[keep]
    uuid_fn = uuid_fn or (lambda: str(_uuid.uuid4()))
    dets = []
    for i, box in enumerate(b):
        loc = np.asarray([[box[0]], [box[1]], [box[2] + 0.5 * box[5]]], dtype=float)
        npts = 0 if points_xyz is None else points_in_box(points_xyz, box[:3], box[3:6], float(box[6]))
        dets.append(Detection(uuid=uuid_fn(), category=class_names[int(lab[i])], location=loc,
                              dimensions=(float(box[3]), float(box[4]), float(box[5])), yaw=-float(box[6]),
                              num_lidar_points=npts, score=float(s[i]), sensor_id=sensor_id))
    return dets
