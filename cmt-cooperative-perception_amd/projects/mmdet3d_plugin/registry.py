"""Minimal OpenMMLab-style registries.

The reference registers its classes into mmcv/mmdet/mmdet3d registries
(``@HEADS.register_module()`` at cmt_head.py:97,206,922,1002,
cmt_head_coop.py:72,812,914; ``@TRANSFORMER.register_module()`` at
cmt_transformer.py:48,130,207; ``@ATTENTION`` / ``@TRANSFORMER_LAYER(_SEQUENCE)``
at petr_transformer.py:182,324,374; ``@BBOX_CODERS`` at
multi_task_bbox_coder.py:15).  mmcv is not available on MI355X boxes here, so
this module provides the same ``register_module`` / ``build`` contract and the
same registry names, so config dicts (``dict(type='CmtHead', ...)``) build
unchanged.
"""
import copy
import inspect

__all__ = ["Registry", "build_from_cfg", "HEADS", "TRANSFORMER", "ATTENTION", "TRANSFORMER_LAYER",
           "TRANSFORMER_LAYER_SEQUENCE", "FEEDFORWARD_NETWORK", "BBOX_CODERS", "VOXEL_LAYERS",
           "NORM_LAYERS", "build_head", "build_transformer", "build_bbox_coder"]


class Registry:
    def __init__(self, name, parent=None):
        self.name = name
        self._modules = {}
        self.parent = parent

    def __contains__(self, key):
        return self.get(key) is not None

    def __repr__(self):
        return f"Registry(name={self.name}, items={sorted(self._modules)})"

    def get(self, key):
        if key in self._modules:
            return self._modules[key]
        if self.parent is not None:
            return self.parent.get(key)
        return None

    def register_module(self, name=None, force=False, module=None):
        def _register(cls):
            key = name or cls.__name__
            if not force and key in self._modules and self._modules[key] is not cls:
                raise KeyError(f"{key} is already registered in {self.name}")
            self._modules[key] = cls
            return cls
        if module is not None:
            return _register(module)
        return _register

    def build(self, cfg, **default_args):
        return build_from_cfg(cfg, self, default_args)


def build_from_cfg(cfg, registry, default_args=None):
    """mmcv.utils.build_from_cfg semantics: pop ``type``, look it up, call it
    with the remaining keys (defaults filled from default_args)."""
    if not isinstance(cfg, dict) or "type" not in cfg:
        raise TypeError(f"cfg must be a dict with a 'type' key, got {cfg!r}")
    args = copy.deepcopy(dict(cfg))
    if default_args:
        for k, v in default_args.items():
            args.setdefault(k, v)
    obj_type = args.pop("type")
    if isinstance(obj_type, str):
        obj_cls = registry.get(obj_type)
        if obj_cls is None:
            raise KeyError(f"{obj_type} is not in the {registry.name} registry")
    elif inspect.isclass(obj_type):
        obj_cls = obj_type
    else:
        raise TypeError(f"type must be a str or class, got {type(obj_type)}")
    return obj_cls(**args)


# mmcv / mmdet registries share one class namespace per kind; mirror the names.
MODELS = Registry("models")
HEADS = Registry("head", parent=MODELS)
TRANSFORMER = Registry("Transformer", parent=MODELS)
ATTENTION = Registry("attention", parent=MODELS)
TRANSFORMER_LAYER = Registry("transformerLayer", parent=MODELS)
TRANSFORMER_LAYER_SEQUENCE = Registry("transformer-layers sequence", parent=MODELS)
FEEDFORWARD_NETWORK = Registry("feed-forward Network", parent=MODELS)
NORM_LAYERS = Registry("norm layer", parent=MODELS)
BBOX_CODERS = Registry("bbox_coder")
VOXEL_LAYERS = Registry("voxel_layer")


def build_head(cfg, **kw):
    return build_from_cfg(cfg, HEADS, kw or None)


def build_transformer(cfg, **kw):
    return build_from_cfg(cfg, TRANSFORMER, kw or None)


def build_bbox_coder(cfg, **kw):
    return build_from_cfg(cfg, BBOX_CODERS, kw or None)
