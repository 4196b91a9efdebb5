"""Weight packing cache: converts module parameters once into the layouts and
dtypes the gfx950 kernels read (e.g. bf16 [N, K] rows, BN folded into the
conv, all decoder layers' K/V projections concatenated), and re-packs only when
a parameter changes (tracked through ``Tensor._version`` and storage
pointers, so optimizer steps and ``load_state_dict`` invalidate it)."""
import torch

__all__ = ["PackCache", "to_dtype"]


def _key(tensors, extra):
    return tuple((t.data_ptr(), t._version, tuple(t.shape)) for t in tensors) + (extra,)


class PackCache:
    def __init__(self):
        self._store = {}

    def get(self, name, tensors, extra, builder):
        k = _key(tensors, extra)
        hit = self._store.get(name)
        if hit is not None and hit[0] == k:
            return hit[1]
        with torch.no_grad():
            val = builder()
        self._store[name] = (k, val)
        return val

    def has(self, name, tensors, extra):
        hit = self._store.get(name)
        return hit is not None and hit[0] == _key(tensors, extra)

    def clear(self):
        self._store.clear()


def to_dtype(t, dtype):
    """Weights in a compute format: a torch dtype, or the split f16 pair
    (runtime.SPLIT, cmt_hip.h CMT_F16P): [..., K] -> [..., 2, K] with
    hi = f16(w), lo = f16(w - hi)."""
    if dtype == torch.uint16:
        w = t.detach().float()
        if w.numel() and w.abs().max().item() >= 65504.0:
            raise ValueError("weights beyond the f16 range cannot take the split f16 pair format")
        hi = w.half()
        lo = (w - hi.float()).half()
        return torch.stack([hi, lo], dim=-2).contiguous().view(torch.uint16)
    return t.detach().to(dtype).contiguous()
