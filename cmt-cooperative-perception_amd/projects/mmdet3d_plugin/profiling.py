"""Optional HIP-event timing of named regions on the launching stream.

``with region_timer() as t: ...`` activates it; hot-path code wraps kernels it
wants timed in ``timed("name")`` (a no-op when no timer is active).  Events
are recorded on torch's current stream, which is the stream every ctypes
launch of this package uses, so a region brackets exactly its kernels.
"""
import contextlib
from collections import defaultdict

import torch

__all__ = ["region_timer", "timed", "RegionTimer"]

_ACTIVE = None


class RegionTimer:
    def __init__(self):
        self.pairs = defaultdict(list)

    def durations_ms(self, name):
        torch.cuda.synchronize()
        return [a.elapsed_time(b) for a, b in self.pairs[name]]

    def mean_ms(self, name):
        d = self.durations_ms(name)
        return sum(d) / len(d) if d else float("nan")


@contextlib.contextmanager
def region_timer():
    global _ACTIVE
    prev = _ACTIVE
    _ACTIVE = RegionTimer()
    try:
        yield _ACTIVE
    finally:
        _ACTIVE = prev


@contextlib.contextmanager
def timed(name):
    t = _ACTIVE
    if t is None or torch.cuda.is_current_stream_capturing():
        yield
        return
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    try:
        yield
    finally:
        b.record()
        t.pairs[name].append((a, b))
