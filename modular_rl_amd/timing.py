"""Optional HIP-event timing of named launch regions on the current stream.

Disabled by default (zero cost); bench.py enables it to measure the average
device duration of the dominant kernels live inside the timed region.
"""
import collections

import torch

_ENABLED = False
_open = {}
_events = collections.defaultdict(list)
meta = {}  # name -> per-launch algorithmic work of the region (e.g. a GEMM's FLOP / bytes)


def enable(on=True):
    global _ENABLED
    _ENABLED = on
    _open.clear()
    if on:  # a new measurement; turning timing off keeps the last one's records readable
        _events.clear()
        meta.clear()


def enabled():
    return _ENABLED


def start(name):
    if _ENABLED:
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        _open[name] = e


def stop(name):
    if _ENABLED:
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        _events[name].append((_open.pop(name), e))


def region(name, fn, *args, **info):
    """fn(*args) timed as one region `name` (when enabled), with the region's per-launch
    work recorded in ``meta[name]``."""
    if not _ENABLED:
        return fn(*args)
    meta.setdefault(name, info)
    start(name)
    out = fn(*args)
    stop(name)
    return out


def drop_last(name, k):
    """Forget the last k timed regions of `name` (launches a device flag made skip, e.g.
    Fisher products after CG converged, so averages cover launches that did the work)."""
    if _ENABLED and k > 0 and name in _events:
        del _events[name][-k:]


def summary():
    """{name: (count, mean_ms, total_ms)} -- synchronises."""
    torch.cuda.synchronize()
    out = {}
    for k, v in _events.items():
        ms = [a.elapsed_time(b) for a, b in v]
        out[k] = (len(ms), sum(ms) / max(len(ms), 1), sum(ms))
    return out
