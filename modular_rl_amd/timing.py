"""Optional HIP-event timing of named launch regions on the current stream.

Disabled by default (zero cost); bench.py enables it to measure the average
device duration of the dominant kernels live inside the timed region.

Every recorded event is a marker packet in the stream's queue, and the kernel after it
starts ≈6 µs later (rocprofv3: the CG loop's launches run back to back untimed, 6 µs apart
with a region around each product).  Regions marked ``detail`` (the many per-iteration
launches: Fisher products, VJPs, layered GEMMs, the GAE scan) are therefore recorded only
on every ``detail_every``-th iteration (``tick()`` once per iteration), and summary()
scales their totals to all iterations; the rollout's region every iteration.
"""
import collections

import torch

_ENABLED = False
_open = {}
_events = collections.defaultdict(list)
_detail_names = set()
_every = 1
_iters = 0          # tick() calls since enable(): the iterations of the measurement
_detail_iters = 0   # of them, the ones detail regions were recorded in
meta = {}  # name -> per-launch algorithmic work of the region (e.g. a GEMM's FLOP / bytes)


def enable(on=True, detail_every=1):
    global _ENABLED, _every, _iters, _detail_iters
    _ENABLED = on
    _open.clear()
    if on:  # a new measurement; turning timing off keeps the last one's records readable
        _events.clear()
        _detail_names.clear()
        meta.clear()
        _every = max(1, int(detail_every))
        _iters = _detail_iters = 0


def enabled():
    return _ENABLED


def tick():
    """One iteration of the measurement begins (detail regions: every _every-th)."""
    global _iters, _detail_iters
    if _ENABLED:
        _iters += 1
        if (_iters - 1) % _every == 0:
            _detail_iters += 1


def _detail_now():
    return _iters == 0 or (_iters - 1) % _every == 0


def detail_now():
    """Timing is on and this iteration records detail regions."""
    return _ENABLED and _detail_now()


def start(name, detail=False):
    if _ENABLED and (not detail or _detail_now()):
        if detail:
            _detail_names.add(name)
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        _open[name] = e


def stop(name):
    if _ENABLED and name in _open:
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        _events[name].append((_open.pop(name), e))


def region(name, fn, *args, **info):
    """fn(*args) timed as one detail region `name` (when enabled and sampled), with the
    region's per-launch work recorded in ``meta[name]``."""
    if not (_ENABLED and _detail_now()):
        return fn(*args)
    meta.setdefault(name, info)
    start(name, detail=True)
    out = fn(*args)
    stop(name)
    return out


def drop_last(name, k):
    """Forget the last k timed regions of `name` (launches a device flag made skip, e.g.
    Fisher products after CG converged, so averages cover launches that did the work) --
    when this iteration recorded them (a detail region of an unsampled iteration did not)."""
    if _ENABLED and k > 0 and name in _events and (name not in _detail_names or _detail_now()):
        del _events[name][-k:]


def summary():
    """{name: (count, mean_ms, total_ms)} -- synchronises.  count: the launches timed;
    total_ms: over all iterations of the measurement (a detail region's sampled total
    scaled by iterations / sampled iterations)."""
    torch.cuda.synchronize()
    out = {}
    for k, v in _events.items():
        ms = [a.elapsed_time(b) for a, b in v]
        tot = sum(ms)
        if k in _detail_names and _detail_iters > 0:
            tot *= _iters / _detail_iters
        out[k] = (len(ms), sum(ms) / max(len(ms), 1), tot)
    return out
