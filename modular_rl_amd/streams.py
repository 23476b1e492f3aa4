"""CU-masked HIP streams (mrl_stream_create_cu_mask) wrapped as torch streams.

Used by the pipelined training loop: the rollout of iteration k+1 (a chain of
latency-bound step launches that occupy one block per CU on E/64 CUs) runs on one
CU set while the value-function fit of iteration k runs on the complementary set.
"""
import atexit
import ctypes

import torch

from . import _lib
from ._lib import call


def cu_count():
    n = ctypes.c_int32(0)
    call("mrl_device_cu_count", ctypes.byref(n))
    return int(n.value)


_created = []  # raw handles of the streams made here, destroyed at interpreter exit


def destroy_all():
    """Destroy every CU-masked stream (after draining the device).  Runs at interpreter
    exit: a stream left to the HIP runtime's own teardown is destroyed after an
    attached profiler (rocprofv3) has finalised, and that crashed the process."""
    if not _created:
        return
    torch.cuda.synchronize()
    _by_cus.clear()
    while _created:
        call("mrl_stream_destroy", ctypes.c_void_p(_created.pop()))


atexit.register(destroy_all)


_by_cus = {}  # (device, CU ids) -> stream: one hardware-queue-backed stream per CU set per process


def masked_stream(cus):
    """The HIP stream restricted to the CU ids in ``cus`` (torch.cuda.ExternalStream),
    created once per (device, CU set) and reused: every IterationRunner asks for the
    same two sets, and the box gives a process few hardware queues.  The stream lives
    until destroy_all() (at the latest, interpreter exit)."""
    key = (torch.cuda.current_device(), tuple(sorted(cus)))
    if key in _by_cus:
        return _by_cus[key]
    _lib.load(require_gpu=True)
    n = cu_count()
    words = (n + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in cus:
        if not 0 <= c < n:
            raise _lib.MrlError(f"CU id {c} out of range [0, {n})")
        mask[c // 32] |= 1 << (c % 32)
    out = ctypes.c_void_p()
    call("mrl_stream_create_cu_mask", mask, words, ctypes.byref(out))
    _created.append(out.value)
    _by_cus[key] = torch.cuda.ExternalStream(out.value)
    return _by_cus[key]


def stream_cus(s):
    """The CU ids a stream may use (hipExtStreamGetCUMask)."""
    n = cu_count()
    words = (n + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    call("mrl_stream_get_cu_mask", ctypes.c_void_p(s.cuda_stream), words, mask)
    return [i for i in range(n) if (mask[i // 32] >> (i % 32)) & 1]


def launch_cus(s=None):
    """CUs a launch on stream ``s`` (default: the current stream) may use: the CU set of
    a stream made by masked_stream, else the whole device."""
    s = torch.cuda.current_stream() if s is None else s
    for (dev, cus), st in _by_cus.items():
        if st.cuda_stream == s.cuda_stream:
            return len(cus)
    return cu_count()


class ValueOrder:
    """Cross-stream ordering on a memory value instead of an event (tools/xstream_probe.py:
    a hop ordered by hipStreamWaitValue32 costs 5.6 us against 15.7 with
    hipStreamWaitEvent).  One int32 slot per producer stream, written by that stream only
    with increasing values; order(producer, consumer) enqueues the producer's write and
    then the consumer's wait, so the awaited value is always on its way."""

    def __init__(self, device="cuda"):
        self.flags = torch.zeros(8, dtype=torch.int32, device=device)
        torch.cuda.synchronize()  # the zeros are in place before any stream waits on them
        self.slot = {}
        self.value = {}

    def order(self, producer, consumer):
        key = producer.cuda_stream
        if key not in self.slot:
            if len(self.slot) >= self.flags.numel():
                raise _lib.MrlError("ValueOrder: too many producer streams")
            self.slot[key] = len(self.slot)
            self.value[key] = 0
        self.value[key] += 1
        v = self.value[key]
        addr = ctypes.c_void_p(self.flags.data_ptr() + 4 * self.slot[key])
        call("mrl_stream_signal", ctypes.c_void_p(producer.cuda_stream), addr, v)
        call("mrl_stream_wait", ctypes.c_void_p(consumer.cuda_stream), addr, v)
