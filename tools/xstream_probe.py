"""Cross-stream dependency latency on this runtime: a ping-pong of tiny kernels between two
streams, each hop ordered either by an event (torch wait_stream: hipStreamWaitEvent) or by
a memory value (hipStreamWriteValue32 on the producer, hipStreamWaitValue32 on the
consumer).  Everything is enqueued behind a sleeping kernel first, so the host's issue rate
is not measured; time per hop = (elapsed - sleep) / hops."""
import ctypes

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipStreamWriteValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint]
hip.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint, ctypes.c_uint32]
GEQ = 0x0  # hipStreamWaitValueGte

N = 200
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
x = torch.zeros(1, device="cuda")
flag = torch.zeros(4, dtype=torch.int32, device="cuda")


def run(kind, sleep_cycles=200_000_000):
    torch.cuda.synchronize()
    flag.zero_()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s1):
        e0.record()
        torch.cuda._sleep(sleep_cycles)
    v = 0
    for i in range(N):
        with torch.cuda.stream(s1):
            x.add_(1.0)
            if kind == "event":
                pass
            else:
                v += 1
                assert hip.hipStreamWriteValue32(ctypes.c_void_p(s1.cuda_stream), ctypes.c_void_p(flag.data_ptr()),
                                                 v, 0) == 0
        if kind == "event":
            s2.wait_stream(s1)
        else:
            assert hip.hipStreamWaitValue32(ctypes.c_void_p(s2.cuda_stream), ctypes.c_void_p(flag.data_ptr()), v,
                                            GEQ, 0xFFFFFFFF) == 0
        with torch.cuda.stream(s2):
            x.add_(1.0)
            if kind != "event":
                v += 1
                assert hip.hipStreamWriteValue32(ctypes.c_void_p(s2.cuda_stream),
                                                 ctypes.c_void_p(flag.data_ptr() + 4), v, 0) == 0
        if kind == "event":
            s1.wait_stream(s2)
        else:
            assert hip.hipStreamWaitValue32(ctypes.c_void_p(s1.cuda_stream), ctypes.c_void_p(flag.data_ptr() + 4), v,
                                            GEQ, 0xFFFFFFFF) == 0
    with torch.cuda.stream(s1):
        e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def sleep_only(sleep_cycles=200_000_000):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s1):
        e0.record()
        torch.cuda._sleep(sleep_cycles)
        e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def same_stream():
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s1):
        e0.record()
        torch.cuda._sleep(200_000_000)
        for i in range(2 * N):
            x.add_(1.0)
        e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


run("event"), run("value")  # warm
base = sleep_only()
for rep in range(2):
    for kind in ("event", "value"):
        ms = run(kind)
        print(f"{kind:6s}: {(ms - base) * 1e3 / (2 * N):7.2f} us per hop (tiny kernel + cross-stream wait)", flush=True)
    ms = same_stream()
    print(f"same  : {(ms - base) * 1e3 / (2 * N):7.2f} us per tiny kernel, one stream", flush=True)
print("x =", float(x.item()))
