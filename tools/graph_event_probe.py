"""Probe: can timing events be recorded inside a captured HIP graph and read after replay?

torch's Event.record() inside torch.cuda.graph capture fails on ROCm 7.2 (hipErrorInvalidHandle);
hipEventRecordWithFlags(ev, stream, hipEventRecordExternal) records an external event node instead.
"""
import ctypes as ct

import torch

hip = ct.CDLL("libamdhip64.so")
hip.hipEventCreate.argtypes = [ct.POINTER(ct.c_void_p)]
hip.hipEventRecordWithFlags.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_uint]
hip.hipEventElapsedTime.argtypes = [ct.POINTER(ct.c_float), ct.c_void_p, ct.c_void_p]
hip.hipEventSynchronize.argtypes = [ct.c_void_p]

x = torch.randn(1 << 24, device="cuda")
y = torch.empty_like(x)
evs = []
for _ in range(6):
    e = ct.c_void_p()
    assert hip.hipEventCreate(ct.byref(e)) == 0
    evs.append(e)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
rcs = []
with torch.cuda.graph(g):
    st = ct.c_void_p(torch.cuda.current_stream().cuda_stream)
    for i in range(3):
        rcs.append(hip.hipEventRecordWithFlags(evs[2 * i], st, 1))
        torch.mul(x, 2.0, out=y)
        rcs.append(hip.hipEventRecordWithFlags(evs[2 * i + 1], st, 1))
print("record rcs during capture:", rcs)
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
ms = []
for i in range(3):
    f = ct.c_float()
    rc = hip.hipEventElapsedTime(ct.byref(f), evs[2 * i], evs[2 * i + 1])
    ms.append((rc, f.value))
print("captured external events (rc, ms):", ms)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
torch.mul(x, 2.0, out=y)
e.record()
torch.cuda.synchronize()
print("eager ms:", s.elapsed_time(e))
