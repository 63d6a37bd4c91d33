"""Probe: can timing events be recorded inside a captured HIP graph and read after replay?"""
import torch

x = torch.randn(1 << 24, device="cuda")
y = torch.empty_like(x)
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(g):
        for s, e in evs:
            s.record()
            torch.mul(x, 2.0, out=y)
            e.record()
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    print("captured-events ms:", [s.elapsed_time(e) for s, e in evs])
except Exception as ex:
    print("capture with events failed:", repr(ex))
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
torch.mul(x, 2.0, out=y)
e.record()
torch.cuda.synchronize()
print("eager ms:", s.elapsed_time(e))
