"""Minimal HIP-graph capture with a nested stream fork (dev tool)."""
import sys

import torch

mode = sys.argv[1] if len(sys.argv) > 1 else "nested"
dev = torch.device("cuda")
A = torch.cuda.Stream(dev)
B = torch.cuda.Stream(dev)
C = torch.cuda.Stream(dev)
x = torch.randn(1 << 20, device=dev)


def body():
    cur = torch.cuda.current_stream(dev)
    B.wait_stream(cur)
    if mode in ("prefork", "prefork2"):
        C.wait_stream(cur)
    with torch.cuda.stream(B):
        y = x * 2
        if mode in ("nested", "prefork", "prefork2", "nojoin"):
            C.wait_event(B.record_event())
            with torch.cuda.stream(C):
                z = y + 1
            y = y * 3
            if mode in ("nested", "prefork"):
                B.wait_stream(C)
        else:
            z = y + 1
    cur.wait_stream(B)
    if mode in ("prefork", "prefork2", "nojoin"):
        cur.wait_stream(C)
    return y, z


body()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    out = body()
g.replay()
torch.cuda.synchronize()
print(mode, "ok", out[0][:2].tolist(), flush=True)
