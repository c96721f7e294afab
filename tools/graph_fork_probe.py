"""HIP-graph capture of nested stream forks (dev probe).

A branch stream S1 forked from the capturing stream forks an auxiliary stream S3 mid-way
(event record on S1, wait on S3).  Variants differ only in where S3 is joined:
  parent: S1 waits S3, then the capturing stream waits S1
  main:   the capturing stream waits S1 and S3 directly
  pool:   as `main`, with S3 allocating tensors inside the capture
Each variant runs in its own process (python tools/graph_fork_probe.py <variant>) and
prints capture / replay status and whether the replayed result matches eager.
"""
import subprocess
import sys

import torch


def body(variant, x, streams):
    main = torch.cuda.current_stream()
    s1, s2, s3 = streams
    ev = main.record_event()
    s1.wait_event(ev)
    s2.wait_event(ev)
    with torch.cuda.stream(s1):
        a = x * 2.0
        e1 = s1.record_event()
        s3.wait_event(e1)
        with torch.cuda.stream(s3):
            b = a + 1.0 if variant != "pool" else (a + 1.0).clone()
        c = a * 3.0
    with torch.cuda.stream(s2):
        d = x - 1.0
    if variant == "parent":
        print("  parent: s1.wait_stream(s3)", flush=True)
        s1.wait_stream(s3)
        print("  parent: main.wait_stream(s1)", flush=True)
        main.wait_stream(s1)
        print("  parent: joined", flush=True)
    else:
        main.wait_stream(s1)
        main.wait_stream(s3)
    main.wait_stream(s2)
    return b + c + d


def run(variant):
    torch.cuda.init()
    dev = torch.device("cuda")
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    x = torch.randn(1 << 16, device=dev)
    ref = body(variant, x, streams)
    torch.cuda.synchronize()
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                out = body(variant, x, streams)
                print(f"{variant}: body captured, ending capture", flush=True)
        torch.cuda.current_stream().wait_stream(side)
        print(f"{variant}: capture ok", flush=True)
    except Exception as e:  # report the failing call
        print(f"{variant}: capture FAILED: {type(e).__name__}: {e}", flush=True)
        return 1
    g.replay()
    torch.cuda.synchronize()
    print(f"{variant}: replay {'matches' if torch.equal(out, ref) else 'DIFFERS'}", flush=True)
    return 0


if __name__ == "__main__":
    if len(sys.argv) > 1:
        sys.exit(run(sys.argv[1]))
    rc = 0
    for v in ("main", "pool", "parent"):
        r = subprocess.run([sys.executable, __file__, v], timeout=120)
        print(f"{v}: exit {r.returncode}", flush=True)
        rc |= r.returncode != 0
    sys.exit(rc)
