"""MFMA recurrences (lstm_mfma.hip) vs the exact fp32 persistent kernels (lstm.hip) at the bench
workload (30 sequences x 1024 frames, synthetic lengths), HIP events: us per launch and ns per
recurrent step.  python tools/lstm_mfma_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import data  # noqa: E402
from ensemble_svs_with_interactions_amd import _lib  # noqa: E402
from ensemble_svs_with_interactions_amd._lib import call  # noqa: E402

B, T = 30, 1024
lengths = data.synthetic_batch(B, T, 1000)["lengths"].tolist()
dev = "cuda"
st = torch.cuda.current_stream().cuda_stream
lens = torch.tensor(lengths, dtype=torch.int64, device=dev)


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for H in (64, 128):
    gx = torch.randn(B * T, 8 * H, device=dev)
    w = [torch.randn(4 * H, H, device=dev) * 0.1 for _ in range(2)]
    y = torch.empty(B * T, 2 * H, device=dev)
    sv = torch.empty(B * T * 10 * H, device=dev)
    dy = torch.randn(B * T, 2 * H, device=dev)
    dg = torch.empty(B * T, 8 * H, device=dev)
    nw = _lib.query("ensvs_lstm_bwd_work_floats", B, H)
    work = torch.empty(max(nw, 1), device=dev)
    wpf = torch.empty(2 * 4 * H * H, dtype=torch.float16, device=dev)
    wpb = torch.empty(2 * 4 * H * H, dtype=torch.bfloat16, device=dev)
    call("ensvs_lstm_mfma_pack", w[0].data_ptr(), w[1].data_ptr(), H, 0, wpf.data_ptr(), st)
    call("ensvs_lstm_mfma_pack", w[0].data_ptr(), w[1].data_ptr(), H, 1, wpb.data_ptr(), st)
    runs = {
        "exact": (lambda: call("ensvs_lstm_fwd", gx.data_ptr(), 8 * H, w[0].data_ptr(),
                               w[1].data_ptr(), lens.data_ptr(), B, T, H, y.data_ptr(), 2 * H,
                               sv.data_ptr(), st),
                  lambda: call("ensvs_lstm_bwd", dy.data_ptr(), 2 * H, w[0].data_ptr(),
                               w[1].data_ptr(), lens.data_ptr(), B, T, H, sv.data_ptr(),
                               dg.data_ptr(), 8 * H, work.data_ptr(), nw, st)),
        "mfma": (lambda: call("ensvs_lstm_mfma_fwd", gx.data_ptr(), 8 * H, wpf.data_ptr(),
                              lens.data_ptr(), B, T, H, y.data_ptr(), 2 * H, sv.data_ptr(), None,
                              0, st),
                 lambda: call("ensvs_lstm_mfma_bwd", dy.data_ptr(), 2 * H, wpb.data_ptr(),
                              lens.data_ptr(), B, T, H, sv.data_ptr(), dg.data_ptr(), 8 * H,
                              None, 0, None, st)),
    }
    for name, (f, b) in runs.items():
        uf, ub = timeit(f), timeit(b)
        steps = max(lengths)
        print(f"H={H:4d} {name:5s}  fwd {uf:8.1f} us ({uf * 1e3 / steps:5.0f} ns/step)  "
              f"bwd {ub:8.1f} us ({ub * 1e3 / steps:5.0f} ns/step)", flush=True)
