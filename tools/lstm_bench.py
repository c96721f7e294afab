"""Time the LSTM recurrence kernels at the bench workload (30 sequences x 1024 frames,
synthetic lengths): us per launch and ns per recurrent step."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import data  # noqa: E402
from ensemble_svs_with_interactions_amd import _lib  # noqa: E402
from ensemble_svs_with_interactions_amd._lib import call  # noqa: E402

if len(sys.argv) > 1:  # A/B timing against another build of the library
    _lib.LIB_PATH = sys.argv[1]

B, T = 30, 1024
lengths = data.synthetic_batch(B, T, 1000)["lengths"].tolist()
dev = "cuda"
st = torch.cuda.current_stream().cuda_stream
lens = torch.tensor(lengths, dtype=torch.int64, device=dev)
for H in (8, 16, 64, 128, 62, 256, 512):
    gx = torch.randn(B * T, 8 * H, device=dev)
    w = [torch.randn(4 * H, H, device=dev) * 0.1 for _ in range(2)]
    y = torch.empty(B * T, 2 * H, device=dev)
    sv = torch.empty(B * T * 10 * H, device=dev)
    dy = torch.randn(B * T, 2 * H, device=dev)
    dg = torch.empty(B * T, 8 * H, device=dev)
    nw = _lib.query("ensvs_lstm_bwd_work_floats", B, H)
    work = torch.empty(max(nw, 1), device=dev)
    res = {}
    for name, fn in (("fwd", lambda: call("ensvs_lstm_fwd", gx.data_ptr(), 8 * H, w[0].data_ptr(),
                                           w[1].data_ptr(), lens.data_ptr(), B, T, H, y.data_ptr(),
                                           2 * H, sv.data_ptr(), st)),
                     ("bwd", lambda: call("ensvs_lstm_bwd", dy.data_ptr(), 2 * H, w[0].data_ptr(),
                                           w[1].data_ptr(), lens.data_ptr(), B, T, H, sv.data_ptr(),
                                           dg.data_ptr(), 8 * H, work.data_ptr(), nw, st))):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        res[name] = f"{us:8.1f} us ({us * 1e3 / max(lengths):6.0f} ns/step)"
    print(f"H={H:4d}  fwd {res['fwd']}  bwd {res['bwd']}", flush=True)
