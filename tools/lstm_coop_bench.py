"""Time the large-H recurrences at the bench workload (30 sequences x 1024 frames, synthetic
lengths): the cooperative kernels (lstm_coop.hip) against the per-step kernels (lstm.hip),
us per launch and us per recurrent step, the cooperative kernels at both tile sizes (16 / 32
sequences per tile) (dev tool).   python tools/lstm_coop_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import data  # noqa: E402
from ensemble_svs_with_interactions_amd._lib import call, query  # noqa: E402

B, T = 30, 1024
lengths = data.synthetic_batch(B, T, 1000)["lengths"].tolist()
dev = "cuda"
st = torch.cuda.current_stream().cuda_stream
lens = torch.tensor(lengths, dtype=torch.int64, device=dev)


def timed(fn, n):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for H in (256, 512):
    gx = torch.randn(B * T, 8 * H, device=dev)
    w = [torch.randn(4 * H, H, device=dev) * (1.0 / H ** 0.5) for _ in range(2)]
    y = torch.empty(B * T, 2 * H, device=dev)
    sv = torch.empty(B * T * 10 * H, device=dev)
    dy = torch.randn(B * T, 2 * H, device=dev)
    dg = torch.empty(B * T, 8 * H, device=dev)
    nw = query("ensvs_lstm_bwd_work_floats", B, H)
    work = torch.empty(max(nw, 1), device=dev)
    call("ensvs_lstm_coop_set_tile_seqs", 32)
    nb = query("ensvs_lstm_coop_work_bytes", H, B)  # the larger of the two layouts
    call("ensvs_lstm_coop_set_tile_seqs", 0)
    nb = max(nb, query("ensvs_lstm_coop_work_bytes", H, B))
    cw = torch.empty(nb, dtype=torch.uint8, device=dev)
    wpf = torch.empty(2 * 4 * H * H, dtype=torch.float16, device=dev)
    wpb = torch.empty(2 * 4 * H * H, dtype=torch.bfloat16, device=dev)
    call("ensvs_lstm_coop_pack", w[0].data_ptr(), w[1].data_ptr(), H, 0, wpf.data_ptr(), st)
    call("ensvs_lstm_coop_pack", w[0].data_ptr(), w[1].data_ptr(), H, 1, wpb.data_ptr(), st)
    res = {}
    res["fwd_step"] = timed(lambda: call("ensvs_lstm_fwd", gx.data_ptr(), 8 * H, w[0].data_ptr(),
                                         w[1].data_ptr(), lens.data_ptr(), B, T, H, y.data_ptr(),
                                         2 * H, sv.data_ptr(), st), 2)
    res["bwd_step"] = timed(lambda: call("ensvs_lstm_bwd", dy.data_ptr(), 2 * H, w[0].data_ptr(),
                                         w[1].data_ptr(), lens.data_ptr(), B, T, H, sv.data_ptr(),
                                         dg.data_ptr(), 8 * H, work.data_ptr(), nw, st), 2)
    for S in (32, 16):
        call("ensvs_lstm_coop_set_tile_seqs", S)
        res[f"fwd_coop{S}"] = timed(lambda: call("ensvs_lstm_coop_fwd", gx.data_ptr(), 8 * H, wpf.data_ptr(),
                                             lens.data_ptr(), B, T, H, y.data_ptr(), 2 * H, sv.data_ptr(),
                                             cw.data_ptr(), nb, st), 5)
        res[f"bwd_coop{S}"] = timed(lambda: call("ensvs_lstm_coop_bwd", dy.data_ptr(), 2 * H, wpb.data_ptr(),
                                             lens.data_ptr(), B, T, H, sv.data_ptr(), dg.data_ptr(),
                                             8 * H, cw.data_ptr(), nb, st), 5)
    call("ensvs_lstm_coop_set_tile_seqs", 0)
    err = cw[128:132].cpu().view(torch.int32).item()
    steps = max(lengths)
    print(f"H={H:4d} " + "  ".join(f"{k} {v:9.1f} us ({v / steps:6.2f} us/step)"
                                    for k, v in res.items()) + f"  err={err}", flush=True)
