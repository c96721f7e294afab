"""AR decoder recurrence timing on the GPU (dev tool): the exact per-sequence kernels vs the
cooperative ones at the recipe's H = 256, 30 sequences x 1024 frames (256 AR steps), HIP
events on the launch stream.  python tools/ardec_bench.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from ensemble_svs_with_interactions_amd._lib import call, query  # noqa: E402
from test_ardec_gpu import CONSTS, _inputs  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
H, B, T = 256, 30, 1024
Tr = T // 4
a = _inputs(B, T, H, 1)
st = torch.cuda.current_stream().cuda_stream
dev = "cuda"
E = lambda *s: torch.empty(s, device=dev)  # noqa: E731
o = dict(lf0=E(B * T), res=E(B * T), sg=E(B * Tr, 4 * H), sc=E(B * Tr, H), sh=E(B * Tr, H),
         so=E(B * Tr, 4), sp=E(B * Tr))
outs = tuple(o[k].data_ptr() for k in ("lf0", "res", "sg", "sc", "sh", "so", "sp"))
ins = (a["wih_p"].data_ptr(), a["wfo"].data_ptr(), H + 130, a["score"].data_ptr() + 4, 3,
       a["mask"].data_ptr(), None, 0, B, T, H, *CONSTS)
dg, do4 = E(B * Tr, 4 * H), E(B * Tr, 4)
bargs = (a["wih_p"].data_ptr(), a["wfo"].data_ptr(), H + 130, a["mask"].data_ptr(), 0, B, T, H,
         *CONSTS, o["sg"].data_ptr(), o["sc"].data_ptr(), o["so"].data_ptr(), dg.data_ptr(),
         do4.data_ptr())
wpf, wpb = E(4 * H * H), E(4 * H * H)
call("ensvs_ardec_pack", a["whh"].data_ptr(), H, wpf.data_ptr(), wpb.data_ptr(), st)
nbytes = 0  # the largest of the tile layouts the runs force
for S in (32, 16, 0):
    call("ensvs_ardec_coop_set_tile_seqs", S)
    nbytes = max(nbytes, query("ensvs_ardec_coop_work_bytes", H, B))
work = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
wf = torch.empty(4 * H * H, dtype=torch.float16, device=dev)
wb = torch.empty(4 * H * H, dtype=torch.bfloat16, device=dev)
call("ensvs_ardec_coop_pack", a["whh"].data_ptr(), H, 0, wf.data_ptr(), st)
call("ensvs_ardec_coop_pack", a["whh"].data_ptr(), H, 1, wb.data_ptr(), st)

runs = {
    "fwd_exact": lambda: call("ensvs_ardec_fwd", a["gx"].data_ptr(), 4 * H, a["ofx"].data_ptr(), 4,
                              wpf.data_ptr(), *ins, *outs, st),
    "bwd_exact": lambda: call("ensvs_ardec_bwd", a["glf0"].data_ptr(), a["gres"].data_ptr(),
                              wpb.data_ptr(), *bargs, st),
    "fwd_coop": lambda: call("ensvs_ardec_coop_fwd", a["gx"].data_ptr(), 4 * H, a["ofx"].data_ptr(),
                             4, wf.data_ptr(), *ins, *outs, work.data_ptr(), nbytes, st),
    "bwd_coop": lambda: call("ensvs_ardec_coop_bwd", a["glf0"].data_ptr(), a["gres"].data_ptr(),
                             wb.data_ptr(), *bargs, work.data_ptr(), nbytes, st),
}
line = []
runs = [(k, v, 0) for k, v in runs.items() if "exact" in k] + \
    [(f"{k}{S}", v, S) for S in (32, 16) for k, v in runs.items() if "coop" in k]
for name, fn, S in runs:
    call("ensvs_ardec_coop_set_tile_seqs", S)
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / iters
    line.append(f"{name} {us:9.1f} us ({us / Tr:5.2f} us/step)")
call("ensvs_ardec_coop_set_tile_seqs", 0)
err = work[128:132].cpu().view(torch.int32).item()
print(f"H={H} B={B} T={T}: " + "  ".join(line) + f"  err={err}", flush=True)
