"""Dump the MFMA LSTM recurrences' outputs (H = 64 / 128, fwd + bwd, 30 x 1024 ragged, fixed
seeds) for a bitwise comparison of two library builds (dev tool):
  ENSVS_LIB=ab/libensvs_HEAD.so python tools/lstm_mfma_dump.py gpurun_out/a.pt
  python tools/lstm_mfma_dump.py gpurun_out/b.pt
  python tools/lstm_mfma_dump.py --compare gpurun_out/a.pt gpurun_out/b.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if sys.argv[1] == "--compare":
    a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
    bad = [k for k in a if not torch.equal(a[k].view(torch.int16 if a[k].dtype == torch.bfloat16
                                                      else torch.int32),
                                         b[k].view(torch.int16 if b[k].dtype == torch.bfloat16
                                                   else torch.int32))]
    print("bitwise equal" if not bad else f"DIFFER: {bad}", f"({len(a)} tensors)")
    sys.exit(1 if bad else 0)

from ensemble_svs_with_interactions_amd._lib import call  # noqa: E402

dev = "cuda"
st = torch.cuda.current_stream().cuda_stream
B, T = 30, 1024
g = torch.Generator().manual_seed(5)
lengths = [T] + torch.randint(1, T + 1, (B - 1,), generator=g).tolist()
lens = torch.tensor(lengths, dtype=torch.int64, device=dev)
res = {}
for H in (64, 128):
    gg = torch.Generator(device=dev).manual_seed(H)
    gx = torch.randn(B * T, 8 * H, device=dev, generator=gg) * 0.5
    w = [(torch.rand(4 * H, H, device=dev, generator=gg) * 2 - 1) * H ** -0.5 for _ in range(2)]
    gy = torch.randn(B * T, 2 * H, device=dev, generator=gg)
    wpf = torch.empty(2 * 4 * H * H, dtype=torch.float16, device=dev)
    wpb = torch.empty(2 * 4 * H * H, dtype=torch.bfloat16, device=dev)
    call("ensvs_lstm_mfma_pack", w[0].data_ptr(), w[1].data_ptr(), H, 0, wpf.data_ptr(), st)
    call("ensvs_lstm_mfma_pack", w[0].data_ptr(), w[1].data_ptr(), H, 1, wpb.data_ptr(), st)
    z = lambda *s, dt=torch.float32: torch.zeros(s, device=dev, dtype=dt)  # noqa: E731
    y, yb, sv = z(B * T, 2 * H), z(B * T, 2 * H, dt=torch.bfloat16), z(B * T * 10 * H)
    dg, dgb, bs = z(B * T, 8 * H), z(B * T, 8 * H, dt=torch.bfloat16), z(B, 8 * H)
    call("ensvs_lstm_mfma_fwd", gx.data_ptr(), 8 * H, wpf.data_ptr(), lens.data_ptr(), B, T, H,
         y.data_ptr(), 2 * H, sv.data_ptr(), yb.data_ptr(), 2 * H, st)
    call("ensvs_lstm_mfma_bwd", gy.data_ptr(), 2 * H, wpb.data_ptr(), lens.data_ptr(), B, T, H,
         sv.data_ptr(), dg.data_ptr(), 8 * H, None, 0, None, st)
    call("ensvs_lstm_mfma_bwd", gy.data_ptr(), 2 * H, wpb.data_ptr(), lens.data_ptr(), B, T, H,
         sv.data_ptr(), None, 0, dgb.data_ptr(), 8 * H, bs.data_ptr(), st)
    torch.cuda.synchronize()
    for k, v in (("y", y), ("yb", yb), ("sv", sv), ("dg", dg), ("dgb", dgb), ("bsum", bs)):
        res[f"H{H}.{k}"] = v.cpu()
torch.save(res, sys.argv[1])
print("saved", sys.argv[1])
