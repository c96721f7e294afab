"""Dev probe: device write / copy rates at the GEMM output sizes (63 MB fp32)."""
import torch
x = torch.empty(30720, 512, device="cuda")
y = torch.empty(30720, 512, device="cuda")


def timed(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for name, fn, b in [("fill 63 MB", lambda: x.fill_(1.0), x.numel() * 4),
                    ("zero 63 MB", lambda: x.zero_(), x.numel() * 4),
                    ("copy 63+63 MB", lambda: y.copy_(x), 2 * x.numel() * 4)]:
    t = timed(fn)
    print(f"{name:16s} {t:7.1f} us  {b / t / 1e6:6.2f} TB/s")
