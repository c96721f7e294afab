"""Vendor-library reference for the training step's GEMM shapes (dev tool): torch.mm in bf16
(hipBLASLt) on the M = 30 720-frame shapes of the DiffNet / encoder GEMMs and their weight
gradients, timed with HIP events; prints TFLOP/s and the fraction of the 2.5 PFLOP/s dense
bf16 peak.  Run under rocprofv3 --kernel-trace --stats to see the library's tile configs.
    python tools/blas_ref.py"""
import torch

SHAPES = [  # (M, K, N, what)
    (30720, 1024, 512, "gate GEMM: dilated k3 256 + cond 256 -> 512"),
    (30720, 256, 512, "res/skip GEMM 256 -> 512"),
    (30720, 768, 256, "encoder k3 conv 256 -> 256"),
    (30720, 512, 256, "gate dgrad 512 -> 256"),
    (512, 30720, 1024, "gate wgrad (N x K over M frames)"),
    (512, 30720, 256, "res/skip wgrad"),
]
PEAK = 2.5e15


def main():
    dev = torch.device("cuda")
    for M, K, N, what in SHAPES:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for _ in range(5):
            torch.mm(a, b, out=c)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            torch.mm(a, b, out=c)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        tf = 2 * M * N * K / us / 1e6
        mb = (M * K + K * N + M * N) * 2 / 1e6
        print(f"M={M:6d} K={K:6d} N={N:5d} {us:7.1f} us {tf:7.0f} TF/s ({tf * 1e12 / PEAK:.2f} "
              f"of peak) {mb / us:5.2f} TB/s  {what}", flush=True)


if __name__ == "__main__":
    main()
