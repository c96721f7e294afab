"""hipBLASLt kernel choice on the recurrences' GEMM shapes (dev tool): run under
rocprofv3 --kernel-trace to read the chosen kernels' names, grids and times; with
TENSILE_STREAMK_DATA_PARALLEL set the grids show whether stream-K splitting is off."""
import torch

M = 30720
for (K, N) in ((1024, 512), (1024, 4096), (512, 4096), (4096, 1024)):
    a = torch.randn(M, K, device='cuda', dtype=torch.bfloat16)
    b = torch.randn(K, N, device='cuda', dtype=torch.bfloat16)
    for _ in range(3):
        c = torch.mm(a, b, out_dtype=torch.float32)
# the W_ih gradient shape: dW (2048 x 1024) = dG^T (2048 x M) x (M x 1024)
g = torch.randn(M, 2048, device='cuda', dtype=torch.bfloat16)
x = torch.randn(M, 1024, device='cuda', dtype=torch.bfloat16)
for _ in range(3):
    w = torch.mm(g.t(), x, out_dtype=torch.float32)
torch.cuda.synchronize()
print("done")
