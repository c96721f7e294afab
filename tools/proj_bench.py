"""The SeparateF0 recurrences' input-projection and input-gradient GEMMs on bf16 operands
(dev tool): 128 x 128 tiles vs the 256 x 256 kernel (ensvs_set_big_tile 3), HIP events, with
torch's bf16 matmul (hipBLASLt) on the same M, N, K as a library anchor.
   python tools/proj_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib, kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def run(name, M, N, Ks, iters=30, T=1024):
    dev = torch.device("cuda")
    pb = K.PackedBuffer(_lib.DT_BF16)
    segs = []
    for Kc in Ks:
        w = torch.randn(N, Kc, device=dev) * 0.02
        ref = pb.add(w, N, Kc, 1, Kc, 1, 1)
        x = torch.randn(M, Kc, device=dev).to(torch.bfloat16)
        segs.append(K.Seg(x, Kc, Kc, ref, T))
    pb.finalize(dev)
    pb.repack()
    Y = torch.empty(M, N, device=dev)
    bias = torch.zeros(N, device=dev)
    out = dict(case=name, M=M, N=N, K=sum(Ks))
    flops = 2.0 * M * N * sum(Ks)
    for mode in (0, 2, 3):
        K.set_big_tile(mode)
        sec = timeit(lambda: K.gemm(segs, M // T, T, N, pb, Y, N, bias=bias), iters)
        out[f"mode{mode}_us"] = round(sec * 1e6, 1)
        out[f"mode{mode}_tflops"] = round(flops / sec / 1e12, 1)
    K.set_big_tile(2)
    a = torch.randn(M, sum(Ks), device=dev, dtype=torch.bfloat16)
    b = torch.randn(sum(Ks), N, device=dev, dtype=torch.bfloat16)
    sec = timeit(lambda: torch.matmul(a, b), iters)
    out["torch_us"] = round(sec * 1e6, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    _lib.load()
    M = 30 * 1024
    run("enc l0 proj 512->4096", M, 4096, [512])
    run("enc l1/2 proj 1024->4096", M, 4096, [1024])
    run("enc dgrad 2x2048->1024", M, 1024, [2048, 2048])
    run("dec proj 512->2048", M, 2048, [512])
    run("dec dgrad 2x1024->512", M, 512, [1024, 1024])
