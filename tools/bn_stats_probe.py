"""ensvs_bn_stats at the encoders' BatchNorm shapes (dev tool): 50 calls per shape, for a
rocprofv3 --kernel-trace --stats run (partial / final kernel durations standalone).
   python tools/bn_stats_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib  # noqa: E402
from ensemble_svs_with_interactions_amd._lib import call, query  # noqa: E402


def main():
    _lib.load()
    dev = torch.device("cuda")
    s = torch.cuda.current_stream().cuda_stream
    for M, C in ((30720, 512), (30720, 256), (30720, 128)):
        y = torch.randn(M, C, device=dev)
        n = query("ensvs_bn_stats_part_floats", M, C, M)
        part = torch.empty(n, device=dev)
        mean, var, rstd = (torch.empty(C, device=dev) for _ in range(3))
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros(1, dtype=torch.int64, device=dev)
        for _ in range(50):
            call("ensvs_bn_stats", y.data_ptr(), C, M, C, M, part.data_ptr(), n, 1e-5,
                 mean.data_ptr(), var.data_ptr(), rstd.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                 0.1, 1, nbt.data_ptr(), s)
        torch.cuda.synchronize()
        print(M, C, "ok", flush=True)


if __name__ == "__main__":
    main()
