"""Weight repack of the bench model's 18 packed buffers (dev tool): the element-per-thread
pack_kernel vs the tiled pack_tile_kernel, HIP events over 20 passes.
   python tools/pack_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import configs, kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda")
    model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev)
    bufs = []
    for _, m in model.named_modules():
        if hasattr(m, "_packs") and hasattr(m, "_register"):
            pk = m._packs.ensure(m, m._register)
            bufs += [pb for pb in (pk.fwd, pk.bwd, pk.bias) if pb._n]
    elems = sum(pb.size for pb in bufs)
    out = dict(buffers=len(bufs), packed_elements=elems)
    for tiled in (False, True, False, True):
        K.PACK_TILED["on"] = tiled
        for pb in bufs:
            pb.repack()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            for pb in bufs:
                pb.repack()
        b.record()
        torch.cuda.synchronize()
        out["tiled_us" if tiled else "element_us"] = round(a.elapsed_time(b) / 20 * 1e3, 1)
    K.PACK_TILED["on"] = True
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
