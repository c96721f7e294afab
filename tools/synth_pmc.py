"""HBM traffic of one synthesis pass (bench.synth_rtf's 6-part ensemble case: timing models,
acoustic inference with the 100-step reverse diffusions, post-processing, uSFGAN), for
rocprofv3 --pmc passes: a warm-up pass, then one measured pass bracketed by marker kernels
(torch.cuda._sleep) so tools/step_pmc_sum.py sums FETCH_SIZE / WRITE_SIZE over its dispatches.
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o pmc -- python3 tools/synth_pmc.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

bench._imports()
import torch  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(20250321)
model = bench.configs.instantiate(bench.configs.multitrack_diffusion(num_speakers=4)).to(dev)


def mark():
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()


bench.SYNTH_MARK = mark
out = bench.synth_rtf(model, dev, reps=1, only="ensemble_6part")
print("passes 1", out["ensemble_6part"]["rtf"], flush=True)
