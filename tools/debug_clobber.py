import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import torch
from ensemble_svs_with_interactions_amd import configs, engine, layers as Ly
from golden_util import load_case, full_shapes
from gpu_util import build

engine.set_gemm_precision("fp32")
CFG = configs.multitrack_diffusion(num_speakers=4)
a, meta = load_case("ffconvlstm_mgc")
mod = build(CFG["mgc_model"]["encoder"], full_shapes(), meta["prefix"])
mod.train()
x = torch.from_numpy(a["x"]).cuda()
B, T = x.shape[:2]
ld = torch.tensor(a["lengths"].tolist(), device="cuda")
spk = torch.from_numpy(a["spk"]).cuda().expand(B, T, -1)
out, st = mod._fwd([(x, x.shape[2], 0, x.shape[2])], B, T, ld, spk, spk.stride(0))
watch = {f"y{li}": st["csv"][li]["y"] for li in range(3)}
watch.update({f"out{li}": st["csv"][li]["out"] for li in range(3)})
watch.update({"X0": st["X0"], "h0": st["hs"][0], "h2": st["hs"][2], "ly": st["y"]})
snap = {k: v.clone() for k, v in watch.items()}
print({k: (v.data_ptr(), v.numel() * 4) for k, v in watch.items()})
orig_call = Ly.call
step = [0]
def traced(name, *args):
    orig_call(name, *args)
    torch.cuda.synchronize()
    for k, v in watch.items():
        if not torch.equal(v, snap[k]):
            print(f"after call #{step[0]} {name}: {k} CHANGED", flush=True)
            snap[k] = v.clone()
    step[0] += 1
import ensemble_svs_with_interactions_amd.kernels as K
Ly.call = traced
K.call = traced
dout = torch.from_numpy(a["R"]).cuda().reshape(B * T, -1).contiguous()
mod._bwd(st, dout)
torch.cuda.synchronize()
print("done", step[0], "calls")
