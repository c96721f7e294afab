import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import torch
import torch.nn.functional as F
from ensemble_svs_with_interactions_amd import configs, engine, layers as Ly
from golden_util import load_case, full_shapes, rel
from gpu_util import build

engine.set_gemm_precision("fp32")
CFG = configs.multitrack_diffusion(num_speakers=4)
a, meta = load_case("ffconvlstm_mgc")
mod = build(CFG["mgc_model"]["encoder"], full_shapes(), meta["prefix"])
mod.train()
x = torch.from_numpy(a["x"]).cuda()
B, T = x.shape[:2]
lens = a["lengths"].tolist()
ld = torch.tensor(lens, device="cuda")
spk = torch.from_numpy(a["spk"]).cuda().expand(B, T, -1)
out, st = mod._fwd([(x, x.shape[2], 0, x.shape[2])], B, T, ld, spk, spk.stride(0))
dout = torch.from_numpy(a["R"]).cuda().reshape(B * T, -1).contiguous()
Ly.DEBUG = {}
mod._bwd(st, dout)
torch.cuda.synchronize()
D = Ly.DEBUG
P = {k: v.detach().cpu() for k, v in mod.state_dict().items()}
for li, (ci, bi) in enumerate(Ly.CONV_IDX):
    s = st["csv"][li]
    C = s["y"].shape[1]
    y = s["y"].cpu().view(B, T, C).transpose(1, 2).clone().requires_grad_()
    g = P[f"conv.{bi}.weight"].clone().requires_grad_()
    bb = P[f"conv.{bi}.bias"].clone().requires_grad_()
    z = F.relu(F.batch_norm(y, None, None, g, bb, True, 0.1, 1e-5))
    (z.transpose(1, 2) * D[f"conv{li}.dout"].cpu().view(B, T, C)).sum().backward()
    print(f"BN{li}: dy {rel(D[f'conv{li}.dy'].cpu().view(B, T, C), y.grad.transpose(1, 2)):.2e}")
    # conv weight grad from this layer's input
    xin = (st["csv"][li - 1]["out"] if li > 0 else st["hs"][2]).cpu().view(B, T, -1)
    xin_p = F.pad(xin.transpose(1, 2), (3, 3), mode="reflect")
    w = P[f"conv.{ci}.weight"].clone().requires_grad_()
    F.conv1d(xin_p, w).backward(D[f"conv{li}.dy"].cpu().view(B, T, C).transpose(1, 2))
    print(f"conv{ci} wgrad {rel(mod.conv[ci].weight.grad.cpu(), w.grad):.2e}")
    if li > 0:
        xr = xin.clone().requires_grad_()
        F.conv1d(F.pad(xr.transpose(1, 2), (3, 3), mode="reflect"), P[f"conv.{ci}.weight"]).backward(
            D[f"conv{li}.dy"].cpu().view(B, T, C).transpose(1, 2))
        print(f"conv{ci} dgrad {rel(D[f'conv{li-1}.dout'].cpu().view(B, T, -1), xr.grad):.2e}")
