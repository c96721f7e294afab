import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import torch
import torch.nn.functional as F
from oracle import ensvs_oracle as O
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
P = {k: v.detach().cpu().clone() for k, v in mod.state_dict().items()}
out, st = mod._fwd([(x, x.shape[2], 0, x.shape[2])], B, T, ld, spk, spk.stride(0))
dout = torch.from_numpy(a["R"]).cuda().reshape(B * T, -1).contiguous()
Ly.DEBUG = {}
mod._bwd(st, dout)
torch.cuda.synchronize()
D = Ly.DEBUG
# oracle with retained intermediates
Pg = {k: v.clone().requires_grad_() for k, v in P.items() if v.dtype == torch.float32}
xc = torch.from_numpy(a["x"])
X0 = O.phoneme_embed(Pg, "", xc, 3, 50) + torch.from_numpy(a["spk"])
h = X0
for i in (0, 2, 4):
    h = F.relu(F.linear(h, Pg[f"ff.{i}.weight"], Pg[f"ff.{i}.bias"]))
hh = h.transpose(1, 2)
acts = []
pre = []
for li, (ci, bi) in enumerate(Ly.CONV_IDX):
    hh = F.conv1d(F.pad(hh, (3, 3), mode="reflect"), Pg[f"conv.{ci}.weight"], Pg[f"conv.{ci}.bias"])
    hh.retain_grad()
    pre.append(hh)
    hh = F.relu(F.batch_norm(hh, None, None, Pg[f"conv.{bi}.weight"], Pg[f"conv.{bi}.bias"], True))
    hh.retain_grad()
    acts.append(hh)
y = O.bilstm(Pg, "", hh.transpose(1, 2), lens, 2)
o = F.linear(y, Pg["fc.weight"], Pg["fc.bias"])
(o * torch.from_numpy(a["R"])).sum().backward()
for li in (2, 1, 0):
    if f"conv{li}.dout" in D:
        print(f"d(act{li}) {rel(D[f'conv{li}.dout'].cpu().view(B, T, -1), acts[li].grad.transpose(1, 2)):.2e}")
for li in (2, 1, 0):
    print(f"d(pre{li}) {rel(D[f'conv{li}.dy'].cpu().view(B, T, -1), pre[li].grad.transpose(1, 2)):.2e}")
    yg = st["csv"][li]["y"].cpu().view(B, T, -1).transpose(1, 2).clone().requires_grad_()
    z = F.relu(F.batch_norm(yg, None, None, P[f"conv.{Ly.CONV_IDX[li][1]}.weight"], P[f"conv.{Ly.CONV_IDX[li][1]}.bias"], True))
    z.backward(acts[li].grad)
    print(f"   cpu-bn(gpu y, oracle dact) vs oracle dpre {rel(yg.grad, pre[li].grad):.2e}  |dpre|={pre[li].grad.abs().max():.3e} |dact|={acts[li].grad.abs().max():.3e}")
for k, p in mod.named_parameters():
    g = p.grad.cpu()
    print(f"{k:32s} {rel(g, Pg[k].grad):.2e}")
