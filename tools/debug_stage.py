"""Stage-wise check of FFConvLSTM backward on GPU vs CPU autograd of the same stage."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import torch
import torch.nn.functional as F
from oracle import ensvs_oracle as O
from ensemble_svs_with_interactions_amd import configs, engine
from golden_util import load_case, full_shapes, rel
from gpu_util import build

engine.set_gemm_precision("fp32")
CFG = configs.multitrack_diffusion(num_speakers=4)
a, meta = load_case("ffconvlstm_mgc")
cfg = CFG["mgc_model"]["encoder"]
mod = build(cfg, full_shapes(), meta["prefix"])
mod.train()
x = torch.from_numpy(a["x"]).cuda()
B, T = x.shape[:2]
lens = a["lengths"].tolist()
ld = torch.tensor(lens, device="cuda")
spk = torch.from_numpy(a["spk"]).cuda().expand(B, T, -1)
out, st = mod._fwd([(x, x.shape[2], 0, x.shape[2])], B, T, ld, spk, spk.stride(0))
dout = torch.from_numpy(a["R"]).cuda().reshape(B * T, -1).contiguous()
P = {k: v.detach().cpu() for k, v in mod.state_dict().items()}
# --- LSTM stage: input a = conv stack output
a_in = st["csv"][2]["out"].detach().cpu().view(B, T, -1).requires_grad_()
y = O.bilstm(P, "", a_in, lens, 2)
o = F.linear(y, P["fc.weight"], P["fc.bias"])
(o * dout.cpu().view(B, T, -1)).sum().backward()
# GPU backward step by step
pk = mod._packs
H2 = 2 * mod.lstm.hidden_size
dy = torch.empty(B * T, H2, device="cuda")
from ensemble_svs_with_interactions_amd import layers as Ly
Ly.K.gemm([Ly.K.Seg(dout, 1 * mod.out_dim, mod.out_dim, pk["fc^T"], T)], B, T, H2, pk.bwd, dy, H2)
da = Ly.lstm_bwd(pk, mod.lstm, st["lsv"], dy, B, T, ld, "cuda")
torch.cuda.synchronize()
print("d(conv out) via LSTM:", rel(da.cpu().view(B, T, -1), a_in.grad), flush=True)
for b in range(B):
    print(" b", b, rel(da.cpu().view(B, T, -1)[b], a_in.grad[b]),
          "pad region max", da.cpu().view(B, T, -1)[b, lens[b]:].abs().max().item() if lens[b] < T else 0,
          "ref pad max", a_in.grad[b, lens[b]:].abs().max().item() if lens[b] < T else 0)
# --- BN3 stage
s3 = st["csv"][2]
y3 = s3["y"].detach().cpu().view(B, T, -1).transpose(1, 2).requires_grad_()
rm = P["conv.10.running_mean"].clone(); rv = P["conv.10.running_var"].clone()
z = F.relu(F.batch_norm(y3, rm, rv, P["conv.10.weight"], P["conv.10.bias"], True, 0.1, 1e-5))
(z.transpose(1, 2) * da.cpu().view(B, T, -1)).sum().backward()
C = y3.shape[1]
dy3 = torch.empty(B * T, C, device="cuda")
part = Ly.K.scratch(64 * 2 * C, "cuda", key="bn")
sums = torch.empty(2 * C, device="cuda")
dg = torch.zeros(C, device="cuda"); db = torch.zeros(C, device="cuda")
bn = mod.conv[10]
Ly.call("ensvs_bn_bwd", da.data_ptr(), C, s3["y"].data_ptr(), C, B * T, C, B * T, s3["mean"].data_ptr(),
        s3["rstd"].data_ptr(), bn.weight.data_ptr(), bn.bias.data_ptr(), part.data_ptr(), 64,
        sums.data_ptr(), dg.data_ptr(), db.data_ptr(), dy3.data_ptr(), C, Ly.stream())
torch.cuda.synchronize()
print("d y3 (BN bwd):", rel(dy3.cpu().view(B, T, -1), y3.grad.transpose(1, 2)))
mean_ref = y3.detach().mean((0, 2))
print("mean:", rel(s3["mean"].cpu().view(-1), mean_ref))
print("rstd:", rel(s3["rstd"].cpu().view(-1), 1 / torch.sqrt(y3.detach().var((0, 2), unbiased=False) + 1e-5)))
