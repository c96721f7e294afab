"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU (PyTorch fp32) restatement of the multi-track timing models of
sarulab-speech/ensemble_svs_with_interactions: the MDN
layer / loss / most-probable selection (nnsvs/mdn.py), the plain MDN duration model
(nnsvs/model.py:538-618, BASELINE config 1) and MultiTrackVariancePredictor
(nnsvs/model.py:1180-1346).  It is the checker for the HIP timing path; only tests/ may
import it.

Parity is PINNED by tests/golden/mdn.npz and variance_predictor.npz, produced by the
reference itself (tests/golden/gen_goldens.py, cases "mdn" / "vp"), which also hold the
reference's own fixture weights tests/data/mdn_test.pth (loaded with weights_only=True).
"""
import torch
import torch.nn.functional as F


def mdn_layer(P, pre, x, G, D, dim_wise):
    """MDNLayer.forward (mdn.py:45-75)."""
    B = x.shape[0]
    lp = F.linear(x, P[pre + "log_pi.weight"], P[pre + "log_pi.bias"])
    if dim_wise:
        lp = F.log_softmax(lp.view(B, -1, G, D), dim=2)
    else:
        lp = F.log_softmax(lp, dim=2)
    ls = F.linear(x, P[pre + "log_sigma.weight"], P[pre + "log_sigma.bias"]).view(B, -1, G, D)
    mu = F.linear(x, P[pre + "mu.weight"], P[pre + "mu.bias"]).view(B, -1, G, D)
    return lp, ls, mu


def mdn_loss(log_pi, log_sigma, mu, target, log_pi_min=-7.0, log_sigma_min=-7.0, reduce=True):
    """mdn_loss (mdn.py:78-154): clamps, +-5 sigma clip of the centred target, Normal
    log-prob, -logsumexp over the mixture axis."""
    dim_wise = log_pi.dim() == 4
    log_sigma = torch.clamp(log_sigma, min=log_sigma_min)
    log_pi = torch.clamp(log_pi, min=log_pi_min)
    target = target.unsqueeze(2).expand_as(log_sigma)
    c = target - mu
    scale = torch.exp(log_sigma)
    edge = 5 * scale
    c = torch.where(c > edge, edge, c)
    c = torch.where(c < -edge, -edge, c)
    lp = torch.distributions.Normal(loc=0, scale=scale).log_prob(c)
    loss = lp + log_pi if dim_wise else lp.sum(dim=3) + log_pi
    loss = -torch.logsumexp(loss, dim=2)
    return loss.mean(dim=1) if reduce else loss


def mdn_most_probable(log_pi, log_sigma, mu):
    """mdn_get_most_probable_sigma_and_mu (mdn.py:167-212): the component of largest
    log_pi (first maximum), its sigma = exp(log_sigma) and mu."""
    dim_wise = log_pi.dim() == 4
    G = mu.shape[2]
    k = torch.max(log_pi, dim=2)[1]
    oh = F.one_hot(k, G).float()
    oh = oh.transpose(2, 3) if dim_wise else oh.unsqueeze(3).expand_as(mu)
    return torch.exp(torch.sum(log_sigma * oh, dim=2)), torch.sum(mu * oh, dim=2)


def mdn_model(P, x, num_layers, G, D, dim_wise=False):
    """nnsvs.model.MDN.forward (model.py:556-602): (Linear + ReLU) x num_layers + MDNLayer."""
    h = x
    for i in range(num_layers):
        h = F.relu(F.linear(h, P[f"model.{2 * i}.weight"], P[f"model.{2 * i}.bias"]))
    return mdn_layer(P, f"model.{2 * num_layers}.", h, G, D, dim_wise)


def variance_predictor(P, cfg, x, spks, dropout_masks=None):
    """MultiTrackVariancePredictor.forward (model.py:1277-1327) without phoneme embedding
    (the recipe: embed_dim None).  x = concat(x0, x1) (B, T, 2*in_dim); spks (spk0, spk1)
    (B, 1) ids.  dropout_masks: per layer scaled keep masks (B, T, hidden) or None (eval)."""
    if cfg.get("mask_indices"):
        x = x.clone()
        for idx in cfg["mask_indices"]:
            x[:, :, idx] *= 0.0
    emb = P["speaker_emb.weight"]
    s0 = F.embedding(spks[0], emb)
    s1 = F.embedding(spks[1], emb)
    T = x.shape[1]
    h = torch.cat([x, s0.expand(-1, T, -1), s1.expand(-1, T, -1)], dim=2).transpose(1, 2)
    k = cfg.get("kernel_size", 5)
    for i in range(cfg.get("num_layers", 5)):
        pre = f"conv.{i}."
        h = F.relu(F.conv1d(h, P[pre + "0.weight"], P[pre + "0.bias"], padding=(k - 1) // 2))
        h = F.layer_norm(h.transpose(1, 2), (h.shape[1],), P[pre + "2.weight"],
                         P[pre + "2.bias"], 1e-12).transpose(1, 2)
        if dropout_masks is not None:
            h = h * dropout_masks[i].transpose(1, 2)
    h = h.transpose(1, 2)
    if cfg.get("use_mdn", False):
        return mdn_layer(P, "mdn_layer.", h, cfg.get("num_gaussians", 1), cfg["out_dim"],
                         cfg.get("dim_wise", False))
    return (F.linear(h, P["fc.weight"], P["fc.bias"]),)


def masked_mdn_loss(log_pi, log_sigma, mu, y, lengths):
    """train_multitrack.py:101-112: mdn_loss(reduce=False).masked_select(mask).mean()."""
    T = y.shape[1]
    mask = torch.arange(T)[None, :] < torch.as_tensor(lengths)[:, None]
    loss = mdn_loss(log_pi, log_sigma, mu, y, reduce=False)
    if loss.dim() == 3:
        mask = mask.unsqueeze(-1).expand_as(loss)
    return loss.masked_select(mask).mean()
