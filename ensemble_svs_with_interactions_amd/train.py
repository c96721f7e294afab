"""Fused multi-track training step (nnsvs/bin/train_acoustic_multitrack.py:40-392).

``train_step`` is the reference step with the recipe settings
(feats_criterion l1, stream_wise_loss False, pitch_reg_weight 0,
logf0_diff_weight 0 -- or > 0 with the output_subtrack model, the interaction-loss
recipe -- clip_norm 1.0, Adam): forward of the pairwise model,
masked L1 over all streams divided by the element count, backward, optional
RCCL gradient all-reduce (data parallel over pairs), global-norm clipping,
non-finite skip and Adam — every arithmetic op in libensvs.so, no host sync.
"""
import ctypes
import math

import torch

from . import layers as Ly
from ._lib import call
from .engine import empty, flatten_parameters, weights_updated


class FusedAdam:
    """clip_grad_norm_(clip_norm) + torch.optim.Adam over the flat parameter buffer.

    Same update as torch.optim.Adam(weight_decay=0, amsgrad=False) after
    torch.nn.utils.clip_grad_norm_; the step is skipped when the norm is not
    finite (train_acoustic_multitrack.py:369-380).
    """

    def __init__(self, model, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 clip_norm=1.0):
        if weight_decay != 0.0:
            raise NotImplementedError("weight_decay != 0 (recipe uses 0.0)")
        if not hasattr(model, "_ensvs_flat"):
            flatten_parameters(model)
        self.model = model
        self.flat, self.gflat = model._ensvs_flat
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        self.lr, self.betas, self.eps, self.clip_norm = lr, betas, eps, clip_norm
        self.step_count = 0
        self.norm = torch.zeros(1, device=self.flat.device)
        self._part = torch.empty(1024, device=self.flat.device)

    def zero_grad(self):
        self.gflat.zero_()
        for p in self.model.parameters():
            if p.grad is None or p.grad.data_ptr() != p._ensvs_gview.data_ptr():
                p.grad = p._ensvs_gview

    def grad_norm(self):
        call("ensvs_l2norm", self.gflat.data_ptr(), self.gflat.numel(), self._part.data_ptr(),
             self.norm.data_ptr(), Ly.stream())
        return self.norm

    def step(self):
        self.step_count += 1
        b1, b2 = self.betas
        self.grad_norm()
        bc1 = 1.0 - b1 ** self.step_count
        bc2 = 1.0 - b2 ** self.step_count
        call("ensvs_adam", self.flat.data_ptr(), self.gflat.data_ptr(), self.m.data_ptr(),
             self.v.data_ptr(), self.flat.numel(), self.norm.data_ptr(), float(self.clip_norm),
             float(self.lr), float(b1), float(b2), float(self.eps), float(bc1),
             float(math.sqrt(bc2)), Ly.stream())
        weights_updated()


def masked_l1(preds, targets, lengths_dev, n_valid_frames, B, T, grad_scale=1.0):
    """Masked L1 summed over streams / element count, with its gradient.

    preds/targets: lists of (tensor, ld, col) with stream widths.  Returns
    (loss (1,) device tensor, list of grad tensors (B*T, n)).  The gradients are
    additionally multiplied by ``grad_scale`` (1/world under data parallelism).
    """
    ns = len(preds)
    dev = preds[0][0].device
    pa = (ctypes.c_void_p * ns)()
    pb = (ctypes.c_void_p * ns)()
    pg = (ctypes.c_void_p * ns)()
    la = (ctypes.c_int * ns)()
    lb = (ctypes.c_int * ns)()
    lg = (ctypes.c_int * ns)()
    nn_ = (ctypes.c_int * ns)()
    grads = []
    total = 0
    for i, ((a, lda, ca, n), (b, ldb, cb)) in enumerate(zip(preds, targets)):
        g = empty(B * T, n, device=dev)
        grads.append(g)
        pa[i] = a.data_ptr() + 4 * ca
        pb[i] = b.data_ptr() + 4 * cb
        pg[i] = g.data_ptr()
        la[i], lb[i], lg[i], nn_[i] = lda, ldb, n, n
        total += n
    N = n_valid_frames * total
    part = empty(1024, device=dev)
    loss = empty(1, device=dev)
    call("ensvs_masked_l1", ctypes.addressof(pa), ctypes.addressof(pb), ctypes.addressof(pg),
         ctypes.addressof(la), ctypes.addressof(lb), ctypes.addressof(lg), ctypes.addressof(nn_),
         ns, lengths_dev.data_ptr(), B, T, 1.0 / N, float(grad_scale), part.data_ptr(), loss.data_ptr(), Ly.stream())
    return loss, grads


def world_size(group=None):
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


def allreduce_grads(gflat, group=None):
    """Data-parallel gradient exchange: ONE sum all-reduce (RCCL over xGMI on the GPU
    box) of the flat gradient buffer.  The 1/world average is already folded into the
    loss gradient (``masked_l1(grad_scale=1/world)``), so no extra pass over the buffer.
    The reference's DDP (train_util.py:1176-1182 batch split + DistributedDataParallel)
    averages the same per-rank gradients."""
    import torch.distributed as dist
    if world_size(group) == 1:
        return
    dist.all_reduce(gflat, op=dist.ReduceOp.SUM, group=group)


def train_step(model, optimizer, x_main, x_sub, y_main, spk_main, spk_sub, lengths, draws=None,
               ddp=True, y_sub=None, logf0_diff_weight=0.0):
    """One training step on a (main, sub) pair batch.  Returns (loss, grad_norm) device tensors.

    lengths = max(L_main, L_sub) per pair (train_acoustic_multitrack.py:82).
    logf0_diff_weight > 0 adds the log-F0 interaction loss between the main and sub tracks
    (train_acoustic_multitrack.py:175-182, 296; needs the output_subtrack model and y_sub).
    """
    model.train()
    optimizer.zero_grad()
    outs, st = model._train_fwd(x_main, x_sub, y_main, spk_main, spk_sub, lengths, draws)
    B, T = st["B"], st["T"]
    Dy = y_main.shape[2]
    o = model._stream_cols()
    nm, nb = model.stream_sizes[0], model.stream_sizes[3]
    preds = [(outs["mgc_recon"], nm, 0, nm), (outs["lf0"], 1, 0, 1), (outs["vuv"], 1, 0, 1),
             (outs["bap_recon"], nb, 0, nb)]
    targets = [(outs["mgc_noise"], nm, 0), (y_main, Dy, o[1]), (y_main, Dy, o[2]),
               (outs["bap_noise"], nb, 0)]
    W = world_size() if ddp else 1
    loss, (g_m, g_l, g_v, g_b) = masked_l1(preds, targets, st["lens_dev"], sum(st["lens_host"]),
                                           B, T, grad_scale=1.0 / W)
    g = dict(mgc_recon=g_m, lf0=g_l.view(-1), vuv=g_v, bap_recon=g_b)
    if logf0_diff_weight > 0.0:
        if not model.output_subtrack or y_sub is None:
            raise ValueError("logf0_diff_weight > 0 needs output_subtrack=True and y_sub")
        y_sub = y_sub.contiguous().float()
        g_sub = empty(B * T, device=y_main.device)
        part = empty(1024, device=y_main.device)
        call("ensvs_lf0_interaction", outs["lf0"].data_ptr(), outs["lf0_sub"].data_ptr(),
             y_main.data_ptr(), y_sub.data_ptr(), Dy, o[1], o[2], st["lens_dev"].data_ptr(), B, T,
             float(logf0_diff_weight), 1.0 / W, part.data_ptr(), loss.data_ptr(),
             g["lf0"].data_ptr(), g_sub.data_ptr(), Ly.stream())
        g["lf0_sub"] = g_sub
    model._train_bwd(st, g)
    if W > 1:
        allreduce_grads(optimizer.gflat)
    optimizer.step()
    return loss, optimizer.norm
