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
from .engine import (branch_streams, check_coop_errors, coop_error_word, empty,
                     flatten_parameters, grad_of, note_coop_check, weights_updated)
from .engine import _STATE as _ENGINE_STATE


class FusedAdam(torch.optim.Optimizer):
    """clip_grad_norm_(clip_norm) + torch.optim.Adam over the flat parameter buffer.

    Same update as torch.optim.Adam(weight_decay=0, amsgrad=False) after
    torch.nn.utils.clip_grad_norm_; the step is skipped when the norm is not
    finite (train_acoustic_multitrack.py:369-380).  The step counter and the bias
    corrections live on the device (ensvs_adam_step), so a skipped step does not
    advance the counter and the update replays correctly from a HIP graph.

    A torch.optim.Optimizer: ``param_groups[0]["lr"]`` is the learning rate, so the
    reference's schedulers drive it (StepLR, train_util.py:1348-1355 ``_instantiate_optim``;
    the new value reaches the device before the next step, eager or replayed), and
    ``state_dict()`` / ``load_state_dict()`` use torch.optim.Adam's format (per-parameter
    ``step`` / ``exp_avg`` / ``exp_avg_sq``), so a checkpoint's ``optimizer_state``
    (train_util.py:1324-1331, resumed at :1381-1384) moves between this optimizer and
    torch.optim.Adam in both directions.
    """

    def __init__(self, model, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 clip_norm=1.0):
        if weight_decay != 0.0:
            raise NotImplementedError("weight_decay != 0 (recipe uses 0.0)")
        if not hasattr(model, "_ensvs_flat"):
            flatten_parameters(model)
        if world_size() > 1:
            # DDP(model) broadcasts rank 0's parameters and buffers when it is built
            # (train_util.py:1446); the fused data-parallel step starts from the same state
            broadcast_state(model)
        self.model = model
        self.flat, self.gflat = model._ensvs_flat
        # torch.optim.Adam's defaults (its state_dict's param_groups carry them)
        defaults = dict(torch.optim.Adam([torch.zeros(1)]).defaults)
        defaults.update(lr=float(lr), betas=tuple(betas), eps=float(eps), weight_decay=0.0)
        super().__init__(list(model.parameters()), defaults)
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        self.betas, self.eps, self.clip_norm = tuple(betas), eps, clip_norm
        self.step_count = 0  # host count of step() calls (skipped steps included)
        # {device step, lr / bc1, sqrt(bc2), lr}
        self.dev_state = torch.zeros(4, dtype=torch.float64, device=self.flat.device)
        self._lr = None
        self.sync_lr()
        self.norm = torch.zeros(1, device=self.flat.device)
        self._part = torch.empty(1024, device=self.flat.device)
        # a cooperative recurrence that timed out (coop.h) makes the norm NaN: update skipped
        self._err = coop_error_word(self.flat.device) if self.flat.is_cuda else None

    @property
    def lr(self):
        return self.param_groups[0]["lr"]

    @lr.setter
    def lr(self, value):
        """Takes effect from the next step, eager or replayed."""
        self.param_groups[0]["lr"] = float(value)
        self.sync_lr()

    def sync_lr(self):
        """Push param_groups[0]["lr"] (set by a scheduler or by hand) to the device state the
        Adam kernel reads; called by step() and before every graph replay."""
        lr = float(self.param_groups[0]["lr"])
        if lr != self._lr:
            self._lr = lr
            self.dev_state[3].fill_(lr)

    @property
    def device_step(self):
        """Number of applied (finite-norm) updates, read from the device."""
        return int(self.dev_state[0].item())

    def zero_grad(self, set_to_none=False):
        self.gflat.zero_()
        for p in self.model.parameters():
            if p.grad is None or p.grad.data_ptr() != p._ensvs_gview.data_ptr():
                p.grad = p._ensvs_gview

    def grad_norm(self):
        call("ensvs_l2norm_chk", self.gflat.data_ptr(), self.gflat.numel(), self._part.data_ptr(),
             self.norm.data_ptr(), None if self._err is None else self._err.data_ptr(),
             Ly.stream())
        return self.norm

    def step(self, closure=None):
        if closure is not None:
            raise NotImplementedError("FusedAdam.step(closure)")
        self.step_count += 1
        self.sync_lr()
        b1, b2 = self.betas
        self.grad_norm()
        call("ensvs_adam_step", self.flat.data_ptr(), self.gflat.data_ptr(), self.m.data_ptr(),
             self.v.data_ptr(), self.flat.numel(), self.norm.data_ptr(), float(self.clip_norm),
             float(b1), float(b2), float(self.eps), self.dev_state.data_ptr(), Ly.stream())
        weights_updated()

    # ---- checkpoints (torch.optim.Adam format) ---------------------------------------
    def _slices(self):
        base = self.flat.data_ptr()
        for i, p in enumerate(self.param_groups[0]["params"]):
            o = (p.data_ptr() - base) // 4
            yield i, p, o

    def state_dict(self):
        """torch.optim.Adam.state_dict() of the same update: per-parameter 'step' (applied
        updates), 'exp_avg', 'exp_avg_sq' (CPU copies), and the param group."""
        step = float(self.device_step)
        state = {}
        if step > 0:
            for i, p, o in self._slices():
                n = p.numel()
                state[i] = {"step": torch.tensor(step, dtype=torch.float32),
                            "exp_avg": self.m[o:o + n].view_as(p).detach().cpu().clone(),
                            "exp_avg_sq": self.v[o:o + n].view_as(p).detach().cpu().clone()}
        g = {k: v for k, v in self.param_groups[0].items() if k != "params"}
        g["params"] = list(range(len(self.param_groups[0]["params"])))
        return {"state": state, "param_groups": [g]}

    def load_state_dict(self, state_dict):
        """Load torch.optim.Adam's (or this optimizer's) state_dict: moments into the flat
        buffers, the step count and bias corrections into the device state, lr / betas / eps
        from the param group."""
        groups = state_dict["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(self.param_groups[0]["params"]):
            raise ValueError("optimizer state does not match this model's parameters")
        g = groups[0]
        if float(g.get("weight_decay", 0.0)) != 0.0 or g.get("amsgrad", False):
            raise NotImplementedError("weight_decay / amsgrad state")
        new_b = tuple(g.get("betas", self.betas))
        new_e = float(g.get("eps", self.eps))
        if getattr(self, "_captured", False) and (new_b != tuple(self.betas) or new_e != self.eps):
            # a GraphedTrainStep baked b1, b2, eps into its captured Adam launch
            raise ValueError("FusedAdam.load_state_dict: betas / eps differ from the ones a "
                             "captured GraphedTrainStep replays; load the state before "
                             "capturing (or capture a new GraphedTrainStep)")
        for k in ("lr", "betas", "eps"):
            if k in g:
                self.param_groups[0][k] = tuple(g[k]) if k == "betas" else float(g[k])
        self.betas, self.eps = tuple(self.param_groups[0]["betas"]), self.param_groups[0]["eps"]
        ids = g["params"]
        st = state_dict["state"]
        steps = set()
        self.m.zero_()
        self.v.zero_()
        for i, p, o in self._slices():
            s = st.get(ids[i])
            if not s:
                continue
            n = p.numel()
            self.m[o:o + n].copy_(s["exp_avg"].reshape(-1))
            self.v[o:o + n].copy_(s["exp_avg_sq"].reshape(-1))
            steps.add(float(s["step"]))
        if len(steps) > 1:
            raise ValueError(f"per-parameter step counts differ: {sorted(steps)}")
        n_state = sum(1 for i in ids if st.get(i))
        if 0 < n_state < len(ids):
            # one device step count serves every parameter: the ones without state get zero
            # moments but the shared count's bias correction (torch.optim.Adam would start
            # them at step 1)
            import warnings
            warnings.warn(f"FusedAdam.load_state_dict: optimizer state for {n_state} of "
                          f"{len(ids)} parameters; the others start from zero moments with the "
                          "shared step count", RuntimeWarning, stacklevel=2)
        c = steps.pop() if steps else 0.0
        b1, b2 = self.betas
        self._lr = None
        self.sync_lr()
        self.dev_state[0].fill_(c)
        if c > 0:  # what adam_prepare_kernel left after step c
            self.dev_state[1].fill_(self.lr / (1.0 - b1 ** c))
            self.dev_state[2].fill_(math.sqrt(1.0 - b2 ** c))


def masked_l1(preds, targets, lengths_dev, n_valid_frames, B, T, grad_scale=1.0,
              total_cols=None):
    """Masked L1 summed over streams / element count, with its gradient.

    preds/targets: lists of (tensor, ld, col) with stream widths.  Returns
    (loss (1,) device tensor, list of grad tensors (B*T, n)).  The gradients are
    additionally multiplied by ``grad_scale`` (1/world under data parallelism).
    total_cols: the element count's stream width when these streams are part of a
    larger loss (default: their own widths).
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
    N = n_valid_frames * (total if total_cols is None else total_cols)
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


def broadcast_state(model, src=0, group=None):
    """Rank ``src``'s parameters (one broadcast of the flat buffer) and buffers (BatchNorm
    running statistics, diffusion schedules) to every rank, as DistributedDataParallel's
    constructor does (``_sync_module_states``)."""
    import torch.distributed as dist
    if world_size(group) == 1:
        return
    flat = getattr(model, "_ensvs_flat", None)
    if flat is not None:
        dist.broadcast(flat[0], src, group=group)
    else:
        for p in model.parameters():
            dist.broadcast(p.data, src, group=group)
    for b in model.buffers():
        dist.broadcast(b, src, group=group)
    weights_updated()


def sync_buffers(model, src=0, group=None):
    """DistributedDataParallel's default ``broadcast_buffers=True`` (the reference wraps the
    model in DDP(model, device_ids=[...]), train_util.py:1446): rank ``src``'s buffers (the
    BatchNorm running statistics) go to every rank before each step's forward, so an eval,
    inference or checkpoint on any rank sees rank src's statistics.  One broadcast per dtype
    of the coalesced buffers (a few KB)."""
    import torch.distributed as dist
    if world_size(group) == 1:
        return
    by_dtype = {}
    for b in model.buffers():
        by_dtype.setdefault((b.dtype, b.device), []).append(b)
    for ts in by_dtype.values():
        flat = torch._utils._flatten_dense_tensors(ts)
        dist.broadcast(flat, src, group=group)
        for t, f in zip(ts, torch._utils._unflatten_dense_tensors(flat, ts)):
            t.copy_(f)


# measurement hook (bench.py): when a list, every whole-buffer exchange of allreduce_grads
# appends its (start, end) HIP events, recorded on the stream the collectives are ordered on
EXCHANGE_EVENTS = None


def allreduce_grads(gflat, group=None):
    """Data-parallel gradient exchange: ONE sum all-reduce (RCCL over xGMI on the GPU
    box) of the flat gradient buffer.  The 1/world average is already folded into the
    loss gradient (``masked_l1(grad_scale=1/world)``), so no extra pass over the buffer.
    The reference's DDP (train_util.py:1176-1182 batch split + DistributedDataParallel)
    averages the same per-rank gradients."""
    import torch.distributed as dist
    if world_size(group) == 1:
        return
    ev = EXCHANGE_EVENTS if gflat.is_cuda else None
    if ev is not None:
        s = torch.cuda.Event(enable_timing=True)
        s.record()
    dist.all_reduce(gflat, op=dist.ReduceOp.SUM, group=group)
    _reduce_flag(gflat, group)
    if ev is not None:
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.append((s, e))


def _reduce_flag(gflat, group, async_op=False):
    """MAX all-reduce of this rank's cooperative-recurrence failure word (coop.h, 4 bytes)
    after the gradient's last collective: when any rank's recurrence failed, every rank's
    gradient norm is NaN, every rank skips the update (a local skip alone would let the
    ranks' parameters diverge) and every rank raises CoopError on the same step."""
    import torch.distributed as dist
    if not gflat.is_cuda:
        return None
    w = coop_error_word(gflat.device)[:1]
    return dist.all_reduce(w, op=dist.ReduceOp.MAX, group=group, async_op=async_op)


class BucketedAllReduce:
    """Data-parallel gradient exchange overlapped with the backward: the flat gradient
    buffer is all-reduced (SUM, async RCCL collectives) in buckets = the flat ranges of
    the parameter groups whose gradients are final at known points of the fused per-branch
    schedule -- the lf0, bap and V/UV models when their branch's backward ends, the mgc
    DiffNet once its backward is done (before the mgc encoder's: the longest tail of the
    step), the mgc encoder at the end of its branch, everything else (speaker embedding)
    after the join.  Each launch is issued on the branch's stream (the collective waits for
    that branch only) in the same host order on every rank; ``finish`` makes the current
    stream wait for all of them.  Same sums as one all-reduce of the whole buffer
    (element-wise); alignment pads between parameters are zeros and ride along."""

    def __init__(self, model, gflat, group=None, align=64):
        self.gflat, self.group, self.works = gflat, group, []
        base, n = gflat.data_ptr(), gflat.numel()

        def rng(params):
            spans = sorted(((grad_of(p).data_ptr() - base) // 4,
                            (grad_of(p).data_ptr() - base) // 4 + p.numel()) for p in params)
            out = []
            for a, b in spans:
                assert 0 <= a and b <= n, "parameter gradient outside the flat buffer"
                if out and a <= -(-out[-1][1] // align) * align:
                    out[-1][1] = max(out[-1][1], b)
                else:
                    out.append([a, b])
            return [tuple(r) for r in out]

        den = list(model.mgc_model.denoise_fn.parameters())
        den_ids = {id(p) for p in den}
        groups = {"lf0": list(model.lf0_model.parameters()), "mgc_denoiser": den,
                  "mgc": [p for p in model.mgc_model.parameters() if id(p) not in den_ids],
                  "bap": list(model.bap_model.parameters()),
                  "vuv": list(model.vuv_model.parameters())}
        seen = {id(p) for ps in groups.values() for p in ps}
        groups["rest"] = [p for p in model.parameters() if id(p) not in seen]
        self.buckets = {k: rng(v) for k, v in groups.items() if v}

    def launch(self, tag):
        import torch.distributed as dist
        from .kernels import flush_wgrad
        flush_wgrad()  # this stream's queued weight-gradient reductions first
        for a, b in self.buckets.get(tag, ()):
            self.works.append(dist.all_reduce(self.gflat[a:b], op=dist.ReduceOp.SUM,
                                              group=self.group, async_op=True))

    def finish(self):
        self.launch("rest")
        w = _reduce_flag(self.gflat, self.group, async_op=True)  # the failure word, MAX
        if w is not None:
            self.works.append(w)
        self.collectives_last_step = len(self.works)  # bench.py reports it
        for w in self.works:
            w.wait()
        self.works = []


# overlapped bucketed all-reduce in the eager fused step (W > 1); set_overlap_allreduce(False):
# one all-reduce of the whole buffer after the backward
_STATE_OVERLAP = {"on": True}


def set_overlap_allreduce(on: bool):
    _STATE_OVERLAP["on"] = bool(on)


def _bucketed(model, optimizer):
    br = getattr(optimizer, "_bucketed", None)
    if br is None or br.gflat is not optimizer.gflat:
        br = optimizer._bucketed = BucketedAllReduce(model, optimizer.gflat)
    return br


def _interaction(optimizer, outs, y_main, y_sub, Dy, o, lens_dev, B, T, w, W, loss, g_lf0):
    """log-F0 interaction loss (train_acoustic_multitrack.py:175-182): its weighted value into
    its own scalar (kept for the metrics), added to ``loss``; gradients into g_lf0 (+=) and a
    new sub-track buffer, returned."""
    ys = y_sub.contiguous().float()
    dev = y_main.device
    g_sub = empty(B * T, device=dev)
    part = empty(1024, device=dev)
    il = torch.zeros(1, device=dev)
    call("ensvs_lf0_interaction", outs["lf0"].data_ptr(), outs["lf0_sub"].data_ptr(),
         y_main.data_ptr(), ys.data_ptr(), Dy, o[1], o[2], lens_dev.data_ptr(), B, T, float(w),
         1.0 / W, part.data_ptr(), il.data_ptr(), g_lf0.data_ptr(), g_sub.data_ptr(), Ly.stream())
    call("ensvs_axpy", loss.data_ptr(), il.data_ptr(), 1.0, 1, Ly.stream())
    optimizer._il = (il, float(w))
    return g_sub


def step_metrics(loss, optimizer):
    """The reference's per-step log metrics (train_acoustic_multitrack.py:382-390) of the last
    train_step, as host floats: Loss, Loss_Feats, Loss_Pitch (pitch_reg_weight 0 in the
    recipe), Loss_LogF0_Interaction (unweighted), Loss_MGC-0th_Interaction (0) and GradNorm
    (only when finite: the reference skips the step and the metric otherwise).  Reads the
    device (a sync); call it only when logging.  Raises engine.CoopError when a cooperative
    recurrence of a step since the last check failed (that step's update was skipped)."""
    check_coop_errors(loss.device, sync=True)
    total = float(loss.item())
    il = getattr(optimizer, "_il", None)
    wil = float(il[0].item()) if il is not None else 0.0
    out = {"Loss": total, "Loss_Feats": total - wil, "Loss_Pitch": 0.0,
           "Loss_LogF0_Interaction": wil / il[1] if il is not None else 0.0,
           "Loss_MGC-0th_Interaction": 0.0}
    gn = float(optimizer.norm.item())
    if math.isfinite(gn):
        out["GradNorm"] = gn
    return out


def train_step(model, optimizer, x_main, x_sub, y_main, spk_main, spk_sub, lengths, draws=None,
               ddp=True, y_sub=None, logf0_diff_weight=0.0):
    """One training step on a (main, sub) pair batch.  Returns (loss, grad_norm) device tensors.

    lengths = max(L_main, L_sub) per pair (train_acoustic_multitrack.py:82).
    logf0_diff_weight > 0 adds the log-F0 interaction loss between the main and sub tracks
    (train_acoustic_multitrack.py:175-182, 296; needs the output_subtrack model and y_sub).
    """
    dev = x_main.device
    # an earlier step's cooperative-recurrence failure, once the device got there (no wait)
    check_coop_errors(dev, sync=False)
    if ddp and world_size() > 1:
        sync_buffers(model)
    loss = _loss_and_grads(model, optimizer, x_main, x_sub, y_main, spk_main, spk_sub, lengths,
                           draws, ddp, y_sub, logf0_diff_weight, overlap=True)
    if ddp and world_size() > 1 and not getattr(optimizer, "_reduced", False):
        allreduce_grads(optimizer.gflat)
    optimizer._reduced = False
    optimizer.step()
    if dev.type == "cuda" and not torch.cuda.is_current_stream_capturing():
        note_coop_check(dev)
    return loss, optimizer.norm


def train_step_single(model, optimizer, x, y, lengths, draws=None, ddp=True):
    """One training step of the single-track NPSSMDNMultistreamParametricModel (BASELINE
    config 2; nnsvs/bin/train_acoustic.py:33-274 with feats_criterion l1, pitch_reg_weight 0):
    forward with teacher forcing, masked L1 over all streams / element count, backward,
    clip, Adam.  lengths: per-sequence valid frames (sorted descending, train_acoustic.py:
    :343).  Returns (loss, grad_norm) device tensors."""
    return train_step(model, optimizer, x, None, y, None, None, lengths, draws=draws, ddp=ddp)


def _loss_and_grads(model, optimizer, x_main, x_sub, y_main, spk_main, spk_sub, lengths, draws,
                    ddp, y_sub, logf0_diff_weight, overlap=False):
    """zero_grad + forward + masked L1 (+ interaction loss) + backward into the flat grads.
    The weighted interaction term is also kept apart (optimizer._il) for the step metrics.
    An eval-mode model is switched to training mode (the reference's train_loop does this per
    phase, train_acoustic_multitrack.py:452); a training-mode model is left as it is, so
    BatchNorm modules frozen with bn.eval() stay frozen (running statistics, ensvs_bn_bwd_frozen)."""
    if not model.training:
        model.train()
    optimizer.zero_grad()
    optimizer._il = None
    with Ly.K.deferred_wgrad():
        return _loss_and_grads_body(model, optimizer, x_main, x_sub, y_main, spk_main, spk_sub,
                                    lengths, draws, ddp, y_sub, logf0_diff_weight, overlap)


def _loss_and_grads_body(model, optimizer, x_main, x_sub, y_main, spk_main, spk_sub, lengths,
                         draws, ddp, y_sub, logf0_diff_weight, overlap):
    """_loss_and_grads with the weight-gradient reductions queued (kernels.deferred_wgrad)."""
    if logf0_diff_weight > 0.0 and (not model.output_subtrack or y_sub is None):
        raise ValueError("logf0_diff_weight > 0 needs output_subtrack=True and y_sub (the "
                         "SeparateF0 model: through its forward, with autograd)")
    if _STATE_FUSED["on"] and getattr(model, "_train_fused", None) is not None:
        reducer = None
        if (overlap and ddp and _STATE_OVERLAP["on"] and world_size() > 1 and
                getattr(model, "mgc_model", None) is not None and
                hasattr(model.mgc_model, "denoise_fn")):
            reducer = _bucketed(model, optimizer)
        loss = _loss_and_grads_fused(model, optimizer, x_main, x_sub, y_main, spk_main, spk_sub,
                                     lengths, draws, ddp, y_sub, logf0_diff_weight, reducer)
        if reducer is not None:
            reducer.finish()
            optimizer._reduced = True
        return loss
    outs, st = model._train_fwd(x_main, x_sub, y_main, spk_main, spk_sub, lengths, draws)
    B, T = st["B"], st["T"]
    Dy = y_main.shape[2]
    o = model._stream_cols()
    preds, targets, keys = model._l1_terms(outs, y_main)
    W = world_size() if ddp else 1
    loss, grads = masked_l1(preds, targets, st["lens_dev"], sum(st["lens_host"]), B, T,
                            grad_scale=1.0 / W)
    g = {k: gi.view(-1) if k == "lf0" else gi for k, gi in zip(keys, grads)}
    if logf0_diff_weight > 0.0:
        if not model.output_subtrack or y_sub is None:
            raise ValueError("logf0_diff_weight > 0 needs output_subtrack=True and y_sub")
        g["lf0_sub"] = _interaction(optimizer, outs, y_main, y_sub, Dy, o, st["lens_dev"], B, T,
                                    logf0_diff_weight, W, loss, g["lf0"])
    model._train_bwd(st, g)
    return loss


# Per-branch fused schedule (forward -> loss gradient -> backward of each branch on its own
# stream, acoustic_models._train_fused), the default: with 8 hardware queues it measured
# 20.4 vs 20.6 ms/step for the forward-all / loss / backward-all schedule (graph replay,
# 30 x 1024; with 4 queues it was 22.3 vs 22.0).  Same gradients bitwise; the loss is the
# sum of the branches' partial losses.  set_fused_branches(False) turns it off.
_STATE_FUSED = {"on": True}


def set_fused_branches(on: bool):
    _STATE_FUSED["on"] = bool(on)


def _loss_and_grads_fused(model, optimizer, x_main, x_sub, y_main, spk_main, spk_sub, lengths,
                          draws, ddp, y_sub, logf0_diff_weight, reducer=None):
    """The loss of _loss_and_grads split by branch: each branch's masked L1 over its own
    streams with the whole loss's element count (same gradients, elementwise), the
    interaction loss inside the lf0 branch; partial losses summed after the join."""
    Dy = y_main.shape[2]
    o = model._stream_cols()
    nm, nb = model.stream_sizes[0], model.stream_sizes[3]
    W = world_size() if ddp else 1
    total = nm + 1 + 1 + nb

    def branch_loss(i, outs, st):
        B, T = st["B"], st["T"]
        nvalid = sum(st["lens_host"])
        if i == 1:
            pt = [(outs["mgc_recon"], nm, 0, nm)], [(outs["mgc_noise"], nm, 0)], "mgc_recon"
        elif i == 2:
            pt = [(outs["bap_recon"], nb, 0, nb)], [(outs["bap_noise"], nb, 0)], "bap_recon"
        elif i == 3:
            pt = [(outs["vuv"], 1, 0, 1)], [(y_main, Dy, o[2])], "vuv"
        else:
            pt = [(outs["lf0"], 1, 0, 1)], [(y_main, Dy, o[1])], "lf0"
        loss, (gi,) = masked_l1(pt[0], pt[1], st["lens_dev"], nvalid, B, T, grad_scale=1.0 / W,
                                total_cols=total)
        g = {pt[2]: gi.view(-1) if i == 0 else gi}
        if i == 0 and logf0_diff_weight > 0.0:
            g["lf0_sub"] = _interaction(optimizer, outs, y_main, y_sub, Dy, o, st["lens_dev"], B,
                                        T, logf0_diff_weight, W, loss, g["lf0"])
        return loss, g

    loss, _ = model._train_fused(x_main, x_sub, y_main, spk_main, spk_sub, lengths, draws,
                                 branch_loss, reduce_hook=None if reducer is None else
                                 reducer.launch)
    return loss


class GraphedTrainStep:
    """``train_step`` on fixed shapes, captured as HIP graphs and replayed.

    Capture records every launch of one step: graph 1 = RNG epoch advance, zero_grad,
    forward, loss, backward; graph 2 = grad-norm, clip and Adam.  Between them the RCCL
    gradient all-reduce runs eagerly when the process group has more than one rank (one
    collective on the flat gradient buffer), so data-parallel runs never depend on
    collective capture.  Each replay draws fresh diffusion steps, noise and dropout masks
    (ensvs_rng_advance) and takes the Adam step count and bias corrections from the
    device (FusedAdam.dev_state), so replay k is the k-th training step, not a repeat.

    ``warmup`` eager steps (real optimizer steps) run first on the capture stream so
    every lazily built cache (packed-weight descriptors, workspaces, lengths) exists
    before capture.  Inputs are copied into static buffers: call ``step(**batch)`` with
    new tensors of the captured shapes, or ``step()`` to retrain on the same batch.
    """

    def __init__(self, model, optimizer, x_main, x_sub, y_main, spk_main, spk_sub, lengths,
                 warmup=1, ddp=True, y_sub=None, logf0_diff_weight=0.0, draws=None, pool=None):
        self.model, self.opt, self.ddp = model, optimizer, ddp
        # explicit draws (train_step's `draws`) become static buffers refilled per step
        self.draws = None if draws is None else {k: v.clone() for k, v in draws.items()}
        self.lengths = [int(v) for v in lengths]
        self.kw = dict(y_sub=None if y_sub is None else y_sub.clone(),
                       logf0_diff_weight=logf0_diff_weight)
        cl = lambda t: None if t is None else t.clone()  # noqa: E731 (single track: None)
        self.inputs = dict(x_main=cl(x_main), x_sub=cl(x_sub), y_main=cl(y_main),
                           spk_main=cl(spk_main), spk_sub=cl(spk_sub))
        dev = x_main.device
        if _ENGINE_STATE["concurrent"]:
            branch_streams(dev)  # before the capture stream (engine.branch_streams)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                loss = self._eager()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        self.warmup_result = (loss, optimizer.norm.clone())
        self.g_grads, self.g_update = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_grads, pool=pool):
            call("ensvs_rng_advance", Ly.stream())
            self.loss = self._grads()
        self.pool = self.g_grads.pool()
        with torch.cuda.graph(self.g_update, pool=self.pool):
            optimizer.step()
        optimizer._captured = True  # b1, b2, eps are now kernel arguments of g_update
        self.norm = optimizer.norm
        # the interaction-loss scalar was allocated in the capture: keep it with the graph
        self.il = getattr(optimizer, "_il", None)

    def _grads(self):
        i = self.inputs
        return _loss_and_grads(self.model, self.opt, i["x_main"], i["x_sub"], i["y_main"],
                               i["spk_main"], i["spk_sub"], self.lengths, self.draws, self.ddp,
                               self.kw["y_sub"], self.kw["logf0_diff_weight"])

    def _eager(self):
        loss = self._grads()
        if self.ddp and world_size() > 1:
            allreduce_grads(self.opt.gflat)
        self.opt.step()
        return loss

    def step(self, draws=None, lengths=None, **batch):
        """One training step (replay).  Returns the static (loss, grad_norm) tensors.

        The valid lengths are part of the captured graph (the masked-L1 element count and
        the packed recurrences' bounds): a batch must have exactly the captured lengths
        (bucketed batches of identical lengths); passing different ``lengths`` raises."""
        if lengths is not None and [int(v) for v in lengths] != self.lengths:
            raise ValueError("GraphedTrainStep: lengths differ from the captured ones "
                             f"({list(lengths)[:4]}... vs {self.lengths[:4]}...); capture "
                             "another GraphedTrainStep for this bucket")
        for k, v in (draws or {}).items():
            if self.draws is None or self.draws[k].shape != v.shape:
                raise ValueError(f"draws[{k}]: not captured with this shape")
            self.draws[k].copy_(v, non_blocking=True)
        for k, v in batch.items():
            dst = self.kw["y_sub"] if k == "y_sub" else self.inputs[k]
            if dst is None or dst.shape != v.shape:
                raise ValueError(f"{k}: shape {tuple(v.shape)} differs from the captured one")
            dst.copy_(v, non_blocking=True)
        dev = self.opt.flat.device
        check_coop_errors(dev, sync=False)  # an earlier replay's failure (no wait)
        self.opt.sync_lr()  # a scheduler's lr change reaches the replayed update
        if self.ddp and world_size() > 1:
            sync_buffers(self.model)
        self.g_grads.replay()
        if self.ddp and world_size() > 1:
            allreduce_grads(self.opt.gflat)
        self.g_update.replay()
        self.opt.step_count += 1
        self.opt._il = self.il
        weights_updated()
        note_coop_check(dev)
        return self.loss, self.norm


class StepGraphCache:
    """Training steps of ragged dynamic batches at graph speed: one GraphedTrainStep per batch
    signature (pair count, frames, per-pair lengths, sub-track target and draw shapes),
    captured the first time the signature comes and replayed whenever it comes again.

    The reference's loop (train_acoustic_multitrack.py:461-563) iterates batch_by_size buckets
    (train_util.py:190-246) that are fixed for the run -- ShuffleBatchSampler only reorders
    them -- so every batch shape of epoch 1 recurs in every later epoch.  A miss runs the
    batch's step eagerly (GraphedTrainStep's warm-up step IS that batch's training step, a real
    update) and captures it; a hit copies the batch into the graph's static inputs and replays.
    So every batch is exactly one training step either way, with the same bits as eager
    train_step calls given the same draws (tests/test_graph_cache_gpu.py).

    Memory: every graph captures into ONE shared pool, so the cache costs about one step's
    working set plus each graph's static inputs, not one working set per shape.  That is safe
    because the graphs replay one at a time on one stream, and what a replay leaves for later
    (parameters, gradients, Adam moments, BatchNorm statistics, the gradient norm) lives
    outside the pool; the loss a replay writes into its static buffer is copied out at once
    (step() returns copies), and caches that a graph's launches point into are never freed
    (engine.retire).  At most ``max_graphs`` signatures are kept (least recently used first out).
    """

    def __init__(self, model, optimizer, ddp=True, logf0_diff_weight=0.0, max_graphs=64):
        from collections import OrderedDict
        self.model, self.opt, self.ddp = model, optimizer, ddp
        self.logf0_diff_weight = float(logf0_diff_weight)
        self.max_graphs = int(max_graphs)
        self.graphs = OrderedDict()
        self.uses = {}  # steps run per signature (capture included)
        self.pool = None
        self.captures = self.replays = 0

    @staticmethod
    def signature(x_main, x_sub, y_main, spk_main, spk_sub, lengths, y_sub=None, draws=None):
        shp = lambda t: None if t is None else (tuple(t.shape), t.dtype)  # noqa: E731
        return (shp(x_main), shp(x_sub), shp(y_main), shp(spk_main), shp(spk_sub),
                tuple(int(v) for v in lengths), shp(y_sub),
                None if draws is None else tuple(sorted((k, shp(v)) for k, v in draws.items())))

    def step(self, x_main, x_sub, y_main, spk_main, spk_sub, lengths, y_sub=None, draws=None):
        """One training step on this batch; returns (loss, grad_norm) as fresh device tensors."""
        key = self.signature(x_main, x_sub, y_main, spk_main, spk_sub, lengths, y_sub, draws)
        self.uses[key] = self.uses.get(key, 0) + 1
        g = self.graphs.get(key)
        if g is None:
            while len(self.graphs) >= self.max_graphs:
                self.graphs.popitem(last=False)
            check_coop_errors(x_main.device, sync=False)
            g = GraphedTrainStep(self.model, self.opt, x_main, x_sub, y_main, spk_main, spk_sub,
                                 lengths, warmup=1, ddp=self.ddp, y_sub=y_sub,
                                 logf0_diff_weight=self.logf0_diff_weight, draws=draws,
                                 pool=self.pool)
            self.pool = g.pool
            self.graphs[key] = g
            self.captures += 1
            loss, norm = g.warmup_result
            note_coop_check(x_main.device)
            return loss, norm
        self.graphs.move_to_end(key)
        batch = dict(x_main=x_main, y_main=y_main)
        for k, v in (("x_sub", x_sub), ("spk_main", spk_main), ("spk_sub", spk_sub),
                     ("y_sub", y_sub)):
            if v is not None:
                batch[k] = v
        loss, norm = g.step(draws=draws, **batch)
        self.replays += 1
        return loss.clone(), norm.clone()


def train_epoch(model, optimizer, feeder, logf0_diff_weight=0.0, ddp=True, graphs=None):
    """The batch loop of train_loop (train_acoustic_multitrack.py:461-484, 94-100) over a
    loader.PairBatchFeeder: each fed batch (tracks already sorted independently by
    length, lengths = max(L0, L1)) goes through one fused training step.  With ``graphs`` (a
    StepGraphCache kept across epochs) each batch shape is captured once and replayed from
    then on; without, every step is issued eagerly (train_step).  Returns the per-step
    (loss, grad_norm) device tensors (copies); the host reads them only when it asks."""
    out = []
    n = len(feeder) if hasattr(feeder, "__len__") else None
    for i, b in enumerate(feeder):
        if i + 1 == n and hasattr(feeder, "prestart"):
            feeder.prestart()  # the next pass's first batches load while this step runs
        lengths = [int(v) for v in b["host_lengths"]]
        y_sub = b["y_sub"] if logf0_diff_weight > 0 else None
        args = (b["x_main"], b["x_sub"], b["y_main"], b["spk_main"], b["spk_sub"], lengths)
        if graphs is not None:
            loss, norm = graphs.step(*args, y_sub=y_sub)
        else:
            loss, norm = train_step(model, optimizer, *args, ddp=ddp, y_sub=y_sub,
                                    logf0_diff_weight=logf0_diff_weight)
            norm = norm.clone()
        out.append((loss, norm))
    if out:
        check_coop_errors(out[0][0].device, sync=True)
    return out
