"""Execution plumbing shared by every module of the path.

* GEMM precision (``bf16`` MFMA operands with fp32 accumulation for production,
  exact ``fp32`` MFMA for parity runs).
* Flat parameter / gradient buffers: every parameter is a view into one fp32
  buffer and its ``.grad`` a view into another, so clipping, Adam and the
  RCCL all-reduce each touch one contiguous buffer (one launch / one
  collective).  Backward kernels always ACCUMULATE into ``.grad`` (autograd
  semantics); ``zero_grad`` zeroes the flat buffer.
* ``ModulePacks``: per-module packed GEMM operands, rebuilt when parameters
  move and repacked (one launch) when they change.
"""

import torch

from . import _lib
from .kernels import PackedBuffer

_STATE = {"gemm_dtype": _lib.DT_BF16, "epoch": 0, "rng": None, "concurrent": True}
_SIDE_STREAMS = {}
# Dev instrumentation: set to a list to collect (branch, start_event, end_event) per
# branch region (tools/branch_times.py); None = off.
BRANCH_TIMES = None


class _timed:
    def __init__(self, ctx, i):
        self.ctx, self.i = ctx, i

    def __enter__(self):
        self.ctx.__enter__()
        self.s = torch.cuda.Event(enable_timing=True)
        self.s.record()
        return self

    def __exit__(self, *exc):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        BRANCH_TIMES.append((self.i, self.s, e))
        return self.ctx.__exit__(*exc)


def branch_streams(device, n_side=3):
    """The side streams of Branches(device, n_side), created on first use, each given its
    first command at once.  HIP binds a stream to a hardware queue when the stream is first
    used: side streams first used inside GraphedTrainStep's warm-up (on its capture stream)
    left the two reverse-diffusion graphs of every later inference unable to overlap (pair
    inference 116 ms, slower than the serial 109 ms); created and touched before the
    capture stream (GraphedTrainStep calls this first): 83 ms
    (tools/infer_streams_probe.py)."""
    key = (str(device), n_side)
    if key not in _SIDE_STREAMS:
        # equal priorities: a high-priority branch stream measured slower (lf0 23.5, mgc
        # 23.4, bap 22.2 vs 22.2 ms/step for none; graph replay, 30 x 1024)
        _SIDE_STREAMS[key] = [torch.cuda.Stream(device) for _ in range(n_side)]
        cur = torch.cuda.current_stream(device)
        for s in _SIDE_STREAMS[key]:  # first command on each new stream now
            s.wait_stream(cur)
            cur.wait_stream(s)
    return _SIDE_STREAMS[key]


def set_concurrency(on: bool):
    """Run the independent branches of the step (lf0 / mgc / bap / vuv) on their own HIP
    streams (default) or serially on the current stream."""
    _STATE["concurrent"] = bool(on)


class Branches:
    """Fork/join of independent branches of one step onto concurrent HIP streams.

    Branch ``i < n_side`` runs on side stream i, anything else on the current (main)
    stream, so n_side + 1 branches use n_side + 1 hardware queues (GPU_MAX_HW_QUEUES
    defaults to 4).  Side streams wait for the main stream at entry; the main stream
    waits for every side stream at exit.  A branch's saved state must be consumed on
    the same branch index in backward (stream-ordered reuse of freed memory).
    """

    def __init__(self, device, n_side=3):
        self.device = device
        self.on_side = _STATE["concurrent"] and torch.cuda.is_available()
        self.side = branch_streams(device, n_side) if self.on_side else []

    def __enter__(self):
        if self.on_side:
            self.main = torch.cuda.current_stream(self.device)
            ev = self.main.record_event()
            for s in self.side:
                s.wait_event(ev)
        return self

    def on(self, i):
        import contextlib
        if self.on_side and i < len(self.side):
            ctx = torch.cuda.stream(self.side[i])
        else:
            ctx = contextlib.nullcontext()
        ctx = _flushing(ctx)
        if BRANCH_TIMES is None:
            return ctx
        return _timed(ctx, i)

    def __exit__(self, *exc):
        if self.on_side:
            for s in self.side:
                self.main.wait_stream(s)
        return False


class _flushing:
    """A branch region that issues its stream's queued weight-gradient reductions
    (kernels.flush_wgrad) before it ends, so the join sees final gradients."""

    def __init__(self, ctx):
        self.ctx = ctx

    def __enter__(self):
        return self.ctx.__enter__()

    def __exit__(self, *exc):
        if exc[0] is None:
            from .kernels import flush_wgrad
            flush_wgrad()
        return self.ctx.__exit__(*exc)


def next_seed() -> int:
    """64-bit seed for the counter-based RNG kernels, derived from torch's global seed so
    torch.manual_seed() makes runs reproducible."""
    import random
    if _STATE["rng"] is None or _STATE["rng"][0] != torch.initial_seed():
        _STATE["rng"] = (torch.initial_seed(), random.Random(torch.initial_seed()))
    return _STATE["rng"][1].getrandbits(64)


class seed_scope:
    """Inside the block, next_seed() draws from a generator seeded with ``seed``: a call
    that takes its randomness as an explicit seed (the torch.library ops, torch_ops.py) is
    a pure function of its arguments."""

    def __init__(self, seed: int):
        import random
        self.rng = (torch.initial_seed(), random.Random(int(seed)))

    def __enter__(self):
        self.saved = _STATE["rng"]
        _STATE["rng"] = self.rng
        return self

    def __exit__(self, *exc):
        _STATE["rng"] = self.saved
        return False


def set_gemm_precision(p: str):
    """'bf16' (default; MFMA bf16 operands, fp32 accumulate) or 'fp32' (exact fp32 MFMA)."""
    _STATE["gemm_dtype"] = {"bf16": _lib.DT_BF16, "fp32": _lib.DT_F32}[p]


def gemm_precision():
    return "bf16" if _STATE["gemm_dtype"] == _lib.DT_BF16 else "fp32"


def gemm_dtype():
    return _STATE["gemm_dtype"]


def weights_updated():
    """Call after parameters were modified through raw pointers (fused optimizer)."""
    _STATE["epoch"] += 1


def grad_of(p: torch.Tensor) -> torch.Tensor:
    """The tensor backward kernels accumulate into for parameter ``p``."""
    if p.grad is None:
        g = getattr(p, "_ensvs_gview", None)
        if g is None:
            g = torch.zeros_like(p)
        else:
            g.zero_()
        p.grad = g
    return p.grad


class GradCapture:
    """Routes the parameter gradients that backward kernels write (through ``grad_of``)
    into fresh buffers that an autograd ``Function.backward`` RETURNS, instead of into
    ``p.grad``.  Autograd then accumulates them into ``p.grad`` itself, so
    DistributedDataParallel's per-parameter hooks fire and ``GradScaler.unscale_`` /
    ``clip_grad_norm_`` see ordinary gradients (the reference's own train_step,
    train_acoustic_multitrack.py:93-100, 358-380).  The fused ``train.train_step``
    does not go through autograd and writes ``p.grad`` directly.

    Buffers are laid out like ``flatten_parameters`` (64-element aligned, module order),
    so kernels that address several blocks' gradients at a constant stride still can."""

    def __init__(self, params, align: int = 64):
        self.params = list(params)
        sizes = [(p.numel() + align - 1) // align * align for p in self.params]
        dev = self.params[0].device
        self.buf = torch.zeros(max(sum(sizes), 1), dtype=torch.float32, device=dev)
        self.views, o = [], 0
        for p, n in zip(self.params, sizes):
            self.views.append(self.buf[o:o + p.numel()].view_as(p))
            o += n

    def __enter__(self):
        self.saved = [p.grad for p in self.params]
        for p, v in zip(self.params, self.views):
            p.grad = v
        return self

    def __exit__(self, *exc):
        for p, g in zip(self.params, self.saved):
            p.grad = g
        self.saved = None
        return False

    def grads(self, needs):
        """Per-parameter gradients for Function.backward (None where not needed)."""
        return tuple(v if n else None for v, n in zip(self.views, needs))


def flatten_parameters(module: torch.nn.Module, align: int = 64):
    """Re-home every parameter of ``module`` into one flat fp32 buffer (and grads
    into another).  Returns (flat_params, flat_grads)."""
    params = [p for p in module.parameters()]
    sizes = [(p.numel() + align - 1) // align * align for p in params]
    dev = params[0].device
    flat = torch.zeros(sum(sizes), dtype=torch.float32, device=dev)
    gflat = torch.zeros_like(flat)
    o = 0
    for p, n in zip(params, sizes):
        v = flat[o:o + p.numel()].view_as(p)
        v.copy_(p.data)
        p.data = v
        g = gflat[o:o + p.numel()].view_as(p)
        p._ensvs_gview = g
        p.grad = g
        o += n
    module._ensvs_flat = (flat, gflat)
    weights_updated()
    return flat, gflat


def _sig(params):
    return (_STATE["epoch"], _STATE["gemm_dtype"],
            tuple((p.data_ptr(), p._version) for p in params))


class ModulePacks:
    """Packed GEMM operands of one module.

    ``build(fn)`` calls ``fn(packs)`` to register weights (fwd / bwd / bias
    buffers) whenever parameter storage or precision changed; ``refresh``
    repacks when values changed.
    """

    def __init__(self):
        self.sig = None
        self.layout_sig = None

    def ensure(self, module, register):
        params = list(module.parameters())
        sig = _sig(params)
        if sig == self.sig:
            return self
        layout = (sig[1], tuple(p.data_ptr() for p in params))
        if layout != self.layout_sig:
            self.fwd = PackedBuffer(gemm_dtype())
            self.bwd = PackedBuffer(gemm_dtype())
            self.bias = PackedBuffer(_lib.DT_F32)
            self.refs = {}
            register(self)
            dev = params[0].device
            for pb in (self.fwd, self.bwd, self.bias):
                pb.finalize(dev)
            self.layout_sig = layout
        for pb in (self.fwd, self.bwd, self.bias):
            pb.repack()
        self.sig = sig
        return self

    # ---- registration helpers ------------------------------------------------
    def linear(self, name, w, cols=None, bwd=True, scale=1.0, perm_c=0, fwd=True):
        """Linear weight (N, K) or a column range of it (fwd=False: only its transpose)."""
        N, K = w.shape
        c0, c1 = (0, K) if cols is None else cols
        src = w[:, c0:c1]
        if fwd:
            self.refs[name] = self.fwd.add(src, N, c1 - c0, 1, K, 1, 1, perm_c=perm_c,
                                           scale=scale)
        if bwd:
            self.refs[name + "^T"] = self.bwd.add(src, N, c1 - c0, 1, K, 1, 1, transpose=True,
                                                   scale=scale)

    def linear_rows(self, name, w, rows, bwd=True, scale=1.0):
        """Row range [r0, r1) of a Linear weight as its own GEMM operand."""
        N, K = w.shape
        r0, r1 = rows
        src = w[r0:r1]
        self.refs[name] = self.fwd.add(src, r1 - r0, K, 1, K, 1, 1, scale=scale)
        if bwd:
            self.refs[name + "^T"] = self.bwd.add(src, r1 - r0, K, 1, K, 1, 1, transpose=True,
                                                   scale=scale)

    def conv(self, name, w, cols=None, bwd=True, perm_c=0, scale=1.0, bwd_rows=None,
             bwd_scale=None):
        """Conv1d weight (N, K, taps) (or input-channel range).  The backward operand is
        transposed and tap-flipped (the dgrad convolution); ``bwd_rows`` restricts it to
        output rows [r0, r1)."""
        N, K, taps = w.shape
        c0, c1 = (0, K) if cols is None else cols
        src = w[:, c0:c1]
        self.refs[name] = self.fwd.add(src, N, c1 - c0, taps, K * taps, taps, 1, perm_c=perm_c,
                                       scale=scale)
        if bwd:
            r0, r1 = (0, N) if bwd_rows is None else bwd_rows
            self.refs[name + "^T"] = self.bwd.add(
                w[r0:r1, c0:c1], r1 - r0, c1 - c0, taps, K * taps, taps, 1, transpose=True,
                flip=True, scale=scale if bwd_scale is None else bwd_scale)

    def bias_vec(self, name, b, perm_c=0, b2=None):
        N = b.shape[0]
        self.refs[name] = self.bias.add(b.view(N, 1, 1), N, 1, 1, 1, 1, 1, perm_c=perm_c,
                                        src2=None if b2 is None else b2.view(N, 1, 1), kpad_to=1)

    def __getitem__(self, name):
        return self.refs[name]

    def bias_ptr_args(self, name):
        return dict(bias=self.bias.buf, bias_off=self.refs[name].offset)


# ---- cooperative-recurrence failure flag (coop.h) ------------------------------------------
class CoopError(RuntimeError):
    """A cooperative recurrence (lstm_coop.hip / ardec.hip) could not get all workgroups of a
    sequence tile resident and timed out: its outputs of that launch are invalid.  The step
    that ran it skipped its update (the gradient norm read the flag); raised on the host by
    check_coop_errors / step_metrics / the next train_step."""


_COOP = {}  # device -> (int32 error words [live, failed steps], pinned host copy, event or None)


def _dev_key(device):
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return str(d)


def coop_error_word(device):
    """The persistent device word every cooperative launch ORs 1 into on a residency
    timeout (registered with the library on first use; one per process and device: the
    library keeps one word per device ordinal and each launch picks its current device's)."""
    key = _dev_key(device)
    ent = _COOP.get(key)
    if ent is None:
        d = torch.device(key)
        # [0]: the live word the cooperative launches OR into; [1]: failed steps, counted by
        # the step's gradient norm (ensvs_l2norm_chk snapshots [0] into [1] and clears [0])
        word = torch.zeros(2, dtype=torch.int32, device=d)
        host = torch.zeros(2, dtype=torch.int32, pin_memory=torch.cuda.is_available())
        _lib.call("ensvs_coop_set_error_word_dev", d.index, word.data_ptr())
        ent = _COOP[key] = [word, host, None]
    return ent[0]


def _coop_raise(ent):
    ent[0].zero_()
    ent[1].zero_()
    raise CoopError("ensvs: a cooperative recurrence timed out waiting for its workgroups "
                    "(grid not co-resident); the step's update was skipped (non-finite "
                    "gradient norm).  The flag is cleared; the next step runs normally.")


def check_coop_errors(device=None, sync=True):
    """Raise CoopError if a cooperative launch flagged a failure.  sync=True reads the word
    now (a device sync); sync=False only looks at the copy taken by note_coop_check() once
    the device has reached it (no wait), so the host never blocks the step pipeline."""
    for key, ent in list(_COOP.items()):
        if device is not None and key != _dev_key(device):
            continue
        if sync:
            if int(ent[0].max().item()):
                _coop_raise(ent)
        elif ent[2] is not None and ent[2].query():
            ent[2] = None
            if int(ent[1].max()):
                _coop_raise(ent)


def coop_failed(device):
    """Host read (a device sync) of the failure words: nonzero when a cooperative launch
    flagged a timeout that no step has counted yet, or a step counted one."""
    ent = _COOP.get(_dev_key(device))
    return 0 if ent is None else int(ent[0].max().item())


def note_coop_check(device):
    """Enqueue an asynchronous copy of the error word after this step's kernels (checked
    without waiting by the next check_coop_errors(sync=False))."""
    ent = _COOP.get(_dev_key(device))
    if ent is None or ent[2] is not None:
        return
    ent[1].copy_(ent[0], non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    ent[2] = ev


def empty(*shape, device, dtype=torch.float32):
    return torch.empty(*shape, dtype=dtype, device=device)


def lengths_pair(lengths, B, T, device):
    """Host list + device int64 tensor of sequence lengths (None -> all T)."""
    if lengths is None:
        host = [T] * B
    elif isinstance(lengths, torch.Tensor):
        host = [int(v) for v in lengths.detach().cpu().tolist()]
    else:
        host = [int(v) for v in lengths]
    # cached: one upload per distinct lengths vector, none inside a captured step
    key = (tuple(host), str(torch.device(device)))
    dev = _LENGTHS.get(key)
    if dev is None:
        if len(_LENGTHS) >= 256:
            for t in _LENGTHS.values():
                retire(t)
            _LENGTHS.clear()
        dev = _LENGTHS[key] = torch.tensor(host, dtype=torch.int64, device=device)
    return host, dev


_LENGTHS = {}
_RETIRED = []


def retire(t):
    """Keep a device buffer that a cache is replacing allocated for the life of the process: a
    captured step graph (train.GraphedTrainStep, kept per batch shape by train.StepGraphCache)
    may hold its address, and freeing it would let the allocator hand it to someone else."""
    _RETIRED.append(t)
