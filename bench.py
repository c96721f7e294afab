"""Throughput bench of the MI355X multi-track SVS training step.

Metric (BASELINE.json): acoustic-model train frames/sec (4-track ensemble), i.e.
main-track frames of (main, sub) pairs through forward + backward + clip + Adam
of MultiTrackNPSSMDNMultistreamParametricModel (recipe diffusion config,
23.5 M parameters, 4 speakers).  Workload per GPU: 3 SATB segments x 10 (i <= j)
pairs = 30 pairs x 1024 frames of synthetic features.
GEMMs run on bf16 MFMA with fp32 accumulation; everything else fp32.

  python bench.py [--gpus N] [--steps K] [--warmup W]
Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) each rank
runs directly; `python bench.py --gpus N` without it starts torch.distributed.run with N
ranks itself (before anything touches the GPU) and exits with its status.  RCCL gradient
all-reduce, pairs sharded per rank (weak scaling).
"""
import argparse
import json
import os
import subprocess
import sys
import time
import types

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def gate_gemm_bytes(M, C, E, a_bytes):
    """Algorithmic HBM bytes of one gate-GEMM launch as the training step issues it
    (DESIGN.md §3): A operand (x+d and cond, a_bytes each), packed weights (bf16), bias, the
    saved gate/filter pre-activations gf (M x 2C) and z (M x C) -- both in bf16 on the
    bf16 path (z: the next GEMM's operand, no fp32 copy; gf: the backward's save), fp32
    otherwise."""
    return (M * (C + E) * a_bytes + 2 * C * (3 * C + E) * 2 + 2 * C * 4 +
            M * C * a_bytes + M * 2 * C * a_bytes)
TRAIN_FLOP_PER_FRAME = 127.5e6  # SURVEY.md §6 (torch.utils.flop_counter on the oracle)
# sub-track lf0 forward the plain recipe does not need (its output is unread): BiLSTM
# 2 layers x 2 directions x 2*4*64*(128+64) + AR decoder (2*1024*(131+256) + 2*4*386) / 4
SUBTRACK_SKIPPED_FLOP = 2 * 2 * 2 * 4 * 64 * (128 + 64) + (2 * 1024 * (131 + 256) + 2 * 4 * 386) / 4
# postprocess_acoustic settings of the recipe's synthesis config
# (nnsvs/bin/conf/synthesis/synthesis/world_gv_usfgan.yaml)
SYNTH_POST = dict(frame_period=5, post_filter_type="gv", trajectory_smoothing=True,
                  trajectory_smoothing_cutoff=50, trajectory_smoothing_cutoff_f0=20,
                  vuv_threshold=0.3)


def _imports():
    """Package imports (they load libensvs.so): only after the launcher decision."""
    global np, torch, configs, data, engine, FusedAdam, GraphedTrainStep, train_step
    global set_overlap_allreduce, train_mod
    import numpy as np  # noqa: F811
    import torch  # noqa: F811
    from ensemble_svs_with_interactions_amd import configs, data, engine  # noqa: F811
    from ensemble_svs_with_interactions_amd.train import (FusedAdam, GraphedTrainStep,  # noqa
                                                          set_overlap_allreduce, train_step)
    from ensemble_svs_with_interactions_amd import train as train_mod  # noqa: F811


def launch_ranks(args):
    """`bench.py --gpus N` outside torch.distributed.run: start N ranks (one per GPU) as a
    child torch.distributed.run on 127.0.0.1 and return its exit status."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=30)
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-synth", action="store_true", help="skip the synthesis RTF leg")
    ap.add_argument("--serial", action="store_true",
                    help="run the lf0/mgc/bap/vuv branches serially (no side streams)")
    ap.add_argument("--eager", action="store_true",
                    help="issue every kernel from the host each step (no HIP graph replay)")
    ap.add_argument("--overlap-ddp", action="store_true",
                    help="with N > 1 ranks, run eager steps whose bucketed all-reduce overlaps "
                         "the backward (train.BucketedAllReduce) instead of the default: the "
                         "HIP-graph replay of the N = 1 line with one whole-buffer all-reduce "
                         "between its two graphs")
    ap.add_argument("--no-overlap-ddp", action="store_true",
                    help="(the default; kept for old command lines)")
    ap.add_argument("--no-sf0", action="store_true",
                    help="skip the recipe-default (MultiTrackMultistreamSeparateF0) leg")
    ap.add_argument("--no-census", action="store_true",
                    help="skip the per-launch census and kernel rooflines")
    ap.add_argument("--no-config2", action="store_true",
                    help="skip the single-track (BASELINE config 2) training leg")
    ap.add_argument("--no-shapes", action="store_true",
                    help="skip the 60 x 512 and ragged-length legs of the main model")
    ap.add_argument("--no-real-data", action="store_true",
                    help="skip the on-disk data-path leg (feeder + train_epoch)")
    ap.add_argument("--no-transformer", action="store_true",
                    help="skip the tier-2 Transformer encoder training leg")
    ap.add_argument("--cpu-pairs", type=int, default=10)
    ap.add_argument("--cpu-frames", type=int, default=1024)
    return ap.parse_args()


def gate_gemm_timing(model, P, T, dev, iters=20):
    """Average duration of the dominant kernel (mgc DiffNet block gate GEMM:
    M = P*T frames, N = 2C = 512, K = 3C + E = 1024) with HIP events on its stream.

    Returns (GEMM kernel seconds, seconds of the whole gate-GEMM call including the
    fp32 -> bf16 operand casts (ensvs_cast_bf16 of x + d and of cond), flops)."""
    import torch
    from ensemble_svs_with_interactions_amd import _lib, kernels as K
    net = model.mgc_model.denoise_fn
    C, E, L = net.C, net.E, len(net.residual_layers)
    M = P * T
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, C, device=dev, generator=g)
    cond = torch.randn(M, E, device=dev, generator=g)
    ds = torch.randn(P, L * C, device=dev, generator=g)
    z = torch.empty(M, C, device=dev)
    pk = net._packs.ensure(net, net._register)
    gf = torch.empty(M, 2 * C, device=dev,
                     dtype=torch.bfloat16 if K.gemm_dtype_is_bf16(pk.fwd) else torch.float32)

    def timed(fn):
        for _ in range(3):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / 1e3 / iters

    b16 = K.gemm_dtype_is_bf16(pk.fwd)
    zb = torch.empty(M, C, device=dev, dtype=torch.bfloat16) if b16 else None
    total = timed(lambda: net._gate_gemm(0, x, cond, E, ds, P, T, z, gf, zb=zb))
    dl = net.residual_layers[0].dilation
    if b16:
        # as the training step issues it: operands already bf16 (cond rounded once for all
        # blocks, x + d_l by the previous block's epilogue), z out in bf16 only
        xb = K.cast_bf16(x, C, C, M, radd=ds, radd_ld=L * C, T=T)
        cb = K.cast_bf16(cond, E, E, M)
        segs = [K.Seg(xb, C, C, pk["dil0"], T, taps=3, dil=dl, shift0=-dl),
                K.Seg(cb, E, E, pk["cond0"], T)]
        gemm = timed(lambda: K.gemm(segs, P, T, 2 * C, pk.fwd, z, C, epi=_lib.EPI_GATE, aux0=gf,
                                    ld0=2 * C, C=C, ybf=zb, ybf_ld=C, keep_y=False,
                                    **pk.bias_ptr_args("g0.b")))
    else:
        gemm = total
    flops = 2.0 * M * (2 * C) * (3 * C + E)
    return gemm, total, flops


def step_census(model, opt, batch):
    """Per-launch census of one serial, eager training step (every libensvs entry point
    bracketed by HIP events on its stream; GEMM / weight-gradient launches tagged with their
    shape, recurrences with H or T): {(entry, tag): [launches, total ms]} and the serial
    total.  Each kernel runs alone on the GPU, so these are the per-launch times a roofline
    compares against; the step itself overlaps the four branches."""
    import torch
    from ensemble_svs_with_interactions_amd import _lib, kernels as K
    import importlib
    import pkgutil
    import ensemble_svs_with_interactions_amd as pkg
    rec, tag = [], [None]
    orig_call, orig_gemm, orig_wgrad = _lib.call, K.gemm, K.wgrad

    def call(name, *args):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        orig_call(name, *args)
        e.record()
        t = tag[0]
        if name in ("ensvs_lstm_fwd", "ensvs_lstm_bwd"):
            t = f"H={args[7]} T={args[6]}"
        elif name in ("ensvs_lstm_mfma_fwd", "ensvs_lstm_mfma_bwd"):
            t = f"H={args[6]} T={args[5]}"
        elif name == "ensvs_colsum":
            t = f"M={args[2]} groups={args[3]} N={args[4]}{' centred' if args[5] else ''}"
        elif name in ("ensvs_ardec_fwd", "ensvs_ardec_coop_fwd"):  # T / 4 autoregressive steps
            t = f"H={args[15]} T={args[14]}"
        elif name in ("ensvs_ardec_bwd", "ensvs_ardec_coop_bwd"):
            t = f"H={args[10]} T={args[9]}"
        rec.append((name, t, s, e))

    def tagged(fn, fmt):
        def w(*a, **k):
            old = tag[0]
            tag[0] = fmt(*a, **k)
            try:
                return fn(*a, **k)
            finally:
                tag[0] = old
        return w

    def gemm_tag(segs, B, Tout, N, W, Y, ldy, **k):
        sg = "+".join(f"{s.K}x{s.taps}{'b' if s.x.dtype == torch.bfloat16 else 'f'}"
                      for s in segs)
        return f"gemm M={B * Tout} N={N} K=[{sg}] epi={k.get('epi', 0)}"

    def wgrad_tag(dy, ldy, x, ldx, B, Tout, Tin, N, Kc, taps, *a, **k):
        return f"wgrad M={B * Tout} N={N} K={Kc}x{taps} {'b' if dy.dtype == torch.bfloat16 else 'f'}"

    mods = [importlib.import_module(f"{pkg.__name__}.{m.name}")
            for m in pkgutil.iter_modules(pkg.__path__) if not m.name.startswith("lib")]
    patched = [m for m in mods if getattr(m, "call", None) is orig_call]
    for m in patched:
        m.call = call
    _lib.call, K.gemm, K.wgrad = call, tagged(orig_gemm, gemm_tag), tagged(orig_wgrad, wgrad_tag)
    engine.set_concurrency(False)
    try:
        torch.cuda.synchronize()
        a0 = torch.cuda.memory_stats(opt.flat.device)["allocated_bytes.all.allocated"]
        train_step(model, opt, *batch)
        torch.cuda.synchronize()
        alloc = torch.cuda.memory_stats(opt.flat.device)["allocated_bytes.all.allocated"] - a0
    finally:
        for m in patched:
            m.call = orig_call
        _lib.call, K.gemm, K.wgrad = orig_call, orig_gemm, orig_wgrad
        engine.set_concurrency(True)
    agg = {}
    for name, t, s, e in rec:
        a = agg.setdefault((name, t), [0, 0.0])
        a[0] += 1
        a[1] += s.elapsed_time(e)
    return agg, sum(v[1] for v in agg.values()), alloc


# MI355X per-CU VALU rate (fp32 FMA: one wave64 instruction per 4 cycles per SIMD) at the
# sustained MFMA clock: the issue floor of a recurrence step's dot products on its CU
CU_FMA_PER_S = 64 * 2.4e9
# one v_mfma_f32_16x16x32 (16 cycles) per SIMD, 4 SIMDs per CU
CU_MFMA16_PER_S = 4 * 2.4e9 / 16
# per AR step: handoff-flag (1.3 us, drained sc1, idle) + 16 KB payload read (~1.0 us)
COOP_HANDOFF_FLOOR_NS = 2300.0
RECURRENCES = ("ensvs_lstm_fwd", "ensvs_lstm_bwd", "ensvs_lstm_mfma_fwd", "ensvs_lstm_mfma_bwd",
               "ensvs_ardec_fwd", "ensvs_ardec_bwd", "ensvs_ardec_coop_fwd",
               "ensvs_ardec_coop_bwd")


def kernel_rooflines(agg, serial_ms, P, T, C=256, E=256):
    """Per-launch rooflines of the training step's largest kernels (census times): the mgc
    DiffNet block's five GEMM launches with their algorithmic FLOPs and HBM bytes, and the
    recurrences' ns per step against the VALU issue floor of their dot products."""
    M = P * T
    bf, f4 = 2, 4
    w = lambda n, k: n * k * bf  # noqa: E731  packed bf16 weights
    # (census tag, name, flops, algorithmic bytes) -- bytes as the production bf16 path moves
    # them: operands read once, taps re-read from cache
    shapes = [
        (("ensvs_conv_gemm_bf16a_out", f"gemm M={M} N={2 * C} K=[{C}x3b+{E}x1b] epi=1"),
         "DiffNet gate GEMM (dilated conv + conditioner, GATE epilogue)",
         2.0 * M * 2 * C * (3 * C + E),
         M * (C + E) * bf + w(2 * C, 3 * C + E) + M * 2 * C * bf + M * C * bf),
        (("ensvs_conv_gemm_bf16a_out", f"gemm M={M} N={2 * C} K=[{C}x1b] epi=2"),
         "DiffNet res/skip GEMM (output projection, RESSKIP epilogue)",
         2.0 * M * 2 * C * C,
         M * C * bf + w(2 * C, C) + 2 * M * C * f4 + M * C * bf + 2 * M * C * f4),
        (("ensvs_conv_gemm_bf16a_out", f"gemm M={M} N={C} K=[{C}x1b+{C}x1b] epi=3"),
         "DiffNet gate-backward dgrad (GATE_BWD epilogue)",
         2.0 * M * C * 2 * C,
         2 * M * C * bf + w(C, 2 * C) + M * 2 * C * bf + M * 2 * C * bf),
        (("ensvs_conv_gemm_bf16a_out", f"gemm M={M} N={C} K=[{2 * C}x3b] epi=4"),
         "DiffNet dilated-conv dgrad (ADDSCALE epilogue)",
         2.0 * M * C * 2 * C * 3,
         M * 2 * C * bf + w(C, 6 * C) + 2 * M * C * f4 + M * C * bf),
        (("ensvs_conv_wgrad_bf16", f"wgrad M={M} N={2 * C} K={C}x3 b"),
         "DiffNet dilated-conv weight gradient",
         2.0 * M * 2 * C * C * 3, M * 2 * C * bf + M * C * bf + 2 * C * 3 * C * f4),
    ]
    out = []
    for key, name, flops, nbytes in shapes:
        n, ms = agg.get(key, (0, 0.0))
        if not n:
            continue
        sec = ms / n / 1e3
        tf, gbs = flops / sec / 1e12, nbytes / sec / 1e9
        mfma = flops / (PEAK_BF16_TFLOPS * 1e12) >= nbytes / (PEAK_HBM_GBS * 1e9)
        out.append({"kernel": name, "tag": key[1], "launches_per_step": n,
                    "us_per_launch": sec * 1e6, "flops": flops, "algorithmic_bytes": nbytes,
                    "bound": "mfma" if mfma else "hbm",
                    "achieved": tf if mfma else gbs, "unit": "TFLOP/s" if mfma else "GB/s",
                    "peak": PEAK_BF16_TFLOPS if mfma else PEAK_HBM_GBS,
                    "frac": tf / PEAK_BF16_TFLOPS if mfma else gbs / PEAK_HBM_GBS,
                    "share_of_serial_step": ms / serial_ms})
    rec = []
    for (name, tag), (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        if name not in RECURRENCES or not tag:
            continue
        kv = dict(p.split("=") for p in tag.split())
        H, steps = int(kv["H"]), int(kv["T"])
        ent = {"kernel": f"{name[6:]} H={H}", "launches_per_step": n,
               "share_of_serial_step": ms / serial_ms}
        if name.startswith("ensvs_lstm_mfma"):
            # h_{t-1} W_hh^T (fwd) / dG W_hh (bwd) of one sequence-direction as 16x16x32 MFMAs
            # (4H/16 x H/32 of them, one useful row), spread over the CU's 4 SIMDs
            floor_ns = (4 * H // 16) * (H // 32) / CU_MFMA16_PER_S * 1e9
            ent["floor"] = ("MFMA issue of the recurrent product on one CU (one workgroup per "
                            "sequence-direction; 16x16x32 tiles, the h / dG vector in every "
                            "row: one useful row)")
        elif name.startswith("ensvs_lstm"):
            floor_ns = 4 * H * H / CU_FMA_PER_S * 1e9
            ent["floor"] = ("VALU fp32 FMA issue of the recurrent dot products on one CU "
                            "(latency-bound: one workgroup per sequence-direction)")
        elif "coop" in name:
            steps //= 4  # r = 4 frames per AR step
            floor_ns = COOP_HANDOFF_FLOOR_NS
            ent["floor"] = ("per-step all-to-all hand-off of h / dG among the H/16 workgroups "
                            "(coop.h): MI355X_MICROARCH.md price list, handoff-flag with drained "
                            "sc1 stores 1.3 us idle + the 16 KB slab read latency-bound at "
                            "~16 GB/s per consumer (handoff-payload) 1.0 us; the step's MFMA "
                            "work (4H/16 x 4 tiles per workgroup) hides under the read")
        else:
            # LSTMCell W_hh + the prenet column of W_ih + feat_out per AR step (r = 4 frames)
            steps //= 4
            floor_ns = (4 * H * H + 4 * H + 4 * (H + 130)) / CU_FMA_PER_S * 1e9
            ent["floor"] = "VALU fp32 FMA issue of one AR step on one CU"
        ns = ms / n * 1e6 / steps
        ent.update(ns_per_step=ns, floor_ns_per_step=floor_ns,
                   frac=floor_ns / ns if floor_ns else None)
        rec.append(ent)
    return out, rec


def _median_time(fn, reps):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.time()
        out = fn()
        torch.cuda.synchronize()
        ts.append(time.time() - t0)
    return float(np.median(ts)), out


ACOUSTIC_INFER_FLOP_PER_FRAME = 3.01e9  # 100 reverse-diffusion steps
VOCODER_FLOP_PER_FRAME = 4.68e6 * 240   # uSFGAN 4.68 MFLOP/sample x 240 samples/frame


def _timing_models(dev):
    """The recipe's multi-track time-lag and duration MDN models (random init) and scalers
    fitted on synthetic statistics (the reference fits them on the corpus)."""
    from ensemble_svs_with_interactions_amd import scalers
    rng = np.random.default_rng(11)
    out = {}
    for name, mu, sd in (("timelag", 0.0, 3.0), ("duration", 12.0, 6.0)):
        m = configs.instantiate(configs.multitrack_timing(name, num_speaker=4)).to(dev).eval()
        fit = rng.random((1000, 82))
        ins = scalers.MinMaxScaler(-fit.min(0) / np.ptp(fit, 0), 1.0 / np.ptp(fit, 0),
                                   fit.min(0), fit.max(0))
        outs = scalers.StandardScaler(np.array([mu]), np.array([sd * sd]))
        out[name] = (m, (ins, outs))
    return out


# tools/synth_pmc.py: called before and after the measured passes of one synthesis case
SYNTH_MARK = None


def synth_rtf(model, dev, T=2000, parts=6, reps=3, only=None):
    """Synthesis real-time factor (BASELINE metric part 2 and config 5):
    elapsed / audio seconds (svs.py:449-452, 581-582) of the pipeline of
    synthesis_multitrack.py:113-288 -- timing inference (time-lag + duration MDN models with
    the onset merge and duration fitting of gen.py:214-1006, per ordered pair), acoustic
    inference (pad_inference_multitrack, free-running AR log-F0, 100-step reverse diffusion
    for mgc and bap, V/UV), the output inverse scaling + postprocess_acoustic (GV,
    WORLD F0 stream, trajectory smoothing; gen.py:1299, 1314-1530) + predict_waveform's
    uSFGAN input preparation (aperiodicity codec round trip, f0; gen.py:1637-1694) and the
    uSFGAN generator -- for one (main, sub) pair of T frames
    (5 ms), for a `parts`-part ensemble (every part paired with its neighbour) batched in
    one acoustic/vocoder pass, and for the reference's ordered-pair sweep (every part with
    every partner, itself included: parts^2 pairs).  The acoustic input frames are
    synthetic features of the song length (the reference's ground-truth-duration path:
    its predicted-timing path fails, Appendix A-12); timing runs on synthetic score tracks
    and its output labels are not fed back into frame features (nnmnkwii frame feature
    extraction is out of scope; the score-pitch column of the input features stands in for
    the note frames).  Scaler statistics are synthetic."""
    from ensemble_svs_with_interactions_amd import postprocess, scalers, synthesis, usfgan
    torch.manual_seed(7)
    voc = configs.instantiate(configs.usfgan_generator()).to(dev)
    voc.remove_weight_norm()  # as load_vocoder does (nnsvs/util.py:412-414)
    wrapper = usfgan.USFGANWrapper({"data": dict(configs.USFGAN_DATA),
                                    "generator": {"aux_context_window": 2}}, voc)
    tm = _timing_models(dev)
    score = data.synthetic_score(99, parts, T)
    spk_of = [p % 4 for p in range(parts)]
    model.eval()
    sc, mu = configs.LF0_STATS["out_lf0_scale"], configs.LF0_STATS["out_lf0_mean"]
    # output statistics: unit variance except the log-F0 stream (synthetic; var_ doubles as
    # the GV target of the mgc post-filter)
    mean_, var_ = np.zeros(67), np.full(67, 0.25)
    mean_[60], var_[60] = mu, sc * sc
    out_scaler = scalers.StandardScaler(mean_, var_)
    stream_cfg = types.SimpleNamespace(stream_sizes=[60, 1, 1, 5], num_windows=1,
                                       has_dynamic_features=[False] * 4)
    out = {}
    for name, pairs in (("pair", [(0, 1)]),
                        (f"ensemble_{parts}part", [(i, (i + 1) % parts) for i in range(parts)]),
                        (f"n2_sweep_{parts}part", [(i, j) for i in range(parts)
                                                   for j in range(parts)])):
        if only is not None and name != only:
            continue
        B = len(pairs)
        b = data.synthetic_batch(B, T, 4242 + B)
        g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
        xm, xs, s0, s1 = g("x_main"), g("x_sub"), g("spk_main"), g("spk_sub")

        def timing():
            res = []
            for i, j in pairs:
                res.append(synthesis.predict_timing_multitrack(
                    tm["timelag"][0], tm["duration"][0], [score[i], score[j]],
                    [spk_of[i], spk_of[j]], tm["timelag"][1], tm["duration"][1],
                    device=dev))
            return res

        def acoustic():
            return model.inference(xm, xs, spks=(s0, s1), lengths=[T] * B)

        def vocoder(feats):
            # predict_acoustic's inverse scaling (gen.py:1299), postprocess_acoustic
            # (gen.py:1314-1530: GV on note frames, WORLD F0 stream, 50 / 20 Hz trajectory
            # smoothing, bap clip) and predict_waveform's uSFGAN inputs (gen.py:1637-1694)
            # per track on the device, then one batched generator pass
            f0s, auxs = [], []
            for bi in range(B):
                f = feats[bi].clone()
                postprocess.inverse_transform(out_scaler, f)
                streams = postprocess.postprocess_acoustic(
                    dev, f, xm[bi], {}, {}, stream_cfg, out_scaler, pitch_idx=51,
                    **SYNTH_POST)
                f0, aux = postprocess.usfgan_inputs(
                    *streams, sine_f0_type=configs.USFGAN_DATA["sine_f0_type"],
                    vuv_threshold=SYNTH_POST["vuv_threshold"])
                f0s.append(f0)
                auxs.append(aux)
            return wrapper.inference_batch(torch.cat(f0s, 1).t().contiguous(),
                                           torch.stack(auxs))

        timing()
        feats = acoustic()  # warm-up (weight packing, graph capture)
        vocoder(feats)
        if SYNTH_MARK is not None:
            SYNTH_MARK()
        tt, _ = _median_time(timing, reps)
        ta, feats = _median_time(acoustic, reps)
        tv, wav = _median_time(lambda: vocoder(feats), reps)
        if SYNTH_MARK is not None:
            SYNTH_MARK()
        assert torch.isfinite(wav).all()
        sec = T * 0.005
        flops = B * T * (ACOUSTIC_INFER_FLOP_PER_FRAME + VOCODER_FLOP_PER_FRAME)
        # rtf: wall-clock / seconds of the song (the whole ensemble rendered);
        # rtf_per_track: wall-clock / seconds of synthesized audio (B tracks), the
        # reference's per-synthesis definition (svs.py:449-452, 581-582)
        out[name] = dict(rtf=(tt + ta + tv) / sec, rtf_per_track=(tt + ta + tv) / (B * sec),
                         timing_ms=tt * 1e3, acoustic_ms=ta * 1e3, vocoder_ms=tv * 1e3,
                         tracks=B, samples_per_track=int(wav.shape[-1]),
                         model_tflops_per_s=flops / (ta + tv) / 1e12)
    model.train()
    ens = out[f"ensemble_{parts}part"]
    achieved = ens["model_tflops_per_s"]
    return dict(metric="synth RTF (timing + acoustic inference + uSFGAN) / audio seconds",
                frames=T, audio_s=T * 0.005, diffusion_steps=100, higher_is_better=False,
                dtype=engine.gemm_precision(), **out,
                roofline={"bound": "mfma", "achieved": achieved, "peak": PEAK_BF16_TFLOPS,
                          "unit": "TFLOP/s", "frac": achieved / PEAK_BF16_TFLOPS,
                          "traffic": _committed("r4_synth_pmc.json", "hbm_bytes_per_step"),
                          "traffic_source": "profiles/r4_synth_pmc.json (rocprofv3 --pmc "
                                            "FETCH_SIZE x2 + WRITE_SIZE over one ensemble pass: "
                                            "timing + acoustic + post-processing + uSFGAN; "
                                            "tools/synth_pmc.py; committed, not this run)",
                          "work": f"ensemble_{parts}part acoustic inference "
                                  f"({ACOUSTIC_INFER_FLOP_PER_FRAME / 1e9:.2f} GFLOP/frame) + "
                                  f"uSFGAN ({VOCODER_FLOP_PER_FRAME / 1e9:.2f} GFLOP/frame), "
                                  "GEMM/conv FLOPs of the whole pipeline over its wall time"})


def cpu_synth_baseline(T=2000):
    """The oracle's synthesis of one (main, sub) pair on the host cores: multi-track
    acoustic inference (100 reverse-diffusion steps) + uSFGAN, full-size random weights,
    T frames; RTF = elapsed / (T * 5 ms).  The GPU leg's length (synth_rtf, T = 2000 =
    10 s of audio: about 20 s of CPU work on 16 cores), so the two RTFs compare like for
    like (the reference probe: acoustic RTF 0.776 at T = 2000, uSFGAN 0.70 at 1 s)."""
    from oracle import ensvs_oracle as O
    from oracle import usfgan_oracle as U
    from oracle.weights import seeded_state_dict
    cfg = configs.multitrack_diffusion(num_speakers=4)
    m = configs.instantiate(cfg)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    del m
    P = {k: torch.from_numpy(v) for k, v in seeded_state_dict(shapes, 1).items()}
    for pre in ("mgc_model.", "bap_model."):
        for k, v in O.diffusion_schedule().items():
            P[pre + k] = v
    vm = configs.instantiate(configs.usfgan_generator())
    vshapes = {k: tuple(v.shape) for k, v in vm.state_dict().items()}
    del vm
    PV = {k: torch.from_numpy(v) for k, v in seeded_state_dict(vshapes, 2).items()}
    b = data.synthetic_batch(1, T, 5)
    rng = torch.Generator().manual_seed(5)
    Tp = T + 4 - T % 4
    t0 = time.time()
    with torch.no_grad():
        feats = O.model_inference(
            P, cfg, torch.from_numpy(b["x_main"]), torch.from_numpy(b["x_sub"]),
            (torch.from_numpy(b["spk_main"]), torch.from_numpy(b["spk_sub"])), [T],
            (torch.rand(1, Tp // 4, 1, generator=rng) < 0.5).float() * 2,
            torch.randn(101, 1, 1, 60, Tp, generator=rng),
            torch.randn(101, 1, 1, 5, Tp, generator=rng), fast=True)
        ta = time.time() - t0
        sc, mu = configs.LF0_STATS["out_lf0_scale"], configs.LF0_STATS["out_lf0_mean"]
        f0 = torch.exp(feats[0, :, 60:61] * sc + mu).numpy()
        aux = torch.cat([feats[0, :, :60], feats[0, :, 62:67]], -1)
        L = T * configs.USFGAN_DATA["hop_size"]
        t1 = time.time()
        wav = U.usfgan_inference(PV, f0, aux, torch.randn(1, 1, L, generator=rng),
                                 torch.randn(1, 1, L, generator=rng))
        tv = time.time() - t1
    assert torch.isfinite(wav).all()
    sec = T * 0.005
    return dict(value=(ta + tv) / sec, unit="RTF (lower is better)",
                cores=torch.get_num_threads(), kind="port", acoustic_s=ta, vocoder_s=tv,
                sample=f"oracle multi-track pair inference (100 diffusion steps) + uSFGAN "
                       f"oracle, {T} frames = {sec:.1f} s of audio, fp32, one run")


def _cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for ln in out.splitlines():
            if ln.startswith("Model name"):
                return ln.split(":", 1)[1].strip()
    except Exception:
        pass
    import platform
    return platform.processor() or "unknown"


def _host_cores():
    cores = os.cpu_count() or 1
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    return min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))


def cpu_baseline(args):
    """The oracle (CPU PyTorch restatement of the reference, fused CPU LSTM) on the host
    cores, BASELINE.md §3: full-size model, P pairs x T frames fp32 (10 x
    1024), median of 5 steps after 2 warm-up steps.  tools/cpu_baseline_check.py pins its
    speed to the reference's own train_step."""
    from oracle import ensvs_oracle as O
    from oracle.weights import seeded_state_dict
    cores = _host_cores()
    torch.set_num_threads(cores)
    cfg = configs.multitrack_diffusion(num_speakers=4)
    model = configs.instantiate(cfg)
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    del model
    P = {k: torch.from_numpy(v) for k, v in seeded_state_dict(shapes, 1).items()}
    for pre in ("mgc_model.", "bap_model."):
        for k, v in O.diffusion_schedule().items():
            P[pre + k] = v
    trainable = [k for k in P if "running" not in k and k.rsplit(".", 1)[-1] not in
                 O.diffusion_schedule()]
    Pp, T = args.cpu_pairs, args.cpu_frames
    b = data.synthetic_batch(Pp, T, 7)
    x = (torch.from_numpy(b["x_main"]), torch.from_numpy(b["x_sub"]))
    y = (torch.from_numpy(b["y_main"]), torch.from_numpy(b["y_sub"]))
    spk = (torch.from_numpy(b["spk_main"]), torch.from_numpy(b["spk_sub"]))
    rng = torch.Generator().manual_seed(3)
    state, times = {}, []
    warm, timed = 2, 5
    for step in range(warm + timed):
        for k in trainable:
            P[k] = P[k].detach().requires_grad_()
        draws = dict(
            lf0_main=(torch.rand(Pp, T // 4, 1, generator=rng) < 0.5).float() * 2,
            lf0_sub=(torch.rand(Pp, T // 4, 1, generator=rng) < 0.5).float() * 2,
            mgc_t=torch.randint(0, 100, (Pp,), generator=rng),
            mgc_noise=torch.randn(Pp, 1, 60, T, generator=rng),
            bap_t=torch.randint(0, 100, (Pp,), generator=rng),
            bap_noise=torch.randn(Pp, 1, 5, T, generator=rng),
            vuv_lstm=[(torch.rand(Pp, T, 128, generator=rng) > 0.1).float() / 0.9])
        t0 = time.time()
        preds, _ = O.model_forward(P, cfg, x[0], x[1], spk, b["lengths"], y, draws,
                                   bn_updates={}, fast=True)
        loss = O.masked_l1_loss(preds, y[0], b["lengths"], cfg["stream_sizes"])
        loss.backward()
        grads = {k: P[k].grad for k in trainable}
        params = {k: P[k].detach() for k in trainable}
        O.clip_and_adam(params, grads, state, step=step + 1)
        P.update(params)
        times.append(time.time() - t0)
    sec = float(np.median(times[warm:]))
    return dict(value=Pp * T / sec, unit="main-track frames/s", cores=cores, kind="port",
                cpu_model=_cpu_model(),
                sample=f"oracle (CPU PyTorch restatement, fused CPU LSTM) full-size model, "
                       f"{Pp} pairs x {T} frames fp32, median of {timed} steps after {warm} "
                       f"warm-up ({sum(times):.1f} s of CPU work)")


def il_train(args, dev):
    """BASELINE config 3 with the interaction-loss recipe (myconfig_useIL /
    multitrack_acoustic_nnsvs_world_multi_ar_f0_diff_mgcbap_subtrack.yaml): output_subtrack
    model (sub-track lf0 decoded and trained too) and the log-F0 difference loss
    (logf0_diff_weight 0.5, train_acoustic_multitrack.py:175-182); same workload shape,
    graph replay."""
    torch.manual_seed(20250323)
    model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4,
                                                             output_subtrack=True)).to(dev)
    opt = FusedAdam(model, lr=1e-4, clip_norm=1.0)
    P, T = args.pairs, args.frames
    b = data.synthetic_batch(P, T, 3000)
    g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
    step = GraphedTrainStep(model, opt, g("x_main"), g("x_sub"), g("y_main"), g("spk_main"),
                            g("spk_sub"), b["lengths"].tolist(), warmup=1, y_sub=g("y_sub"),
                            logf0_diff_weight=0.5).step
    for _ in range(max(0, args.warmup - 1)):
        step()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(args.steps):
        loss, norm = step()
    torch.cuda.synchronize()
    el = time.time() - t0
    return dict(metric="acoustic-model train frames/sec, interaction-loss recipe (output_subtrack,"
                       " logf0_diff_weight 0.5)", value=P * T * args.steps / el,
                unit="main-track frames/s", ms_per_step=el / args.steps * 1e3, steps=args.steps,
                pairs=P, frames=T, dtype=engine.gemm_precision(), train_loss=loss.item(),
                grad_norm=norm.item())


SF0_TRAIN_FLOP_PER_FRAME = 276.5e6  # SURVEY.md section 6 (torch.utils.flop_counter on the oracle)


def _graphed_leg(model, opt, P, T, seed, steps, lengths=None, warmup=1):
    """Graph-replayed training steps of `model` on a synthetic P x T batch (optionally ragged
    `lengths`, fixed across steps): (ms per step, valid main-track frames per step, loss,
    grad norm)."""
    b = data.synthetic_batch(P, T, seed, lengths=lengths)
    g = lambda k: torch.from_numpy(b[k]).to(opt.flat.device).contiguous()  # noqa: E731
    step = GraphedTrainStep(model, opt, g("x_main"), g("x_sub"), g("y_main"), g("spk_main"),
                            g("spk_sub"), b["lengths"].tolist(), warmup=1).step
    for _ in range(max(0, warmup - 1)):
        step()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(steps):
        loss, norm = step()
    torch.cuda.synchronize()
    el = time.time() - t0
    return el / steps * 1e3, int(b["lengths"].sum()), loss.item(), norm.item()


def sf0_train(args, dev, steps=4):
    """The recipe's default acoustic model (MultiTrackMultistreamSeparateF0ParametricModel,
    multitrack_acoustic_nnsvs_world_multi_ar_f0.yaml; config.yaml:93-95): concatenation-fusion
    MultiTrackLSTMEncoder (H = 512 x 3 layers), teacher-forced multi-track lf0 model, main
    and sub FFConvLSTM decoders (H = 256 / 64 / 62), masked L1 over the main output; same
    per-GPU workload, graph replay, bf16 GEMM operands, and the same 30 720 frames as 60
    pairs x 512 (two 32-sequence tiles of the cooperative recurrences).  276.5 MFLOP per
    frame."""
    torch.manual_seed(20250324)
    model = configs.instantiate(configs.multitrack_separate_f0(num_speakers=4)).to(dev)
    opt = FusedAdam(model, lr=1e-4, clip_norm=1.0)
    P, T = args.pairs, args.frames
    ms, frames, loss, norm = _graphed_leg(model, opt, P, T, 4000, steps)
    v = frames / ms * 1e3
    tf = v * SF0_TRAIN_FLOP_PER_FRAME / 1e12
    out = dict(metric="recipe-default acoustic model train frames/sec (SeparateF0, "
                      "MultiTrackLSTMEncoder H=512)", value=v, unit="main-track frames/s",
               ms_per_step=ms, steps=steps, pairs=P, frames=T, dtype=engine.gemm_precision(),
               train_loss=loss, grad_norm=norm, model_tflops_per_s=tf,
               roofline={"bound": "mfma", "achieved": tf, "peak": PEAK_BF16_TFLOPS,
                         "unit": "TFLOP/s", "frac": tf / PEAK_BF16_TFLOPS, "traffic": None,
                         "work": f"{SF0_TRAIN_FLOP_PER_FRAME / 1e6:.1f} MFLOP per main-track "
                                 "frame (forward + backward GEMM / conv / LSTM FLOPs, SURVEY.md "
                                 "section 6) x frames/s"})
    P2, T2 = 2 * P, T // 2
    ms2, frames2, loss2, norm2 = _graphed_leg(model, opt, P2, T2, 4001, steps)
    out[f"p{P2}x{T2}"] = dict(value=frames2 / ms2 * 1e3, ms_per_step=ms2, pairs=P2, frames=T2,
                              train_loss=loss2, grad_norm=norm2,
                              ratio_to_p30=(frames2 / ms2) / (frames / ms))
    return out


def sf0_cpu_baseline(pairs=4, frames=512, warm=1, timed=3):
    """The oracle's SeparateF0 training step (separate_f0_forward with teacher forcing, the
    main output's masked L1, backward, clip + Adam) on the host cores: a bounded sample of
    the leg's workload (the CPU needs ~7 s per 2 048-frame step)."""
    from oracle import ensvs_oracle as O
    from oracle.weights import seeded_state_dict
    cores = _host_cores()
    torch.set_num_threads(cores)
    cfg = configs.multitrack_separate_f0(num_speakers=4)
    model = configs.instantiate(cfg)
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    del model
    P = {k: torch.from_numpy(v) for k, v in seeded_state_dict(shapes, 2).items()}
    trainable = [k for k in P if "running" not in k and "num_batches" not in k]
    b = data.synthetic_batch(pairs, frames, 9)
    x = [torch.from_numpy(b[k]) for k in ("x_main", "x_sub")]
    y = [torch.from_numpy(b[k]) for k in ("y_main", "y_sub")]
    spk = (torch.from_numpy(b["spk_main"]), torch.from_numpy(b["spk_sub"]))
    rng = torch.Generator().manual_seed(4)
    state, times = {}, []
    for step in range(warm + timed):
        for k in trainable:
            P[k] = P[k].detach().requires_grad_()
        draws = dict(lf0_main=(torch.rand(pairs, frames // 4, 1, generator=rng) < 0.5).float() * 2,
                     lf0_sub=(torch.rand(pairs, frames // 4, 1, generator=rng) < 0.5).float() * 2)
        t0 = time.time()
        (om, _), _ = O.separate_f0_forward(P, cfg, x[0], x[1], spk, b["lengths"].tolist(), y,
                                           draws, training=True, bn_updates={}, fast=True)
        loss = O.masked_l1_loss(O.split_streams(om, cfg["stream_sizes"]), y[0], b["lengths"],
                                cfg["stream_sizes"])
        loss.backward()
        grads = {k: P[k].grad for k in trainable if P[k].grad is not None}
        params = {k: P[k].detach() for k in grads}
        O.clip_and_adam(params, grads, state, step=step + 1)
        P.update(params)
        times.append(time.time() - t0)
    sec = float(np.median(times[warm:]))
    return dict(value=pairs * frames / sec, unit="main-track frames/s", cores=cores, kind="port",
                cpu_model=_cpu_model(),
                sample=f"oracle SeparateF0 step (CPU PyTorch restatement, fused CPU LSTM), "
                       f"{pairs} pairs x {frames} frames fp32, median of {timed} steps after "
                       f"{warm} warm-up ({sum(times):.1f} s of CPU work)")


def shape_legs(args, dev, model, opt, base_ms, steps=5):
    """The main line's model at other batch shapes of the same workload size (graph replay):
    60 pairs x 512 frames (the recipe's batch_by_size packs up to 32 000 frames, so short
    pairs come 60+ to a batch: two 32-sequence tiles of the cooperative AR decoder) and the
    30 x 1024 batch with ragged lengths U[T/2, T] (multiples of 4; the recurrences run to
    each sequence's own length, the per-frame kernels over the padded batch)."""
    P, T = args.pairs, args.frames
    out = {}
    # the main batch issued eagerly (every launch from the host): graph replay's gain
    b = data.synthetic_batch(P, T, 1499)
    g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
    args_e = (g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub"),
              b["lengths"].tolist())
    train_step(model, opt, *args_e)
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(steps):
        loss, norm = train_step(model, opt, *args_e)
    torch.cuda.synchronize()
    ms = (time.time() - t0) / steps * 1e3
    out[f"eager_p{P}x{T}"] = dict(value=P * T / ms * 1e3, ms_per_step=ms, pairs=P, frames=T,
                                  execution="eager train_step (host issues every launch)",
                                  train_loss=loss.item(), ratio_to_main=base_ms / ms)
    ms, frames, loss, norm = _graphed_leg(model, opt, 2 * P, T // 2, 1500, steps)
    out[f"p{2 * P}x{T // 2}"] = dict(value=frames / ms * 1e3, ms_per_step=ms, pairs=2 * P,
                                     frames=T // 2, train_loss=loss, grad_norm=norm,
                                     ratio_to_main=base_ms / ms)
    # long segments: the multitrack pairing never filters them (train_util.py:160-166 hard-codes
    # filter_long_segments=False), so 4096-step recurrences reach the step;
    # 15 x 2048 is the on-disk leg's longest bucket shape (songs of up to 2 048 frames)
    for PL, TL, seed in ((15, 2048, 1503), (8, 4096, 1502)):
        ms, frames, loss, norm = _graphed_leg(model, opt, PL, TL, seed, steps)
        out[f"p{PL}x{TL}"] = dict(value=frames / ms * 1e3, ms_per_step=ms, pairs=PL, frames=TL,
                                  train_loss=loss, grad_norm=norm,
                                  ratio_to_main=(frames / ms) / (P * T / base_ms))
    rng = np.random.default_rng(8)
    lens = (rng.integers(T // 2, T + 1, size=P) // 4) * 4
    ms, frames, loss, norm = _graphed_leg(model, opt, P, T, 1501, steps, lengths=lens)
    out[f"ragged_p{P}x{T}"] = dict(
        value=frames / ms * 1e3, unit="valid main-track frames/s", ms_per_step=ms,
        padded_frames_per_s=P * T / ms * 1e3, valid_fraction=frames / (P * T), pairs=P,
        frames=T, lengths="U[T/2, T], multiples of 4", train_loss=loss, grad_norm=norm,
        ratio_to_main=(frames / ms) / (P * T / base_ms))
    return out


def real_data_train(args, dev, segments=24, epochs=2, batch_max_frames=32000):
    """The path a user runs (train_acoustic_multitrack.py:461-563): synthetic on-disk
    `-feats.npy` corpus (4 SATB parts x `segments` songs, lengths U[256, 2048] per song),
    file pairing, shuffled batch_by_size(32 000 frames) buckets, PairBatchFeeder (reader
    thread -> pinned buffers -> copy stream) and train.train_epoch (eager: every batch has
    its own shape).  One untimed epoch, then `epochs` timed ones."""
    import tempfile
    from ensemble_svs_with_interactions_amd import loader
    from ensemble_svs_with_interactions_amd.train import StepGraphCache, train_epoch
    rng = np.random.default_rng(21)
    spks = ["S", "A", "T", "B"]
    with tempfile.TemporaryDirectory() as root:
        dirs = {k: os.path.join(root, "dump", s, d) for k, s, d in
                (("in", "norm", "in_acoustic"), ("out", "norm", "out_acoustic"),
                 ("times", "org", "in_acoustic"))}
        for d in dirs.values():
            os.makedirs(d)
        for i in range(segments):
            n = int(rng.integers(256, 2049))
            sb = data.synthetic_batch(4, n, 7000 + i)
            for j, spk in enumerate(spks):
                seg = f"song_{i:03d}"
                np.save(os.path.join(dirs["in"], f"{spk}_{seg}-feats.npy"), sb["x_main"][j])
                np.save(os.path.join(dirs["out"], f"{spk}_{seg}-feats.npy"), sb["y_main"][j])
                np.save(os.path.join(dirs["times"], f"{spk}_{seg}-times.npy"),
                        np.arange(5) * 50000)
        torch.manual_seed(20250325)
        model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev)
        opt = FusedAdam(model, lr=1e-4, clip_norm=1.0)
        np.random.seed(1)
        ds, batches = loader.setup_multitrack_batches(dirs["in"], dirs["out"], spks,
                                                      batch_max_frames=batch_max_frames,
                                                      allow_cache=True)
        feeder = loader.PairBatchFeeder(ds, batches, device=dev)
        valid = sum(max(ds.lengths[i]) for b in batches for i in b)
        padded = sum(len(b) * max(max(ds.lengths[i]) for i in b) for b in batches)
        # epoch 1 (untimed): every bucket's step runs eagerly once and is captured
        # (train.StepGraphCache); the timed epochs replay the captured steps
        graphs = StepGraphCache(model, opt)
        t0 = time.time()
        train_epoch(model, opt, feeder, graphs=graphs)
        torch.cuda.synchronize()
        el_first = time.time() - t0
        t0 = time.time()
        w0 = feeder.wait_s
        for _ in range(epochs):
            res = train_epoch(model, opt, feeder, graphs=graphs)
        torch.cuda.synchronize()
        el = (time.time() - t0) / epochs
        feeder_wait = (feeder.wait_s - w0) / epochs
        # the same epochs issued eagerly (every launch from the host), for the host-issue cost
        t0 = time.time()
        for _ in range(epochs):
            train_epoch(model, opt, feeder)
        torch.cuda.synchronize()
        el_eager = (time.time() - t0) / epochs
        # the same shapes at fixed-shape speed: each bucket's captured step replayed back to
        # back on its static batch (real updates), weighted by its batches per epoch -- what an
        # epoch costs with no loop at all around the steps (feeder, copies, cache lookup)
        fixed = 0.0
        reps = 3
        buckets = []
        for key, g in graphs.graphs.items():
            g.step()
            torch.cuda.synchronize()
            t0 = time.time()
            for _ in range(reps):
                g.step()
            torch.cuda.synchronize()
            dt = (time.time() - t0) / reps
            per_epoch = graphs.uses[key] / (1 + epochs)
            fixed += dt * per_epoch
            lens_k = key[5]
            buckets.append(dict(pairs=len(lens_k), frames=key[0][0][1],
                                valid_frames=int(sum(lens_k)), ms_per_step=dt * 1e3,
                                frames_per_s=sum(lens_k) / dt, steps_per_epoch=per_epoch))
        buckets.sort(key=lambda b: -b["frames"])
        n_graphs, reserved = len(graphs.graphs), torch.cuda.memory_reserved(dev)
        del graphs
        feeder.close()
    sizes = [len(b) for b in batches]
    return dict(metric="acoustic-model train frames/sec on the on-disk data path (feeder + "
                       "train_epoch, ragged dynamic batches)",
                value=valid / el, unit="main-track frames/s (pair length max(L_main, L_sub))",
                padded_frames_per_s=padded / el, s_per_epoch=el, steps_per_epoch=len(batches),
                pairs=sum(sizes), pairs_per_batch=[min(sizes), max(sizes)],
                batch_max_frames=batch_max_frames, lengths="U[256, 2048] per song",
                execution="train.StepGraphCache: one captured step per batch_by_size bucket "
                          "(captured in the untimed first epoch, replayed from then on), all "
                          "graphs in one shared memory pool",
                first_epoch_s=el_first, captured_signatures=n_graphs,
                feeder_wait_s_per_epoch=feeder_wait,
                memory_reserved_gb=reserved / 1e9,
                eager_value=valid / el_eager, eager_s_per_epoch=el_eager,
                same_shapes_back_to_back_s_per_epoch=fixed,
                ratio_to_same_shapes_back_to_back=fixed / el,
                buckets=buckets,
                last_loss=float(res[-1][0].item()), dtype=engine.gemm_precision())


TF_CFG = dict(in_dim=87, out_dim=67, hidden_dim=256, attention_dim=1024, num_heads=2,
              num_layers=2, kernel_size=3, dropout=0.1)


def transformer_flops(B, T, cfg=TF_CFG):
    """Forward GEMM / attention FLOPs of TransformerEncoder (nnsvs/model.py:1540-1671) on B x T
    frames: fc, per layer the q / k / v / o projections, QK^T and PV (T x T per head), the
    relative-key / value band (2w + 1 = 9 per row) and the two k-tap FFN convolutions, fc_out."""
    M, C, F, k = B * T, cfg["hidden_dim"], cfg["attention_dim"], cfg["kernel_size"]
    per_layer = 4 * 2 * M * C * C + 2 * 2 * B * T * T * C + 2 * 2 * M * 9 * C \
        + 2 * 2 * M * C * F * k
    return 2 * M * cfg["in_dim"] * C + cfg["num_layers"] * per_layer + 2 * M * C * cfg["out_dim"]


def transformer_train(dev, B=8, T=1024, steps=10, warm=3):
    """Tier-2 Transformer encoder (no recipe instantiates it, so
    the reference's constructor defaults at acoustic-model widths: hidden 256, FFN filter
    1 024, 2 heads, 2 layers, kernel 3, dropout 0.1): training steps (forward with dropout,
    backward through autograd, clip + Adam) on B x T ragged frames, eager issue."""
    from ensemble_svs_with_interactions_amd.transformer import TransformerEncoder
    torch.manual_seed(20250326)
    mod = TransformerEncoder(**TF_CFG).to(dev)
    mod.train()
    opt = FusedAdam(mod, lr=1e-4, clip_norm=1.0)
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(B, T, TF_CFG["in_dim"], device=dev, generator=g)
    y = torch.randn(B, T, TF_CFG["out_dim"], device=dev, generator=g)
    lens = [T - 64 * (i % 4) for i in range(B)]
    mask = torch.zeros(B, T, 1, device=dev)
    for i, n in enumerate(lens):
        mask[i, :n] = 1.0

    denom = mask.sum() * TF_CFG["out_dim"]

    def grads():
        opt.zero_grad()
        out = mod(x, lens)
        loss = ((out - y).abs() * mask).sum() / denom
        loss.backward()
        return loss

    def step():
        loss = grads()
        opt.step()
        return loss
    # eager warm-up on a side stream (workspaces, packed weights, lengths), then the step
    # captured as two HIP graphs (RNG epoch + forward + loss + backward; clip + Adam), as
    # train.GraphedTrainStep does: the eager step is launch-bound (~1 100 launches per step)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(warm):
            step()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    from ensemble_svs_with_interactions_amd._lib import call
    execution = "hip-graph replay of the autograd step through the drop-in module"
    try:
        g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            call("ensvs_rng_advance", torch.cuda.current_stream().cuda_stream)
            gloss = grads()
        with torch.cuda.graph(g2, pool=g1.pool()):
            opt.step()
        opt._captured = True

        def replay():
            g1.replay()
            g2.replay()
            return gloss
    except RuntimeError as e:  # keep the leg measurable: eager issue, and say why
        torch.cuda.synchronize()
        execution = f"eager (graph capture failed: {str(e)[:120]})"
        replay = step
    replay()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(steps):
        loss = replay()
    torch.cuda.synchronize()
    el = (time.time() - t0) / steps
    fl = 3 * transformer_flops(B, T)
    tf = fl / el / 1e12
    peak = PEAK_BF16_TFLOPS if engine.gemm_precision() == "bf16" else 157.3
    return dict(metric="Transformer encoder train frames/sec (tier 2, row a14)",
                value=B * T / el, unit="frames/s", ms_per_step=el * 1e3, steps=steps,
                batch=B, frames=T, lengths=lens, config=TF_CFG, dtype=engine.gemm_precision(),
                execution=execution,
                train_loss=float(loss.item()),
                roofline={"bound": "mfma", "achieved": tf, "peak": peak, "unit": "TFLOP/s",
                          "frac": tf / peak, "traffic": None,
                          "work": f"3 x {transformer_flops(B, T) / 1e9:.1f} GFLOP forward per "
                                  "step (backward = 2 x forward: input and weight gradients)"})


def transformer_cpu_baseline(B=4, T=1024, warm=1, timed=5):
    """The oracle's Transformer encoder (float32, no dropout) forward + backward on the host
    cores: a bounded sample of the leg's workload."""
    from ensemble_svs_with_interactions_amd.transformer import TransformerEncoder
    from oracle import ensvs_oracle as O
    cores = _host_cores()
    torch.set_num_threads(cores)
    torch.manual_seed(20250326)
    P = {k: v.detach().clone().requires_grad_() for k, v in
         TransformerEncoder(**TF_CFG).state_dict().items()}
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, T, TF_CFG["in_dim"], generator=g)
    y = torch.randn(B, T, TF_CFG["out_dim"], generator=g)
    times = []
    for _ in range(warm + timed):
        t0 = time.time()
        out = O.transformer_encoder(P, TF_CFG, x, [T] * B)
        (out - y).abs().mean().backward()
        times.append(time.time() - t0)
    sec = float(np.median(times[warm:]))
    return dict(value=B * T / sec, unit="frames/s", cores=cores, kind="port",
                cpu_model=_cpu_model(),
                sample=f"oracle transformer_encoder forward + backward (CPU PyTorch, fp32, no "
                       f"dropout, no optimizer), {B} x {T} frames, median of {timed} steps after "
                       f"{warm} warm-up")


def config2_train(args, dev):
    """BASELINE config 2: single-track NPSSMDNMultistreamParametricModel (teacher-forced
    lf0 decoder, both diffusions, V/UV) training steps, same per-GPU workload (pairs ->
    utterances x frames), graph replay, bf16 GEMM operands."""
    from ensemble_svs_with_interactions_amd.train import train_step_single
    torch.manual_seed(20250322)
    model = configs.instantiate(configs.singletrack_diffusion()).to(dev)
    opt = FusedAdam(model, lr=1e-4, clip_norm=1.0)
    P, T = args.pairs, args.frames
    b = data.synthetic_batch(P, T, 2000)
    g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
    x, y = g("x_main"), g("y_main")
    lens = b["lengths"].tolist()
    if args.eager:
        def step():
            return train_step_single(model, opt, x, y, lens)
        step()
    else:
        step = GraphedTrainStep(model, opt, x, None, y, None, None, lens, warmup=1).step
    for _ in range(max(0, args.warmup - 1)):
        step()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(args.steps):
        loss, norm = step()
    torch.cuda.synchronize()
    el = time.time() - t0
    return dict(metric="single-track acoustic-model train frames/sec (BASELINE config 2)",
                value=P * T * args.steps / el, unit="frames/s", ms_per_step=el / args.steps * 1e3,
                steps=args.steps, utterances=P, frames=T, dtype=engine.gemm_precision(),
                train_loss=loss.item(), grad_norm=norm.item(),
                model="NPSSMDNMultistreamParametricModel (acoustic_nnsvs_world_multi_ar_f0_"
                      "diff_mgcbap.yaml)")


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    _imports()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("ENSVS_BENCH_BACKEND", "nccl") != "nccl":
        local %= torch.cuda.device_count()  # rehearsal: several ranks share the GPUs
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    backend = None
    if world > 1:
        import torch.distributed as dist
        # ENSVS_BENCH_BACKEND=gloo: rehearse N ranks on one GPU (RCCL needs one GPU per rank)
        be = os.environ.get("ENSVS_BENCH_BACKEND", "nccl")
        if be == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(be)
        world = dist.get_world_size()
        backend = dist.get_backend()
        # the default data-parallel schedule: the N = 1 line's HIP-graph replay with one
        # 94 MB all-reduce of the flat gradient (+ the 4-byte failure word) between the grads
        # and update graphs (gloo rehearsal, 2 ranks on one GPU: 51.8 ms/step with a 20.4 ms
        # host-side all-reduce, profiles/r6_bench_gloo2.json; round 5 55.3 / 22.0 ms,
        # profiles/r5_bench_gloo2_graph.json).  --overlap-ddp: eager
        # steps whose bucketed all-reduce (lf0 / bap / V/UV at their branch end, the mgc
        # DiffNet before the mgc encoder's backward) overlaps the rest of the backward (same
        # rehearsal: 929 ms/step, 7 collectives, profiles/r5_bench_gloo2_overlap.json,
        # DESIGN.md section 6 -- gloo reduces on the host); --eager alone: eager steps with
        # the one all-reduce after the backward.
        if args.overlap_ddp:
            args.eager = True
        else:
            set_overlap_allreduce(False)
    engine.set_gemm_precision(args.precision)
    engine.set_concurrency(not args.serial)
    torch.manual_seed(20250321)
    model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev)
    opt = FusedAdam(model, lr=1e-4, clip_norm=1.0)
    P, T = args.pairs, args.frames
    b = data.synthetic_batch(P, T, 1000 + rank)
    g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
    xm, xs, ym = g("x_main"), g("x_sub"), g("y_main")
    s0, s1 = g("spk_main"), g("spk_sub")
    lens = b["lengths"].tolist()
    if args.eager:
        def step():
            return train_step(model, opt, xm, xs, ym, s0, s1, lens)
        for _ in range(args.warmup):
            step()
    else:
        # one eager warm-up step, capture, then replays: every step is a full training step
        graphed = GraphedTrainStep(model, opt, xm, xs, ym, s0, s1, lens, warmup=1)
        step = graphed.step
        for _ in range(max(0, args.warmup - 1)):
            step()
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()
    barrier()
    if world > 1:  # event-time the whole-buffer exchange of every timed step
        train_mod.EXCHANGE_EVENTS = []
    t0 = time.time()
    for _ in range(args.steps):
        loss, norm = step()
    barrier()
    elapsed = time.time() - t0
    exchange = None
    if world > 1:
        exchange = exchange_report(train_mod.EXCHANGE_EVENTS, opt, model, world, backend,
                                   args, elapsed / args.steps * 1e3)
        train_mod.EXCHANGE_EVENTS = None
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    frames = P * T * world * args.steps
    value = frames / elapsed
    loss_v, norm_v = loss.item(), norm.item()
    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    sec, sec_call, flops = gate_gemm_timing(model, P, T, dev)
    net = model.mgc_model.denoise_fn
    gbytes = gate_gemm_bytes(P * T, net.C, net.E, 2 if args.precision == "bf16" else 4)
    per_gpu = value / world
    step_tf = per_gpu * TRAIN_FLOP_PER_FRAME / 1e12
    peak_tf = PEAK_BF16_TFLOPS if args.precision == "bf16" else 157.3
    roof = {
        "scope": "the whole training step (every kernel of forward, backward, clip and Adam; "
                 "the lf0 / mgc / bap / vuv branches on concurrent streams)",
        "bound": "mfma", "achieved": step_tf, "peak": peak_tf, "unit": "TFLOP/s",
        "frac": step_tf / peak_tf, "traffic": _committed("r6_step_pmc.json",
                                                         "hbm_bytes_per_step"),
        "traffic_source": "profiles/r6_step_pmc.json (rocprofv3 --pmc FETCH_SIZE x2 + "
                          "WRITE_SIZE summed over one step's dispatches, separate passes; "
                          "committed, not this run)",
        "work": f"{TRAIN_FLOP_PER_FRAME / 1e6:.1f} MFLOP per main-track frame (GEMM / conv / "
                "LSTM FLOPs of forward + backward, torch.utils.flop_counter on the oracle, "
                "SURVEY.md section 8(d)) x frames/s per GPU",
        "gate_gemm_live": _gate_roofline(args, P, T, sec, sec_call, flops, gbytes)}
    if world == 1 and not args.no_census:
        agg, serial_ms, alloc = step_census(model, opt, (xm, xs, ym, s0, s1, lens))
        # step-level algorithmic bytes: every tensor the step materialises written once and
        # read once (2 x the bytes the step allocates: activations, saved state, gradients
        # of activations, bf16 copies), plus 9 passes over the flat fp32 parameters (weight
        # repack read, zero_grad, clip + Adam: p, g, m, v read, p, m, v written)
        flat_bytes = opt.flat.numel() * 4
        alg = 2 * alloc + 9 * flat_bytes
        roof["algorithmic_bytes"] = alg
        roof["algorithmic_bytes_model"] = (
            f"2 x {alloc / 1e9:.2f} GB allocated by one eager step (each tensor written once, "
            f"read once) + 9 x {flat_bytes / 1e6:.0f} MB of flat parameters")
        if roof["traffic"]:
            roof["traffic_over_algorithmic"] = roof["traffic"] / alg
        roof["kernels"], roof["recurrences"] = kernel_rooflines(agg, serial_ms, P, T)
        rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
        census = {"serial_step_ms": serial_ms, "launches": sum(v[0] for v in agg.values()),
                  "rows": [[k[0][6:], k[1] or "", n, round(ms / n * 1e3, 1), round(ms, 3)]
                           for k, (n, ms) in rows[:30]],
                  "columns": ["entry", "shape", "launches", "us_per_launch", "ms_total"]}
    out = {
        "metric": "acoustic-model train frames/sec/GPU (4-track ensemble); synth RTF",
        "value": value, "unit": "main-track frames/s", "value_per_gpu": value / world,
        "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": args.precision, "data": "synthetic (SURVEY.md §8(d) feature layout), random-init "
                                          "weights of the recipe architecture",
        "config": {"workload": "4-track SATB ensemble, MultiTrackNPSSMDNMultistreamParametric"
                               "Model (multitrack_acoustic_nnsvs_world_multi_ar_f0_diff_mgcbap)",
                   "value_is": "aggregate main-track frames/s over all ranks (value_per_gpu "
                               "= value / n_gpus is the metric's per-GPU figure)",
                   "pairs_per_gpu": P, "frames_per_pair": T, "global_batch_pairs": P * world,
                   "parallelism": f"dp{world}",
                   "process_group": {"backend": backend, "world_size": world} if world > 1
                   else None,
                   "execution": ("eager, bucketed all-reduce overlapped with the backward"
                                 if world > 1 and args.overlap_ddp else
                                 "eager" if args.eager else "hip-graph replay") +
                                (", one whole-buffer all-reduce per step" if world > 1 and
                                 not args.overlap_ddp else "")},
        "train_loss": loss_v, "grad_norm": norm_v,
        "exchange": exchange,
        # reference-equivalent work (the oracle's flop count); the path skips the sub-track
        # lf0 BiLSTM + AR decoder forward, whose output the plain recipe never reads
        # (acoustic_models._bn_only): executed work per frame is 0.59 MFLOP less
        "model_tflops_per_s": value * TRAIN_FLOP_PER_FRAME / 1e12,
        "executed_tflops_per_s": value * (TRAIN_FLOP_PER_FRAME - SUBTRACK_SKIPPED_FLOP) / 1e12,
        "roofline": roof,
    }
    if world == 1 and not args.no_census:
        out["census"] = census
    if not args.no_shapes and world == 1:
        out["shapes"] = shape_legs(args, dev, model, opt, elapsed / args.steps * 1e3)
    if not args.no_real_data and world == 1:
        out["real_data"] = real_data_train(args, dev)
        out["real_data"]["ratio_to_fixed_shape"] = out["real_data"]["value"] / value
    if not args.no_sf0 and world == 1:
        out["separate_f0"] = sf0_train(args, dev)
    if not args.no_config2 and world == 1:
        out["config2"] = config2_train(args, dev)
        out["interaction_loss"] = il_train(args, dev)
    if not args.no_transformer and world == 1:
        out["transformer"] = transformer_train(dev)
    if not args.no_synth and world == 1:
        out["synth"] = synth_rtf(model, dev)
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(args)
        if "separate_f0" in out:
            out["separate_f0"]["cpu_baseline"] = sf0_cpu_baseline()
        if "synth" in out:
            out["synth"]["cpu_baseline"] = cpu_synth_baseline(out["synth"]["frames"])
        if "transformer" in out:
            out["transformer"]["cpu_baseline"] = transformer_cpu_baseline()
    print(json.dumps(out), flush=True)


def exchange_report(events, opt, model, world, backend, args, step_ms):
    """The data-parallel exchange of the timed steps (rank 0's view): the whole-buffer
    all-reduce of the flat gradient (+ the 4-byte failure word, MAX) timed with HIP events on
    the stream the collectives are ordered on, its bytes, algorithm and bus bandwidth (ring:
    2 (W-1)/W of the buffer through every rank's links), and the number of collectives one
    step issues.  The overlap path's bucketed collectives run beside the backward, so only
    their count and bytes are reported."""
    nbytes = opt.gflat.numel() * 4
    out = {"backend": backend, "world_size": world, "bytes_per_step": nbytes + 4,
           "reference": "nnsvs/train_util.py:1444-1446 (DistributedDataParallel all-reduce)"}
    if args.overlap_ddp:
        br = getattr(opt, "_bucketed", None)
        out.update(schedule="bucketed all-reduce overlapped with the backward (eager)",
                   collectives_per_step=getattr(br, "collectives_last_step", None),
                   buckets={k: len(v) for k, v in br.buckets.items()} if br else None)
        return out
    torch.cuda.synchronize()
    ms = [s.elapsed_time(e) for s, e in events]
    per = float(np.mean(ms)) if ms else None
    out.update(schedule="one whole-buffer all-reduce between the grads and update graphs",
               collectives_per_step=2, exchanges_timed=len(ms))
    if per:
        alg = nbytes / (per * 1e-3) / 1e9
        out.update(allreduce_ms_per_step=per, allreduce_ms_max=float(np.max(ms)),
                   algbw_gbs=alg, busbw_gbs=alg * 2 * (world - 1) / world,
                   share_of_step=per / step_ms)
    return out


def _gate_roofline(args, P, T, sec, sec_call, flops, gbytes):
    """Roofline of the dominant kernel.  The binding roof is the larger of its two lower
    bounds: algorithmic bytes / 8 TB/s and FLOPs / dense MFMA peak.  With bf16 operands
    and bf16 outputs the gate GEMM moves 79.7 MB (10.0 us of HBM) for 32.2 GFLOP (12.9 us
    of bf16 MFMA): intensity 404 FLOP/B above the ridge (312), so MFMA binds; the fp32
    parity mode (exact fp32 MFMA, 157 TFLOP/s) is MFMA-bound as well."""
    peak_tf = PEAK_BF16_TFLOPS if args.precision == "bf16" else 157.3
    t_mfma, t_hbm = flops / (peak_tf * 1e12), gbytes / (PEAK_HBM_GBS * 1e9)
    tflops, gbs = flops / sec / 1e12, gbytes / sec / 1e9
    r = {"kernel": "conv_gemm_b16_p8_kernel (256x256 tile, four-phase counted LDS-DMA "
                   f"pipeline; mgc DiffNet block gate GEMM, M={P * T} N=512 K=1024, bf16 operands)"
                   if args.precision == "bf16" else "conv_gemm_kernel<float>"}
    if t_mfma >= t_hbm:
        r.update(bound="mfma", achieved=tflops, peak=peak_tf, unit="TFLOP/s",
                 frac=tflops / peak_tf, hbm_gbs=gbs, hbm_frac=gbs / PEAK_HBM_GBS)
    else:
        r.update(bound="hbm", achieved=gbs, peak=PEAK_HBM_GBS, unit="GB/s",
                 frac=gbs / PEAK_HBM_GBS, tflops=tflops, mfma_frac=tflops / peak_tf)
    r.update(flops=flops, algorithmic_bytes=gbytes, launch_us=sec * 1e6,
             call_us_incl_operand_casts=sec_call * 1e6, traffic=_traffic(),
             traffic_source="profiles/r6_gate_gemm_pmc.json (rocprofv3 --pmc FETCH_SIZE x2 + "
                            "WRITE_SIZE per dispatch, separate passes; not this run)")
    return r


def _traffic():
    """HBM bytes per launch of the gate GEMM from the committed rocprofv3 PMC pass
    (profiles/r6_gate_gemm_pmc.json, written by tools/round_profiles.sh), if any."""
    return _committed("r6_gate_gemm_pmc.json", "hbm_bytes_per_launch")


def _committed(name, key):
    p = os.path.join(ROOT, "profiles", name)
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f).get(key)
    return None


if __name__ == "__main__":
    main()
