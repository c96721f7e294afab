"""Data-parallel product step at world size 2 on one MI355X (two processes, gloo over CUDA
tensors; the bench's N-GPU runs use RCCL with the same code).

Pairs are split x[rank::W] (train_util.py:1176-1182).  Per rank:
  1. FusedAdam broadcasts rank 0's state (as DDP's constructor does): ranks seeded
     differently start equal.
  2. train.train_step (ddp): the flat gradient after the all-reduce equals the mean of the
     ranks' own (pre-reduce, 1/W-scaled) shard gradients, and the updated parameters are
     identical on both ranks.
  3. GraphedTrainStep: the same relation on graph replays (the all-reduce runs between the
     two captured graphs).
  4. torch DistributedDataParallel(model) around the drop-in model with the reference-style
     autograd step: DDP's hooks average the gradients that Function.backward returns, and
     the result equals the fused data-parallel gradient of the same shards.
  5. SURVEY 8(e)'s parity definition: with BatchNorm frozen (bn.eval() inside the training
     step) and equal lengths, the all-reduced gradient of the two shards equals the
     product's own single-process gradient of the concatenated 4-pair batch -- at the tiny
     widths and at the recipe widths (full-size model, P = 4, T = 64).
  6. A cooperative-recurrence failure on one rank (coop.h; the test switch makes rank 1's
     cooperative AR decoder time out) skips the update on EVERY rank: the failing rank
     writes NaN into a gradient element before the all-reduce (bucketed and whole-buffer
     schedules), so both ranks' norms are NaN and both keep their parameters.
BatchNorm statistics stay per rank, as in the reference (no SyncBN).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
W = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, port, out_dir):
    import sys
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    sys.path.insert(0, here)
    from ensemble_svs_with_interactions_amd import configs, data, engine, train
    from golden_util import load_case
    from gpu_util import build
    from test_dropin_gpu import _reference_style_loss

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=W)
    res = {}
    try:
        engine.set_gemm_precision("fp32")
        a, meta = load_case("train_step_tiny")
        cfg = configs.multitrack_diffusion(num_speakers=4, tiny=True)
        b = data.synthetic_batch(4, 32, 77)
        (mine,) = data.shard_pairs([list(range(4))], rank, W)
        sel = np.asarray(mine)
        g = lambda k: torch.from_numpy(np.ascontiguousarray(b[k][sel])).cuda()  # noqa: E731
        xm, xs, ym, ys, s0, s1 = (g(k) for k in ("x_main", "x_sub", "y_main", "y_sub",
                                                  "spk_main", "spk_sub"))
        lens = b["lengths"][sel].tolist()
        Bs, T = xm.shape[:2]
        gen = torch.Generator().manual_seed(100 + rank)
        draws = dict(lf0_main=(torch.rand(Bs * T // 4, generator=gen) > 0.5).float().cuda() * 2,
                     lf0_sub=(torch.rand(Bs * T // 4, generator=gen) > 0.5).float().cuda() * 2,
                     mgc_t=torch.randint(0, 100, (Bs,), generator=gen).cuda(),
                     bap_t=torch.randint(0, 100, (Bs,), generator=gen).cuda(),
                     mgc_noise=torch.randn(Bs * T, 60, generator=gen).cuda(),
                     bap_noise=torch.randn(Bs * T, 5, generator=gen).cuda())

        def gather(t):
            out = [torch.zeros_like(t.cpu()) for _ in range(W)]
            dist.all_gather(out, t.detach().cpu().contiguous())
            return out

        # record each rank's own gradient right before the exchange
        pre = []
        orig = train.allreduce_grads

        def spy(gflat, group=None):
            pre.append(gflat.detach().clone())
            return orig(gflat, group)
        train.allreduce_grads = spy

        def check_mean(opt, tag):
            mine_pre = pre[-1]
            allpre = gather(mine_pre)
            mean = sum(allpre)  # each rank's gradient is already scaled by 1/W
            got = opt.gflat.detach().cpu()
            res[tag + "_grad_err"] = ((got - mean).norm() / mean.norm()).item()
            res[tag + "_rank_grads_differ"] = float((allpre[0] - allpre[1]).abs().max())
            flats = gather(opt.flat)
            res[tag + "_param_mismatch"] = float((flats[0] - flats[1]).abs().max())

        # 1 + 2: broadcast at init, fused step (one all-reduce of the whole buffer)
        torch.manual_seed(1234 + rank)  # ranks initialise differently on purpose
        model = configs.instantiate(cfg).cuda()
        model.vuv_model.lstm.dropout = 0.0
        opt = train.FusedAdam(model, lr=1e-3)
        flats = gather(opt.flat)
        res["init_param_mismatch"] = float((flats[0] - flats[1]).abs().max())
        train.set_overlap_allreduce(False)
        loss, norm = train.train_step(model, opt, xm, xs, ym, s0, s1, lens, draws=draws)
        torch.cuda.synchronize()
        check_mean(opt, "fused")
        fused_grad = opt.gflat.detach().cpu().clone()
        # DDP's broadcast_buffers: the ranks' BatchNorm statistics differ after a step on
        # their own shards; the next step starts from rank 0's on every rank
        bufs = lambda m: torch.cat([b.detach().float().flatten() for b in m.buffers()])  # noqa: E731
        after = gather(bufs(model))
        res["bn_stats_differ_after_step"] = float((after[0] - after[1]).abs().max())
        synced = []
        orig_sync = train.sync_buffers

        def sync_spy(m, *a, **k):
            orig_sync(m, *a, **k)
            synced.append(bufs(m).cpu())
        train.sync_buffers = sync_spy
        train.train_step(model, opt, xm, xs, ym, s0, s1, lens, draws=draws)
        torch.cuda.synchronize()
        train.sync_buffers = orig_sync
        got = gather(synced[0])
        res["bn_sync_rank_mismatch"] = float((got[0] - got[1]).abs().max())
        res["bn_sync_vs_rank0"] = float((got[1] - after[0]).abs().max())

        # 2b: the same step with the bucketed all-reduce overlapped with the backward
        # (train.BucketedAllReduce): the same reduced gradient, no whole-buffer all-reduce
        torch.manual_seed(1234 + rank)
        m2 = configs.instantiate(cfg).cuda()
        m2.vuv_model.lstm.dropout = 0.0
        o2 = train.FusedAdam(m2, lr=1e-3)
        train.set_overlap_allreduce(True)
        n_before = len(pre)
        train.train_step(m2, o2, xm, xs, ym, s0, s1, lens, draws=draws)
        torch.cuda.synchronize()
        res["overlap_whole_buffer_calls"] = len(pre) - n_before
        res["overlap_grad_err"] = float((o2.gflat.detach().cpu() - fused_grad).abs().max() /
                                        fused_grad.abs().max())
        res["overlap_buckets"] = sum(len(v) for v in o2._bucketed.buckets.values())
        flats2 = gather(o2.flat)
        res["overlap_param_mismatch"] = float((flats2[0] - flats2[1]).abs().max())
        del m2, o2

        # 3: graph-replayed data-parallel steps
        gstep = train.GraphedTrainStep(model, opt, xm, xs, ym, s0, s1, lens, warmup=1)
        for _ in range(2):
            gstep.step()
        torch.cuda.synchronize()
        check_mean(opt, "graph")
        train.allreduce_grads = orig

        # 4: torch DDP around the drop-in model, reference-style autograd step
        torch.manual_seed(0)
        ref = build(cfg, meta["shapes"])
        ref.vuv_model.lstm.dropout = 0.0
        torch.manual_seed(0)
        fz = build(cfg, meta["shapes"])
        fz.vuv_model.lstm.dropout = 0.0
        fopt = train.FusedAdam(fz, lr=1e-3)
        train._loss_and_grads(fz, fopt, xm, xs, ym, s0, s1, lens, draws, True, None, 0.0)
        train.allreduce_grads(fopt.gflat)
        ddp = torch.nn.parallel.DistributedDataParallel(ref, device_ids=[0])
        ref.train()
        ref._replay_draws = draws
        for p in ref.parameters():
            p.grad = None
        lengths = torch.tensor(lens, device="cuda")
        # DDP averages; the reference's loss is per-rank (not 1/W scaled)
        loss = _reference_style_loss(ddp, xm, xs, ym, ys, (s0, s1), lengths, 0.0,
                                     cfg["stream_sizes"])
        loss.backward()
        torch.cuda.synchronize()
        num = den = 0.0
        for (k, p), (k2, q) in zip(ref.named_parameters(), fz.named_parameters()):
            assert k == k2
            num += ((p.grad - q.grad) ** 2).sum().item()
            den += (q.grad ** 2).sum().item()
        res["ddp_grad_err"] = (num / den) ** 0.5
        res["fused_grad_norm"] = float(fused_grad.norm())

        # 5: data-parallel parity as SURVEY 8(e) defines it: with BatchNorm frozen (eval)
        # and equal lengths, the all-reduced gradient of the W shards equals the product's
        # own single-process gradient of the concatenated 4-pair batch (same draws)
        gf = torch.Generator().manual_seed(55)
        P4 = 4
        full_draws = dict(
            lf0_main=(torch.rand(P4, T // 4, generator=gf) > 0.5).float() * 2,
            lf0_sub=(torch.rand(P4, T // 4, generator=gf) > 0.5).float() * 2,
            mgc_t=torch.randint(0, 100, (P4,), generator=gf),
            bap_t=torch.randint(0, 100, (P4,), generator=gf),
            mgc_noise=torch.randn(P4, T, 60, generator=gf),
            bap_noise=torch.randn(P4, T, 5, generator=gf))

        def take(idx):
            out = {}
            for k, v in full_draws.items():
                v = v[torch.as_tensor(idx)]
                out[k] = (v.reshape(len(idx) * T, -1) if k.endswith("noise")
                          else v.reshape(-1)).contiguous().cuda()
            return out

        def frozen_bn_model():
            torch.manual_seed(4321)
            m = configs.instantiate(cfg).cuda()
            m.vuv_model.lstm.dropout = 0.0
            m.train()
            for mod in m.modules():
                if isinstance(mod, torch.nn.BatchNorm1d):
                    mod.eval()
            return m

        allp = list(range(P4))

        def dp_vs_full(tag, bb):
            fb = lambda k, idx: torch.from_numpy(np.ascontiguousarray(bb[k][idx])).cuda()  # noqa: E731
            mdp = frozen_bn_model()
            odp = train.FusedAdam(mdp, lr=1e-3)
            train.set_overlap_allreduce(True)
            ldp, _ = train.train_step(mdp, odp, *(fb(k, sel) for k in (
                "x_main", "x_sub", "y_main", "spk_main", "spk_sub")),
                bb["lengths"][sel].tolist(), draws=take(mine))
            m1 = frozen_bn_model()
            o1 = train.FusedAdam(m1, lr=1e-3)
            l1, _ = train.train_step(m1, o1, *(fb(k, allp) for k in (
                "x_main", "x_sub", "y_main", "spk_main", "spk_sub")),
                bb["lengths"].tolist(), draws=take(allp), ddp=False)
            torch.cuda.synchronize()
            assert all(not mod.training for mod in mdp.modules()
                       if isinstance(mod, torch.nn.BatchNorm1d))
            gdp, g1 = odp.gflat.detach().cpu(), o1.gflat.detach().cpu()
            res[tag + "_grad_rel_l2"] = ((gdp - g1).norm() / g1.norm()).item()
            res[tag + "_grad_norm"] = float(g1.norm())
            losses = gather(ldp.detach().view(1))
            res[tag + "_loss_rel"] = abs(float(sum(losses)) / W - l1.item()) / abs(l1.item())
            flats = gather(odp.flat)
            res[tag + "_param_mismatch"] = float((flats[0] - flats[1]).abs().max())
            del mdp, odp, m1, o1

        dp_vs_full("dp_vs_full", b)
        # the same at the recipe widths (full-size model), P = 4 pairs of T = 64 frames
        T = 64
        cfg = configs.multitrack_diffusion(num_speakers=4)
        gf = torch.Generator().manual_seed(56)
        full_draws = dict(
            lf0_main=(torch.rand(P4, T // 4, generator=gf) > 0.5).float() * 2,
            lf0_sub=(torch.rand(P4, T // 4, generator=gf) > 0.5).float() * 2,
            mgc_t=torch.randint(0, 100, (P4,), generator=gf),
            bap_t=torch.randint(0, 100, (P4,), generator=gf),
            mgc_noise=torch.randn(P4, T, 60, generator=gf),
            bap_noise=torch.randn(P4, T, 5, generator=gf))
        dp_vs_full("dp_vs_full_recipe", data.synthetic_batch(P4, T, 78))

        # 6: one rank's cooperative-recurrence failure skips the update on every rank
        engine.set_gemm_precision("bf16")
        bb = data.synthetic_batch(P4, T, 79)
        fb = lambda k: torch.from_numpy(np.ascontiguousarray(bb[k][sel])).cuda()  # noqa: E731
        batch = [fb(k) for k in ("x_main", "x_sub", "y_main", "spk_main", "spk_sub")]
        from ensemble_svs_with_interactions_amd._lib import call
        for overlap in (True, False):
            torch.manual_seed(99)
            mf = configs.instantiate(cfg).cuda()
            of = train.FusedAdam(mf, lr=1e-3)
            train.set_overlap_allreduce(overlap)
            before = of.flat.detach().clone()
            if rank == 1:
                call("ensvs_coop_set_timeout_us", 20000)
                call("ensvs_coop_inject_fault", 1)
            _, nf = train.train_step(mf, of, *batch, bb["lengths"][sel].tolist())
            torch.cuda.synchronize()
            call("ensvs_coop_inject_fault", 0)
            call("ensvs_coop_set_timeout_us", 1000000)
            tag = "fault_overlap" if overlap else "fault_whole"
            res[tag + "_norm_finite"] = float(np.isfinite(nf.item()))
            res[tag + "_params_changed"] = float((of.flat - before).abs().max())
            res[tag + "_device_step"] = float(of.device_step)
            raised = 0.0
            try:
                engine.check_coop_errors("cuda")
            except engine.CoopError:
                raised = 1.0
            res[tag + "_raised"] = raised
            del mf, of
    finally:
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), **{k: np.float64(v) for k, v in res.items()})
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_data_parallel_world2_product_step(tmp_path):
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank, args=(r, port, str(tmp_path))) for r in range(W)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(280)
        if p.exitcode is None:
            p.kill()
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    for r in range(W):
        z = dict(np.load(tmp_path / f"r{r}.npz"))
        print(r, {k: float(v) for k, v in z.items()})
        assert z["init_param_mismatch"] == 0.0
        for tag in ("fused", "graph"):
            assert z[tag + "_grad_err"] < 1e-6, (tag, z[tag + "_grad_err"])
            assert z[tag + "_param_mismatch"] == 0.0, tag
            assert z[tag + "_rank_grads_differ"] > 0.0, tag  # the shards really differ
        # bucketed all-reduce overlapped with the backward: same reduced gradient (2 ranks:
        # a + b either way), equal parameters on both ranks, no whole-buffer collective
        assert z["overlap_grad_err"] < 1e-6, z["overlap_grad_err"]
        assert z["overlap_param_mismatch"] == 0.0
        assert z["overlap_whole_buffer_calls"] == 0 and z["overlap_buckets"] >= 6
        assert z["ddp_grad_err"] < 1e-5, z["ddp_grad_err"]
        # broadcast_buffers: statistics differ after a step, equal rank 0's at the next one
        assert z["bn_stats_differ_after_step"] > 0.0
        assert z["bn_sync_rank_mismatch"] == 0.0 and z["bn_sync_vs_rank0"] == 0.0
        # DP-W gradient == 1-process full-batch gradient (BN frozen, equal lengths)
        for tag in ("dp_vs_full", "dp_vs_full_recipe"):
            assert z[tag + "_grad_rel_l2"] < 1e-6, (tag, z[tag + "_grad_rel_l2"])
            assert z[tag + "_loss_rel"] < 1e-6, (tag, z[tag + "_loss_rel"])
            assert z[tag + "_param_mismatch"] == 0.0, tag
        # rank 1's recurrence failed: no rank applied an update, every rank raises (the
        # failure word is MAX-reduced after the gradient's last collective)
        for tag in ("fault_overlap", "fault_whole"):
            assert z[tag + "_norm_finite"] == 0.0, (r, tag)
            assert z[tag + "_params_changed"] == 0.0, (r, tag)
            assert z[tag + "_device_step"] == 0.0, (r, tag)
            assert z[tag + "_raised"] == 1.0, (r, tag)
