"""Data-parallel path on CPU (gloo, world_size 2).

The product's multi-GPU step (train.train_step under torch.distributed) shards
pairs as the reference does (train_util.py:1176-1182, ``x[rank::W]``), folds the
1/W gradient average into the loss gradient (masked_l1 grad_scale) and exchanges
gradients with ONE sum all-reduce of the flat buffer (train.allreduce_grads).
Here each rank computes its shard's gradient with the oracle (the same loss
arithmetic; BatchNorm in eval mode, SURVEY.md §8(e) parity definition) scaled by
1/W, runs the product's allreduce_grads over gloo, and the result must equal the
single-process gradient of the whole batch.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from ensemble_svs_with_interactions_amd import configs, data
from golden_util import params_from_shapes, tiny_shapes
from oracle import ensvs_oracle as O

P_PAIRS, T, W = 4, 32, 2


def _batch():
    b = data.synthetic_batch(P_PAIRS, T, 11)
    g = torch.Generator().manual_seed(5)
    r = 4
    draws = dict(
        lf0_main=(torch.rand(P_PAIRS, T // r, 1, generator=g) > 0.5).float() * 2.0,
        lf0_sub=(torch.rand(P_PAIRS, T // r, 1, generator=g) > 0.5).float() * 2.0,
        mgc_t=torch.randint(0, 100, (P_PAIRS,), generator=g),
        mgc_noise=torch.randn(P_PAIRS, 1, 60, T, generator=g),
        bap_t=torch.randint(0, 100, (P_PAIRS,), generator=g),
        bap_noise=torch.randn(P_PAIRS, 1, 5, T, generator=g))
    return b, draws


def _shard_grad(idx, scale):
    """Oracle gradient (flat, sorted trainable keys) of the masked L1 loss on pairs idx."""
    torch.manual_seed(0)
    cfg = configs.multitrack_diffusion(num_speakers=4, tiny=True)
    P = params_from_shapes(tiny_shapes())
    keys = sorted(k for k in P if "running" not in k and "num_batches" not in k
                  and k.rsplit(".", 1)[-1] not in O.diffusion_schedule())
    for k in keys:
        P[k] = P[k].detach().requires_grad_()
    b, dr = _batch()
    sel = torch.as_tensor(idx)
    t = {k: torch.from_numpy(v)[sel] for k, v in b.items()}
    d = {k: v[sel] for k, v in dr.items()}
    ys = (t["y_main"], t["y_sub"])
    preds, _ = O.model_forward(P, cfg, t["x_main"], t["x_sub"], (t["spk_main"], t["spk_sub"]),
                               t["lengths"].numpy(), ys, d, training=False)
    loss = O.masked_l1_loss(preds, ys[0], t["lengths"].numpy(), cfg["stream_sizes"]) * scale
    loss.backward()
    return torch.cat([(P[k].grad if P[k].grad is not None else torch.zeros_like(P[k])).reshape(-1)
                      for k in keys])


def _rank(rank, port, out_dir):
    import torch.distributed as dist
    from ensemble_svs_with_interactions_amd import train
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=W)
    try:
        (mine,) = data.shard_pairs([list(range(P_PAIRS))], rank, W)
        assert train.world_size() == W
        gflat = _shard_grad(mine, 1.0 / train.world_size())
        train.allreduce_grads(gflat)
        np.save(os.path.join(out_dir, f"g{rank}.npy"), gflat.numpy())
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_pairs_matches_reference_split():
    batches = [list(range(8)), list(range(8, 13)), list(range(13, 19))]
    assert data.shard_pairs(batches, 0, 2) == [[0, 2, 4, 6], [13, 15, 17]]
    assert data.shard_pairs(batches, 1, 2) == [[1, 3, 5, 7], [14, 16, 18]]
    assert data.shard_pairs(batches, 0, 1) == batches
    # every index of the kept batches lands on exactly one rank
    got = sorted(i for r in range(3) for b in data.shard_pairs(batches, r, 3) for i in b)
    assert got == list(range(13, 19))


def test_allreduce_without_process_group_is_noop():
    from ensemble_svs_with_interactions_amd import train
    g = torch.arange(5, dtype=torch.float32)
    train.allreduce_grads(g)
    assert torch.equal(g, torch.arange(5, dtype=torch.float32))
    assert train.world_size() == 1


@pytest.mark.timeout(600)
def test_ddp_world2_equals_full_batch(tmp_path):
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank, args=(r, port, str(tmp_path))) for r in range(W)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(540)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    g0 = np.load(tmp_path / "g0.npy")
    g1 = np.load(tmp_path / "g1.npy")
    assert np.array_equal(g0, g1)  # every rank holds the same averaged gradient
    full = _shard_grad(list(range(P_PAIRS)), 1.0).numpy()
    # equal lengths: mean over ranks of per-shard means == mean over the whole batch
    err = np.abs(g0 - full).max() / np.abs(full).max()
    assert err < 1e-5, err
