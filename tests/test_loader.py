"""On-disk pair dataset (ensemble_svs_with_interactions_amd/loader.py) against fixtures the
reference generated on the same files (tests/golden/gen_goldens.py::case_loader):
train_util.py get_filtered_files_multitrack :153-177, SyncMultiTrackDataset :439-520,
batch_by_size :190-246, collate_fn_syncmultitrack_acoustic :937-1019.  Bit-exact."""
import os

import numpy as np
import pytest
import torch

from golden_util import load_case, loader_tree
from ensemble_svs_with_interactions_amd import data, loader


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    a, meta = load_case("loader")
    root = str(tmp_path_factory.mktemp("ensvs_loader"))
    dirs = loader_tree(root, a)
    return root, dirs, a, meta


def _dataset(tree, shuffle=True, allow_cache=False):
    root, dirs, a, meta = tree
    in_files, lengths = loader.get_filtered_files_multitrack(dirs["in"])
    out_files, _ = loader.get_filtered_files_multitrack(dirs["out"])
    return loader.SyncMultiTrackDataset(in_files, out_files, lengths, meta["spk_list"],
                                        shuffle=shuffle, allow_cache=allow_cache)


def test_file_pairs_match_reference(tree):
    root, dirs, a, meta = tree
    rel = lambda p: os.path.relpath(p, root)  # noqa: E731
    in_files, lengths = loader.get_filtered_files_multitrack(dirs["in"])
    out_files, _ = loader.get_filtered_files_multitrack(dirs["out"])
    assert [[rel(x), rel(y)] for x, y in in_files] == meta["in_pairs"]
    assert [[rel(x), rel(y)] for x, y in out_files] == meta["out_pairs"]
    assert [[int(x), int(y)] for x, y in lengths] == meta["lengths"]


def test_filters_ignored_for_multitrack(tree):
    """App. A-17: the multitrack discovery ignores filter_long_segments."""
    root, dirs, a, meta = tree
    pairs, _ = loader.get_filtered_files_multitrack(dirs["in"], None, True, 40, 35)
    assert len(pairs) == len(meta["in_pairs"])
    files, lens = loader.get_filtered_files(dirs["in"], None, True, 150, 60)
    assert files and all(60 < n < 150 for n in lens)


def test_dataset_items(tree):
    root, dirs, a, meta = tree
    ds = _dataset(tree)
    assert len(ds) == len(meta["items"])
    for i, (s0, s1, n0, n1) in enumerate(meta["items"]):
        it = ds[i]
        assert (it[2], it[6]) == (s0, s1)
        assert np.array_equal(it[3], a[f"item{i}::times0"])
        assert np.array_equal(it[7], a[f"item{i}::times1"])
        utt0 = os.path.basename(ds.in_paths[i][0]).split("-feats")[0]
        assert np.array_equal(it[0], a[f"file::in::{utt0}"])
        assert np.array_equal(it[1], a[f"file::out::{utt0}"])


def test_cache_returns_same_item(tree):
    ds = _dataset(tree, allow_cache=True)
    first = ds[3]
    assert ds[3] is first


def test_ordered_indices_and_batches(tree):
    root, dirs, a, meta = tree
    ds = _dataset(tree)
    for seed in (0, 7):
        np.random.seed(seed)
        idx = ds.ordered_indices()
        assert [int(i) for i in idx] == meta["orders"][str(seed)]
        for mt in (250, 700, 2000):
            for w in (1, 2, 3):
                b = loader.batch_by_size(idx, ds.num_tokens, max_tokens=mt,
                                         required_batch_size_multiple=w)
                assert [[int(i) for i in x] for x in b] == meta["batches"][f"{seed}/{mt}/{w}"]
    assert list(_dataset(tree, shuffle=False).ordered_indices()) == list(range(len(ds)))


def test_batch_by_size_edge_cases():
    assert loader.batch_by_size([], lambda i: 1, max_tokens=10) == []
    assert loader.batch_by_size([0, 1, 2], lambda i: 5, max_sentences=2) == [[0, 1], [2]]
    with pytest.raises(AssertionError):
        loader.batch_by_size([0], lambda i: 11, max_tokens=10)


def test_collate_of_loaded_batch(tree):
    root, dirs, a, meta = tree
    ds = _dataset(tree)
    out = data.collate_syncmultitrack_acoustic([ds[i] for i in meta["collate_batch"]],
                                               reduction_factor=4)
    for j, o in enumerate(out):
        ref = a[f"collate{j}"]
        assert o.shape == ref.shape and np.array_equal(o.astype(ref.dtype), ref), j


def test_feeder_cpu_order_and_sort(tree):
    """The feeder yields the collated batches in sampler order, each track sorted by its
    own lengths (train_acoustic_multitrack.py:472-483), lengths = max(L0, L1)."""
    root, dirs, a, meta = tree
    ds = _dataset(tree)
    batches = meta["batches"]["7/700/1"]
    feeder = loader.PairBatchFeeder(ds, batches, reduction_factor=4, device="cpu")
    n = 0
    for b, fb in zip(batches, feeder):
        cols = data.collate_syncmultitrack_acoustic([ds[i] for i in b], reduction_factor=4)
        i0, i1, lmax = data.sort_pair_batch(cols[3], cols[7])
        assert torch.equal(fb["x_main"], torch.from_numpy(cols[0][i0]))
        assert torch.equal(fb["y_sub"], torch.from_numpy(cols[5][i1]))
        assert fb["spk_main"].dtype == torch.int64
        assert np.array_equal(fb["spk_sub"].numpy()[:, 0], cols[6][i1][:, 0].astype(np.int64))
        assert np.array_equal(fb["host_lengths"], lmax)
        n += 1
    assert n == len(batches)


def test_feeder_surfaces_reader_errors(tree):
    ds = _dataset(tree)
    feeder = loader.PairBatchFeeder(ds, [[0], [10 ** 6]], device="cpu")
    with pytest.raises(IndexError):
        for _ in feeder:
            pass


def test_setup_multitrack_batches_sharding(tree):
    root, dirs, a, meta = tree
    np.random.seed(7)
    _, full = loader.setup_multitrack_batches(dirs["in"], dirs["out"], meta["spk_list"], 700,
                                              world=2, rank=0)
    np.random.seed(7)
    _, r1 = loader.setup_multitrack_batches(dirs["in"], dirs["out"], meta["spk_list"], 700,
                                            world=2, rank=1)
    ref = meta["batches"]["7/700/2"]
    assert full == [x[0::2] for x in ref if len(x) % 2 == 0]
    assert r1 == [x[1::2] for x in ref if len(x) % 2 == 0]


@pytest.mark.gpu
def test_feeder_device_copy(tree):
    """Pinned host buffers copied on the feeder's copy stream arrive intact on the
    consumer stream (bitwise), with the consumer running work in between."""
    root, dirs, a, meta = tree
    ds = _dataset(tree)
    batches = meta["batches"]["0/2000/1"]
    host = loader.PairBatchFeeder(ds, batches, device="cpu")
    dev = loader.PairBatchFeeder(ds, batches, device="cuda:0", prefetch=3)
    side = torch.zeros(1 << 22, device="cuda:0")
    for hb, db in zip(host, dev):
        side.mul_(1.0001)  # keep the consumer stream busy while copies land
        for k in ("x_main", "y_main", "spk_main", "len_main", "x_sub", "y_sub", "spk_sub",
                  "len_sub", "lengths"):
            assert db[k].device.type == "cuda"
            assert torch.equal(db[k].cpu(), hb[k]), k


@pytest.mark.gpu
def test_train_epoch_from_disk(tmp_path):
    """The reference's data path end to end on the GPU: on-disk features -> pairs ->
    dynamic batches -> feeder -> train_epoch.  Each step equals train_step on the same
    collated, track-sorted batch with the same RNG stream (bitwise)."""
    from ensemble_svs_with_interactions_amd import configs, engine
    from ensemble_svs_with_interactions_amd.train import FusedAdam, train_epoch, train_step
    from gpu_util import build

    engine.set_gemm_precision("fp32")
    a, meta = load_case("train_step_tiny")
    Din, Dout = a["x_main"].shape[2], a["y_main"].shape[2]
    rng = np.random.default_rng(5)
    dirs = {k: tmp_path / "dump" / s / d for k, s, d in
            (("in", "norm", "in_acoustic"), ("out", "norm", "out_acoustic"),
             ("times", "org", "in_acoustic"))}
    for d in dirs.values():
        d.mkdir(parents=True)
    spks = ["S", "A", "T", "B"]
    for seg in ("song_001", "song_002"):
        for spk in spks:
            n = int(rng.integers(40, 72))
            sb = data.synthetic_batch(1, n, int(rng.integers(1 << 30)), in_dim=Din,
                                      out_dim=Dout)
            np.save(dirs["in"] / f"{spk}_{seg}-feats.npy", sb["x_main"][0])
            np.save(dirs["out"] / f"{spk}_{seg}-feats.npy", sb["y_main"][0])
            np.save(dirs["times"] / f"{spk}_{seg}-times.npy", np.arange(5) * 50000)
    np.random.seed(1)
    ds, batches = loader.setup_multitrack_batches(str(dirs["in"]), str(dirs["out"]), spks,
                                                  batch_max_frames=400)
    batches = batches[:3]

    def fresh():
        model = build(configs.multitrack_diffusion(num_speakers=4, tiny=True), meta["shapes"])
        model.vuv_model.lstm.dropout = 0.0
        torch.manual_seed(11)
        engine._STATE["rng"] = None
        return model, FusedAdam(model, lr=meta["lr"])

    m1, o1 = fresh()
    got = train_epoch(m1, o1, loader.PairBatchFeeder(ds, batches, device="cuda:0"))
    got = [(l.item(), n.item()) for l, n in got]
    m2, o2 = fresh()
    want = []
    for hb in loader.PairBatchFeeder(ds, batches, device="cpu"):
        c = lambda k: hb[k].cuda().contiguous()  # noqa: E731
        l, n = train_step(m2, o2, c("x_main"), c("x_sub"), c("y_main"), c("spk_main"),
                          c("spk_sub"), [int(v) for v in hb["host_lengths"]])
        want.append((l.item(), n.item()))
    assert len(got) == len(batches) and got == want
    assert all(np.isfinite(v).all() for v in got)
