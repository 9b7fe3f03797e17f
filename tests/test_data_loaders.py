"""Batch-supply contract (utils/data_loaders.py:31-138, :465-598) on CPU:
label split, 60/20/20 index cuts, test = test-normal + novelties, novelty
ratio balancing, train order reshuffled every epoch (seeded), sequential
valid/test, (x [B, D], y [B]) batches without drop_last, and
get_transformed_data in sampler order."""
import types

import numpy as np
import torch

from icra2021_multimodal_ad_amd.data_loaders import (BatchLoader, TabularDatasetManager, get_balance,
                                                     get_loaders, split_labels)


def _cfg(**kw):
    c = dict(input_size=64, sensor="force_torque", data="hsr_objectdrop", target_class=1,
             unimodal_normal=False, novelty_ratio=0.0, batch_size=128, gpu_id=-1, n_normal=1000,
             n_novelty=150, data_seed=3, verbose=0)
    c.update(kw)
    return types.SimpleNamespace(**c)


def test_label_split_rules():
    assert split_labels(_cfg()) == ([0], [1])
    assert split_labels(_cfg(unimodal_normal=True)) == ([1], [0])
    c = _cfg(target_class="1")            # not in [0, 1]: hsr_objectdrop falls back to labels[1]
    assert split_labels(c) == ([0], [1]) and c.target_class == 1
    assert split_labels(_cfg(), use_full_class=True) == ([0, 1], [])


def test_index_splits_and_loaders():
    cfg = _cfg()
    dm, tr, va, te = get_loaders(cfg)
    y = dm.total_y.numpy()
    seen = list(np.where(np.isin(y, [0]))[0])
    cuts = [int(e) for e in (np.array([0.6, 0.2, 0.2]).cumsum()[:-1] * len(seen))]  # :521
    assert list(tr.sampler.indices) == seen[:cuts[0]]
    assert list(va.sampler.indices) == seen[cuts[0]:cuts[1]]
    unseen = list(np.where(y == 1)[0])
    assert list(te.sampler.indices) == seen[cuts[1]:] + unseen
    # train order: a fresh permutation of the same subset every pass
    e1, e2 = list(iter(tr.sampler)), list(iter(tr.sampler))
    assert sorted(e1) == sorted(seen[:cuts[0]]) and e1 != e2
    # ... and reproducible from the seed
    dm2, tr2, _, _ = get_loaders(_cfg())
    assert list(iter(tr2.sampler)) == e1
    # batches: (x [B, D], y [B]), last one short, sampler order
    batches = list(va)
    assert [b[0].shape[0] for b in batches] == [128] * (len(va.sampler) // 128) + \
        ([len(va.sampler) % 128] if len(va.sampler) % 128 else [])
    assert len(batches) == len(va)
    x_all = torch.cat([b[0] for b in batches])
    xt, yt = dm.get_transformed_data(va)
    assert torch.equal(x_all, xt) and torch.equal(yt, dm.total_y[va.sampler.indices])
    assert torch.equal(xt, dm.total_x[va.sampler.indices])
    assert xt.shape[1] == 64 and yt.dtype == torch.float32


def test_novelty_ratio_balancing():
    rng = np.random.Generator(np.random.PCG64(0))
    seen, unseen = list(range(100)), list(range(100, 140))
    s, u = get_balance(seen, unseen, 0.1, rng)            # too many novelties: drop some
    assert s == seen and len(u) == int(100 * 0.1 / 0.9) and set(u) <= set(unseen)
    s, u = get_balance(seen, unseen, 0.5, rng)            # too few: drop normals
    assert u == unseen and len(s) == int(40 / 0.5 - 40)
    assert get_balance(seen, unseen, 0.0) == (seen, unseen)
    dm, tr, va, te = get_loaders(_cfg(novelty_ratio=0.2))
    y = dm.total_y.numpy()[te.sampler.indices]
    assert abs(y.mean() - 0.2) < 0.01


def test_dataset_is_seeded_and_labelled():
    a = TabularDatasetManager(_cfg())
    b = TabularDatasetManager(_cfg())
    c = TabularDatasetManager(_cfg(data_seed=4))
    assert torch.equal(a.total_x, b.total_x) and not torch.equal(a.total_x, c.total_x)
    assert int(a.total_y.sum()) == 150 and a.total_size == 1150
    tr, va, te = a.get_loaders(500, indexes_list=[[0, 1], [2], [3, 4]])
    assert [x.shape[0] for x, _ in va] == [1] and [x.shape[0] for x, _ in te] == [2]
    assert isinstance(tr, BatchLoader) and sorted(tr.sampler) == [0, 1]


def test_dp_tail_batch_too_small_for_every_rank_is_dropped():
    """world 2, batch 4: 9 windows = two global batches of 8 and a tail of 1
    (< 2 * world) -- dropped on both ranks; a tail of 4 (= 2 rows per rank) is
    kept.  No rank ever gets fewer than 2 rows; both ranks yield the same
    number of batches; single process keeps every window."""
    from icra2021_multimodal_ad_amd.data_loaders import SequentialIndicesSampler
    ds = types.SimpleNamespace(data=torch.arange(20, dtype=torch.float32)[:, None],
                               targets=torch.zeros(20))
    for n, want in ((17, 2), (20, 3), (19, 2), (21, 3)):
        if n > 20:
            ds = types.SimpleNamespace(data=torch.arange(n, dtype=torch.float32)[:, None],
                                       targets=torch.zeros(n))
        lens = []
        for rank in (0, 1):
            ld = BatchLoader(ds, 4, SequentialIndicesSampler(list(range(n))), rank, 2)
            got = [x.shape[0] for x, _ in ld]
            assert len(got) == len(ld) == want, (n, rank, got)
            assert min(got) >= 2, (n, rank, got)
            lens.append(got)
        assert len(lens[0]) == len(lens[1])
        single = BatchLoader(ds, 4, SequentialIndicesSampler(list(range(n))), 0, 1)
        assert sum(x.shape[0] for x, _ in single) == n
