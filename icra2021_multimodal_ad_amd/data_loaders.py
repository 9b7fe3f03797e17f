"""Batch supply with the reference's contract (utils/data_loaders.py):
``get_loaders(config) -> (dset_manager, train_loader, valid_loader,
test_loader)``, loaders yielding ``(x [B, D], y [B])`` with the data already
resident on the GPU, ``TabularDatasetManager.get_indexes`` /
``get_transformed_data`` / ``get_loaders``.

What is kept from the reference (file:line):
* label split (:50-90): ``labels`` of the dataset config ([0, 1] for
  hsr_objectdrop), the target class is the novelty (unseen) class unless
  ``unimodal_normal``; a target class not in the label set falls back to
  labels[1] for hsr_objectdrop, labels[0] otherwise (:63-67);
* index splits (:507-526): ``np.where(np.isin(y, labels))`` in dataset order,
  cut at ``int(cumsum(ratios)[:-1] * len)``; seen labels 60/20/20 into
  train/valid/test-normal, all unseen to test (:100-132); ``get_balance``
  (:31-48) to a novelty ratio;
* loaders (:554-598): train draws a fresh random order over its indices every
  epoch (SubsetRandomSampler), valid/test are sequential
  (SequentialIndicesSampler), ``num_workers=0``, no ``drop_last``;
* ``get_transformed_data`` (:528-552): the whole split in sampler order --
  here ONE device gather instead of the per-index Python loop.

The dataset is the HSR export when ``config.data_folder_name`` holds one
(``hsr_dataset.TabularDataset``: the data_sum CSV schema, PNG look-ups, native
normalisation and HSR_Net fusion), else the seeded synthetic window generator
(data.synth_windows; the HSR recordings are not public, README.md:15); every
random choice (row order, sampler order, balancing) comes from a seeded
numpy PCG64 generator, so a run is reproducible and the reference can be fed
the very same batches (tests/golden/gen_e2e.py).
"""
import numpy as np
import torch

from .data import SENSOR_WIDTH, synth_windows

DATA_CONFIG = {"hsr_objectdrop": {"labels": [0, 1]}}   # datasets/data_config.json:115-124


def get_input_size(config):
    """utils/data_loaders.py:16-29."""
    return SENSOR_WIDTH.get(config.sensor)


def get_balance(seen_index_list, unseen_index_list, novelty_ratio=.5, rng=None):
    """utils/data_loaders.py:31-48 (np.random.choice -> the seeded rng)."""
    if novelty_ratio <= 0.:
        return seen_index_list, unseen_index_list
    rng = rng or np.random.Generator(np.random.PCG64(0))
    current_ratio = len(unseen_index_list) / (len(seen_index_list) + len(unseen_index_list))
    if current_ratio < novelty_ratio:
        target_seen_cnt = int(len(unseen_index_list) / novelty_ratio - len(unseen_index_list))
        return list(rng.choice(seen_index_list, target_seen_cnt, replace=False)), unseen_index_list
    if current_ratio > novelty_ratio:
        target_unseen_cnt = int((len(seen_index_list) * novelty_ratio) / (1 - novelty_ratio))
        return seen_index_list, list(rng.choice(unseen_index_list, target_unseen_cnt, replace=False))
    return seen_index_list, unseen_index_list


class SequentialIndicesSampler:
    """utils/data_loaders.py:141-149."""

    def __init__(self, indices):
        self.indices = list(indices)

    def __iter__(self):
        return iter(self.indices)

    def __len__(self):
        return len(self.indices)


class SubsetRandomSampler:
    """torch SubsetRandomSampler semantics (a new permutation of the subset on
    every pass) with a seeded numpy generator."""

    def __init__(self, indices, seed=0):
        self.indices = list(indices)
        self.rng = np.random.Generator(np.random.PCG64(seed))

    def __iter__(self):
        perm = self.rng.permutation(len(self.indices))
        return iter([self.indices[i] for i in perm])

    def __len__(self):
        return len(self.indices)


class BatchLoader:
    """torch DataLoader(dataset, batch_size, sampler, num_workers=0) over a
    device-resident dataset: each batch is one gather of the sampler's
    indices, ``(x [B, D] on the data's device, y [B] float32 on the host)``;
    the last batch may be short (drop_last=False).

    Data parallel (world > 1): every rank draws the same sampler order (same
    seed), a global batch is ``batch_size * world`` windows and this rank gets
    its contiguous rows of it (dist.shard_rows), so the ranks together step
    through exactly the single-process sequence of windows.  The one
    exception: a last global batch of fewer than 2 * world windows is dropped
    on every rank (the decision depends only on the global count, so all ranks
    agree) -- some shard would get 0 rows (no native step exists for it, while
    the other ranks wait in the exchange) or 1 row (train-mode BatchNorm over
    one window, which torch's BatchNorm1d refuses too)."""

    def __init__(self, dataset, batch_size, sampler, rank=0, world=1):
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.sampler = sampler
        self.rank, self.world = int(rank), int(world)

    def _global_batches(self):
        n, gb = len(self.sampler), self.batch_size * self.world
        starts = list(range(0, n, gb))
        if self.world > 1 and starts and n - starts[-1] < 2 * self.world:
            starts.pop()
        return starts

    def __iter__(self):
        order = np.fromiter(iter(self.sampler), dtype=np.int64, count=len(self.sampler))
        dev = self.dataset.data.device
        gb = self.batch_size * self.world
        for s in self._global_batches():
            idx = order[s:s + gb]
            if self.world > 1:
                q, r = divmod(len(idx), self.world)
                lo = self.rank * q + min(self.rank, r)
                idx = idx[lo:lo + q + (1 if self.rank < r else 0)]
            yield (self.dataset.data[torch.from_numpy(idx).to(dev)],
                   self.dataset.targets[torch.from_numpy(idx)])

    def __len__(self):
        return len(self._global_batches())


class SyntheticWindowDataset:
    """TabularDataset counterpart (utils/data_loaders.py:233-463): ``.data``
    [N, D] fp32 (on ``device``), ``.targets`` [N] fp32 labels (0 normal, 1
    object drop).  n_normal normal windows and n_novelty anomalous ones
    (data.synth_windows), rows in a seeded random order (the reference
    shuffles its CSV rows, :287)."""

    def __init__(self, config, device="cpu"):
        d = get_input_size(config) if getattr(config, "input_size", None) is None else \
            int(config.input_size)
        n_normal = int(getattr(config, "n_normal", 3000))
        n_novelty = int(getattr(config, "n_novelty", 600))
        seed = int(getattr(config, "data_seed", 0))
        strength = float(getattr(config, "anomaly_strength", 1.0))
        rng = np.random.Generator(np.random.PCG64(seed))
        normal = synth_windows(n_normal, d, rng=rng)
        anom = synth_windows(n_novelty, d, rng=rng, anomaly=np.ones(n_novelty, bool), strength=strength)
        x = np.concatenate([normal, anom])
        y = np.concatenate([np.zeros(n_normal, np.float32), np.ones(n_novelty, np.float32)])
        perm = rng.permutation(len(x))
        self.data = torch.from_numpy(x[perm]).to(device)
        self.targets = torch.from_numpy(y[perm])
        self.transform = None
        self.target_transform = None

    def __len__(self):
        return len(self.targets)

    def __getitem__(self, idx):
        return self.data[idx], self.targets[idx]


class TabularDatasetManager:
    """utils/data_loaders.py:465-598."""

    def __init__(self, config, dataset=None, device="cpu", shuffle=False, data_size=0):
        if dataset is None:
            dataset = self._get_dataset(config, device)
        self.train_dataset = dataset
        # :476-486: the last data_size windows (0 = all), optionally permuted
        x, y = dataset.data, dataset.targets
        if data_size:
            x, y = x[-data_size:], y[-data_size:]
        if shuffle:
            rng = np.random.Generator(np.random.PCG64(int(getattr(config, "data_seed", 0)) + 2))
            perm = torch.from_numpy(rng.permutation(len(x)))
            x, y = x[perm.to(x.device)], y[perm]
        dataset.data, dataset.targets = x, y
        self.total_x = x
        self.total_y = y
        self.total_size = len(self.total_x)
        self.sampler_seed = int(getattr(config, "sampler_seed", getattr(config, "data_seed", 0)))

    @staticmethod
    def _get_dataset(config, device):
        """utils/data_loaders.py:501-505: the HSR recordings when an export is
        there (config.data_folder_name / file_name, hsr_dataset.TabularDataset),
        else the seeded synthetic windows."""
        from .hsr_dataset import TabularDataset, has_recordings
        if has_recordings(config):
            return TabularDataset(config, device=device)
        return SyntheticWindowDataset(config, device)

    def get_indexes(self, ratios=None, labels=None):
        """utils/data_loaders.py:507-526."""
        if labels is not None:
            if not isinstance(labels, (list, tuple, np.ndarray)):
                labels = [labels]
            indexes = list(np.where(np.isin(self.total_y.numpy(), labels))[0])
        else:
            indexes = list(range(self.total_size))
        if ratios:
            assert sum(ratios) == 1
            if len(ratios) == 1:
                return indexes
            ratios = np.array(ratios)
            cuts = [int(e) for e in (ratios.cumsum()[:-1] * len(indexes))]
            return [list(ix) for ix in np.split(np.asarray(indexes, dtype=np.int64), cuts)]
        return [indexes]

    def get_transformed_data(self, data_loader):
        """utils/data_loaders.py:528-552: the split in sampler order, one gather."""
        idx = np.fromiter(iter(data_loader.sampler), dtype=np.int64, count=len(data_loader.sampler))
        ds = data_loader.dataset
        return ds.data[torch.from_numpy(idx).to(ds.data.device)], ds.targets[torch.from_numpy(idx)]

    def get_loaders(self, batch_size, ratios=None, indexes_list=None, use_gpu=False, rank=0, world=1):
        """utils/data_loaders.py:554-598 (rank / world: data-parallel shards
        of every batch, BatchLoader)."""
        if ratios and indexes_list:
            raise Exception("Only either `ratios` or `indexes_list` is allowed")
        elif ratios:
            indexes_list = self.get_indexes(ratios=ratios)
        loaders = [BatchLoader(self.train_dataset, batch_size,
                               SubsetRandomSampler(indexes_list[0], seed=self.sampler_seed), rank, world)]
        for ix in indexes_list[1:3]:
            loaders.append(BatchLoader(self.train_dataset, batch_size, SequentialIndicesSampler(ix),
                                       rank, world))
        return loaders


def split_labels(config, use_full_class=False):
    """utils/data_loaders.py:59-82: (seen, unseen) label lists."""
    class_list = DATA_CONFIG.get(config.data, DATA_CONFIG["hsr_objectdrop"])["labels"]
    if config.target_class not in class_list:
        config.target_class = class_list[1] if config.data == "hsr_objectdrop" else class_list[0]
    seen, unseen = [], []
    for i in class_list:
        if use_full_class:
            seen += [i]
            continue
        if i != config.target_class:
            (unseen if config.unimodal_normal else seen).append(i)
        else:
            (seen if config.unimodal_normal else unseen).append(i)
    return seen, unseen


def get_loaders(config, use_full_class=False, device=None, rank=0, world=1):
    """utils/data_loaders.py:50-138 (rank / world: data-parallel batch shards)."""
    if config.data not in DATA_CONFIG:
        raise ValueError("no dataset config for" + config.data)
    if device is None:
        gpu = getattr(config, "gpu_id", 0)
        device = torch.device("cuda", gpu) if gpu >= 0 and torch.cuda.is_available() else "cpu"
    seen, unseen = split_labels(config, use_full_class)
    dset_manager = TabularDatasetManager(config, device=device)
    if use_full_class:
        s = dset_manager.get_indexes(labels=seen, ratios=[0.6, 0.2, 0.2])
        indexes_list = [s[0], s[1], s[2]]
    else:
        s = dset_manager.get_indexes(labels=seen, ratios=[0.6, 0.2, 0.2])
        u = dset_manager.get_indexes(labels=unseen)
        rng = np.random.Generator(np.random.PCG64(int(getattr(config, "data_seed", 0)) + 1))
        s[2], u[0] = get_balance(s[2], u[0], getattr(config, "novelty_ratio", 0.0), rng=rng)
        if getattr(config, "verbose", 0) >= 1:
            print("After balancing:\t|train|=%d |valid|=%d |test_normal|=%d |test_novelty|=%d "
                  "|novelty_ratio|=%.4f" % (len(s[0]), len(s[1]), len(s[2]), len(u[0]),
                                           len(u[0]) / max(len(u[0]) + len(s[2]), 1)))
        indexes_list = [s[0], s[1], list(s[2]) + list(u[0])]
    train, valid, test = dset_manager.get_loaders(batch_size=config.batch_size,
                                                  indexes_list=indexes_list, rank=rank, world=world)
    return dset_manager, train, valid, test
