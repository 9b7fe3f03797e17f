"""Dataset ingest of the HSR object-drop recordings -- the producer side of the
windows the autoencoder trains on.

``TabularDataset(config)`` mirrors ``utils/data_loaders.py:233-434``:

* the ``data_sum{k}.csv`` schema ``concatdata_maker.py:153-181`` writes
  (13 MFCCs ``mfcc00..12``, ``now_timegap``, ``cur_depth_id``,
  ``cur_hand_id``, ``cur_hand_weight``, ``data_dir``, 963 ``LiDAR###``,
  ``label``, ``id``, the index column ``Unnamed: 0``);
* file selection (:258-283): ``file_name != 'data_sum'`` -> only
  ``{file_name}0.csv``; ``object_select_mode`` -> the 8 files filtered to the
  ``objectsplit.csv[object_type]`` recording directories; otherwise the 8
  files; rows shuffled (``sklearn.utils.shuffle``, here seeded by
  ``config.data_seed``) and cut to ``slicing_size`` (:285-286);
* per-sensor selection (:296-330) and the PNG look-ups (:332-365):
  ``{image_root}{data_dir}/data/img/hand/{cur_hand_id}.png`` and
  ``.../img/d/{cur_depth_id}.png`` through PIL ``Image.open(..).resize((32,
  24))`` exactly as the reference calls it (decoded on a thread pool and
  stacked once instead of the reference's O(N^2) ``np.concatenate``);
* ``norm_vec_np`` + view + ``F.interpolate`` (:367-394) as ONE native call per
  modality (``mmad_minmax_norm``, fp64 statistics, raw uint8 / uint16 pixels
  uploaded as they are), then the HSR_Net fusion (:397-424) as one native call
  (``hsr_net.HSR_Net`` -> ``mmad_hsr_fuse``).

``image_root`` (reference: the hard-coded ``/data_ssd/hsr_dropobject/data/``)
comes from ``config.image_root``.  ``.data`` is the fp32 [N, width] device
tensor, ``.targets`` the fp32 labels (host), as the reference's.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from . import _native
from .hsr_net import HSR_Net

IMAGE_ROOT = "/data_ssd/hsr_dropobject/data/"
N_LIDAR = 963
N_MFCC = 13
WIDTH = {"All": 1728, "hand_camera": 1024, "force_torque": 64, "head_depth": 512, "mic": 128}


def lidar_columns():
    """concatdata_maker.py:143-149 / data_loaders.py:305-312 column names."""
    return ["LiDAR%03d" % i for i in range(N_LIDAR)]


def mfcc_columns():
    """utils/data_loaders.py:320-328."""
    return ["mfcc%02d" % i for i in range(N_MFCC)]


def read_data_sum(config):
    """utils/data_loaders.py:258-286 -> the selected, shuffled, sliced rows
    (a pandas DataFrame indexed 0..N-1)."""
    import pandas as pd
    import sklearn.utils

    folder, name = config.data_folder_name, config.file_name
    seed = int(getattr(config, "data_seed", 0))
    if name != "data_sum":
        # the reference's `is not 'data_sum'` identity test (:258): a file name
        # other than the default reads only its first file, unshuffled
        df = pd.read_csv(folder + name + "0.csv")
    else:
        df = pd.concat([pd.read_csv(folder + name + "%d.csv" % k) for k in range(8)],
                       ignore_index=True)
        if getattr(config, "object_select_mode", False):
            objects = pd.read_csv(folder + "objectsplit.csv")[config.object_type].to_list()
            df = df[df["data_dir"].isin(objects)]
        df = sklearn.utils.shuffle(df, random_state=seed)
    df.index = list(range(len(df.index)))
    return df.loc[:config.slicing_size - 1]


def _sensor_flags(sensor):
    """utils/data_loaders.py:243-253 (an unknown sensor sets nothing)."""
    return {k: sensor == k for k in ("All", "hand_camera", "force_torque", "head_depth", "mic")}


def _load_png(path):
    from PIL import Image
    with Image.open(path) as im:
        return np.array(im.resize((32, 24)))


def load_images(paths, workers=16):
    """PIL decode + resize((32, 24)) of every path (utils/data_loaders.py:
    340-352), in row order, stacked into one [N, ...] array of the PNGs'
    own dtype (uint8 RGB, uint16 depth)."""
    if not paths:
        return None
    with ThreadPoolExecutor(max_workers=min(workers, len(paths))) as ex:
        arrs = list(ex.map(_load_png, paths))
    return np.stack(arrs).reshape(len(arrs), -1)


_SRC = {np.dtype(np.float64): 0, np.dtype(np.uint8): 1, np.dtype(np.uint16): 2,
        np.dtype(np.int32): 3, np.dtype(np.float32): 4}


def minmax_norm(v, device, image=False):
    """norm_vec_np over axis 0 of v [N, F] (+ the image view / nearest
    upsampling when ``image``) on the device -> fp32 [N, F'] (mmad_minmax_norm)."""
    v = np.ascontiguousarray(v)
    if v.ndim == 1:
        v = v.reshape(-1, 1)
    if v.dtype not in _SRC:
        v = v.astype(np.float64)
    n, f = v.shape
    lib = _native.load()
    _native.require_gpu()
    src = torch.from_numpy(v.view(np.uint8).reshape(n, -1)).to(device)
    out_w = (f // 768) * 1024 if image else f
    out = torch.empty((n, out_w), device=device, dtype=torch.float32)
    ws_b = int(lib.mmad_minmax_norm_ws_bytes(n, f))
    ws = torch.empty(ws_b, device=device, dtype=torch.uint8)
    _native.call("mmad_minmax_norm", n, f, _native.ptr(src), _SRC[v.dtype], 1 if image else 0,
                 _native.ptr(out), _native.ptr(ws), ws_b, _native.stream_ptr())
    return out


class TabularDataset:
    """utils/data_loaders.py:233-463."""

    def __init__(self, config, transform=None, target_transform=None, device=None, hsr_net=None):
        flags = _sensor_flags(config.sensor)
        if not any(flags.values()):
            # the reference leaves `data` as the raw CSV frame for an unknown
            # sensor (:296-330) and never builds HSR_Net
            raise ValueError("TabularDataset: unknown sensor %r" % (config.sensor,))
        All, hand, ft, depth, mic = (flags[k] for k in ("All", "hand_camera", "force_torque",
                                                        "head_depth", "mic"))
        unimodal = not All
        if device is None:
            device = torch.device("cuda", max(int(getattr(config, "gpu_id", 0)), 0))
        root = getattr(config, "image_root", IMAGE_ROOT)
        df = read_data_sum(config)
        self.rows = df
        n = len(df)
        label = df["label"].to_numpy()
        r = d = t = m = None
        if hand or All:
            paths = [root + dd + "/data/img/hand/" + str(int(i)) + ".png"
                     for dd, i in zip(df["data_dir"], df["cur_hand_id"])]
            if n == 1:
                # the reference's .squeeze() drops the window axis and its
                # view(-1, 1, 3, 32, 32) then fails (:370-372)
                raise RuntimeError("TabularDataset: a single hand-camera window cannot be reshaped")
            r = minmax_norm(load_images(paths), device, image=True).view(n, 1, 3, 32, 32)
        if depth or All:
            paths = [root + dd + "/data/img/d/" + str(int(i)) + ".png"
                     for dd, i in zip(df["data_dir"], df["cur_depth_id"])]
            d = minmax_norm(load_images(paths), device, image=True).view(n, 1, 1, 32, 32)
        if ft or All:
            t = minmax_norm(df["cur_hand_weight"].to_numpy(), device).view(n, 1)
        if mic or All:
            m = minmax_norm(df[mfcc_columns()].to_numpy(), device).view(n, 1, 1, N_MFCC)
        self.inputs = {"r": r, "d": d, "t": t, "m": m}
        net = hsr_net if hsr_net is not None else HSR_Net(unimodal, config).to(device)
        self.hsr_net = net
        with torch.no_grad():
            out = net(r, d, None, t, m)
        self.data = out.reshape(-1, WIDTH[config.sensor])
        self.targets = torch.from_numpy(label.astype(np.float32))
        self.transform = transform
        self.target_transform = target_transform

    def __len__(self):
        return len(self.targets)

    def __getitem__(self, idx):
        return self.data[idx], self.targets[idx]


def has_recordings(config):
    """Is there an HSR data_sum export to ingest (else the synthetic windows)?"""
    folder = getattr(config, "data_folder_name", None)
    name = getattr(config, "file_name", "data_sum")
    return bool(folder) and os.path.exists(folder + name + "0.csv")
