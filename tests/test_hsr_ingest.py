"""Dataset ingest (TabularDataset, utils/data_loaders.py:233-434) against the
reference's own TabularDataset run on the same seeded export
(tests/golden/ingest.npz, tests/golden/gen_ingest_golden.py).

CPU: the oracle restatement of norm_vec_np + view + F.interpolate reproduces
the reference's HSR_Net inputs exactly from the rows / PNGs the product's host
side selects (read_data_sum, load_images): file selection, object filter,
seeded shuffle, slicing, PNG paths and PIL resize all pinned.
GPU: the native path (mmad_minmax_norm + mmad_hsr_fuse) gives the reference's
inputs bit for bit and its dataset rows within 2e-6 (the fusion's fp32 sums
run in a different order than torch's CPU convolutions, tests/test_hsr.py)."""
import types

import numpy as np
import pytest
import torch

from oracle import ingest_oracle as IO
from tests.hsr_fixture import CASES, SHUFFLE_SEED, write_recordings


@pytest.fixture(scope="module")
def export(tmp_path_factory):
    return write_recordings(str(tmp_path_factory.mktemp("hsr")))


def _cfg(export, name):
    folder, img = export
    return types.SimpleNamespace(data_folder_name=folder, image_root=img, gpu_id=0,
                                 data_seed=SHUFFLE_SEED, **CASES[name])


@pytest.mark.parametrize("name", list(CASES))
def test_host_selection_and_oracle_match_reference(golden, export, name):
    from icra2021_multimodal_ad_amd import hsr_dataset as H
    g = golden("ingest")
    cfg = _cfg(export, name)
    df = H.read_data_sum(cfg)
    n = len(df)
    assert n == cfg.slicing_size
    np.testing.assert_array_equal(df["label"].to_numpy().astype(np.float32), g[f"{name}/targets"])
    sensor = cfg.sensor
    if sensor in ("All", "force_torque"):
        t = IO.flat_input(df["cur_hand_weight"].to_numpy()).reshape(n, 1)
        np.testing.assert_array_equal(t, g[f"{name}/in_t"])
    if sensor in ("All", "mic"):
        m = IO.flat_input(df[H.mfcc_columns()].to_numpy()).reshape(n, 1, 1, 13)
        np.testing.assert_array_equal(m, g[f"{name}/in_m"])
    root = cfg.image_root
    if sensor in ("All", "hand_camera"):
        px = H.load_images([root + dd + "/data/img/hand/" + str(int(i)) + ".png"
                            for dd, i in zip(df["data_dir"], df["cur_hand_id"])])
        assert px.dtype == np.uint8 and px.shape == (n, 24 * 32 * 3)
        np.testing.assert_array_equal(IO.image_input(px, 3).reshape(n, 1, 3, 32, 32),
                                      g[f"{name}/in_r"])
    if sensor in ("All", "head_depth"):
        px = H.load_images([root + dd + "/data/img/d/" + str(int(i)) + ".png"
                            for dd, i in zip(df["data_dir"], df["cur_depth_id"])])
        np.testing.assert_array_equal(IO.image_input(px, 1).reshape(n, 1, 1, 32, 32),
                                      g[f"{name}/in_d"])


def test_unknown_sensor_and_single_window(export):
    from icra2021_multimodal_ad_amd import hsr_dataset as H
    cfg = _cfg(export, "All")
    cfg.sensor = "lidar"
    with pytest.raises(ValueError):
        H.TabularDataset(cfg)


def _net_from_golden(g, unimodal, n):
    from icra2021_multimodal_ad_amd.hsr_net import HSR_Net
    net = HSR_Net(unimodal, types.SimpleNamespace(slicing_size=n))
    net.load_state_dict({k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("w_")})
    return net.cuda()


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_native_ingest_matches_reference(golden, export, name):
    from icra2021_multimodal_ad_amd import hsr_dataset as H
    g = golden("ingest")
    cfg = _cfg(export, name)
    net = _net_from_golden(g, cfg.sensor != "All", cfg.slicing_size)
    ds = H.TabularDataset(cfg, hsr_net=net)
    for k, v in ds.inputs.items():
        if v is not None:
            assert torch.equal(v.cpu(), torch.from_numpy(g[f"{name}/in_{k}"])), k
    ref = g[f"{name}/data"]
    got = ds.data.cpu().numpy()
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 2e-6 * max(1.0, np.abs(ref).max())
    np.testing.assert_array_equal(ds.targets.numpy(), g[f"{name}/targets"])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.uint8, np.uint16, np.int32, np.float32, np.float64])
def test_minmax_norm_kernel_matches_oracle(dtype):
    """mmad_minmax_norm on ragged shapes (n not a multiple of the 1024-row
    partial, constant columns) for every source type, both layouts."""
    from icra2021_multimodal_ad_amd import hsr_dataset as H
    rng = np.random.default_rng(3)
    for n, f, image in ((1, 5, False), (2500, 37, False), (1300, 768 * 3, True), (3, 768, True)):
        if np.issubdtype(dtype, np.integer):
            v = rng.integers(0, 200, size=(n, f)).astype(dtype)
        else:
            v = rng.normal(size=(n, f)).astype(dtype)
        v[:, 0] = v[0, 0]                       # a constant column -> 0
        got = H.minmax_norm(v, "cuda", image=image).cpu().numpy()
        # fp32 sources are normalised in float64 like every other source (the
        # reference's own streams are uint8 / uint16 PNGs and float64 CSVs)
        w = v.astype(np.float64) if dtype == np.float32 else v
        want = IO.image_input(w, f // 768).reshape(n, -1) if image else IO.flat_input(w)
        np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
def test_get_loaders_on_recordings(golden, export):
    """get_loaders (utils/data_loaders.py:50-138) over the export: the
    manager ingests it (not the synthetic windows), 60/20/20 of the normal
    windows + all drops in test, (x [B, 1728], y [B]) batches on the device."""
    from icra2021_multimodal_ad_amd.data_loaders import get_loaders
    g = golden("ingest")
    cfg = _cfg(export, "All")
    cfg.data, cfg.target_class, cfg.unimodal_normal = "hsr_objectdrop", 1, False
    cfg.batch_size, cfg.novelty_ratio, cfg.verbose = 7, 0.0, 0
    torch.manual_seed(100)
    mgr, train, valid, test = get_loaders(cfg)
    y = g["All/targets"]
    assert mgr.total_x.shape == (40, 1728) and mgr.total_x.is_cuda
    np.testing.assert_array_equal(mgr.total_y.numpy(), y)
    n_norm = int((y == 0).sum())
    assert len(train.sampler) == int(0.6 * n_norm)
    assert len(test.sampler) == n_norm - int(0.8 * n_norm) + int((y == 1).sum())
    xb, yb = next(iter(train))
    assert xb.shape == (7, 1728) and xb.is_cuda and yb.shape == (7,)
    assert float(yb.max()) == 0.0
