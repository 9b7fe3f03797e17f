"""Synthetic sensor windows in the reference's fused layout.

The reference's real data (HSR object-drop recordings) is not public
(README.md:15), so the hot path is fed seeded synthetic windows shaped like the
tensor ``utils/data_loaders.py:400-404`` hands to the model: one 0.1 s window =
the HSR_Net fusion output [27 x 8 x 8] flattened channel-major:

  [0, 1024)     RGB hand camera conv features (16 ch)   ~50 % zeros, mean 0.03
  [1024, 1536)  head depth conv features (8 ch)         ~46 % zeros, mean 0.033
  [1536, 1600)  force/torque scalar broadcast x64       (data_loaders.py:213)
  [1600, 1728)  mic MFCC conv, 16 values each x8        (data_loaders.py:218-220)
  [1728, D)     aligned-width filler for D=2048

``D=64`` is the F/T-only case (one U[0,1] scalar x 64).  Anomalies (object
slip/drop) shift the F/T scalar by +0.6 and scale the RGB block by 1.5
(SURVEY §8(d)).  Sensor -> width follows get_input_size
(utils/data_loaders.py:16-29).
"""
import numpy as np

SENSOR_WIDTH = {"All": 1728, "hand_camera": 1024, "force_torque": 64,
                "head_depth": 512, "LiDAR": 2048, "mic": 128}


def get_input_size(config):
    """utils/data_loaders.py:16-29 (config.sensor -> flattened width)."""
    return SENSOR_WIDTH.get(config.sensor)


def _relu_normal(rng, mean, sd, shape):
    return np.maximum(rng.normal(mean, sd, shape), 0.0)


def synth_windows(n, d, seed=0, anomaly=None, rng=None, strength=1.0):
    """n windows of width d (float32, [n, d]).  ``anomaly`` is a bool mask of
    length n (True = anomalous window) or None; ``strength`` scales the
    anomaly (F/T shift 0.6*strength, RGB gain 1 + 0.5*strength)."""
    rng = rng or np.random.Generator(np.random.PCG64(seed))
    x = np.zeros((n, d), np.float64)
    ft = rng.uniform(0.0, 1.0, (n, 1))
    if anomaly is not None:
        anomaly = np.asarray(anomaly, bool)
        ft = ft + (0.6 * strength) * anomaly[:, None]
    if d == 64:
        x[:] = ft
        return x.astype(np.float32)
    if d < 1728:
        # unimodal widths: a scaled-down copy of the fused layout statistics
        x[:] = _relu_normal(rng, 0.0, 0.075, (n, d))
        x[:, : min(64, d)] = ft
        return x.astype(np.float32)
    rgb = _relu_normal(rng, 0.0, 0.075, (n, 1024))
    if anomaly is not None:
        rgb = rgb * np.where(anomaly[:, None], 1.0 + 0.5 * strength, 1.0)
    x[:, 0:1024] = rgb
    x[:, 1024:1536] = _relu_normal(rng, 0.01, 0.08, (n, 512))
    x[:, 1536:1600] = ft
    mic = _relu_normal(rng, 0.04, 0.2, (n, 16))
    x[:, 1600:1728] = np.repeat(mic, 8, axis=1)
    if d > 1728:
        x[:, 1728:d] = _relu_normal(rng, 0.0, 0.075, (n, d - 1728))
    return x.astype(np.float32)


def synth_split(n_normal, n_anomaly, d, seed=0):
    """Normal windows split 60/20/20 into train/valid/test-normal; the test set
    is test-normal + all anomalies (utils/data_loaders.py:100,128-132).
    Returns dict(train, valid, test, test_label) with label True = anomaly."""
    rng = np.random.Generator(np.random.PCG64(seed))
    normal = synth_windows(n_normal, d, rng=rng)
    anom = synth_windows(n_anomaly, d, rng=rng, anomaly=np.ones(n_anomaly, bool))
    n_tr = int(0.6 * n_normal)
    n_va = int(0.8 * n_normal) - n_tr
    test = np.concatenate([normal[n_tr + n_va:], anom])
    label = np.concatenate([np.zeros(n_normal - n_tr - n_va, bool), np.ones(n_anomaly, bool)])
    return {"train": normal[:n_tr], "valid": normal[n_tr:n_tr + n_va], "test": test,
            "test_label": label}


def synth_windows_device(n, d, device, seed=0, dtype=None):
    """Same distribution as ``synth_windows`` drawn on the device with torch's
    generator (bench / streaming inputs; not bit-identical to the numpy draw)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    dtype = dtype or torch.float32
    if d == 64:
        return torch.rand((n, 1), generator=g, device=device).expand(n, 64).contiguous().to(dtype)
    x = torch.empty((n, d), device=device, dtype=torch.float32)
    if d < 1728:
        x.normal_(0.0, 0.075, generator=g).clamp_(min=0)
        x[:, : min(64, d)] = torch.rand((n, 1), generator=g, device=device)
        return x.to(dtype)
    x[:, 0:1024].normal_(0.0, 0.075, generator=g)
    x[:, 1024:1536].normal_(0.01, 0.08, generator=g)
    x[:, 0:1536].clamp_(min=0)
    x[:, 1536:1600] = torch.rand((n, 1), generator=g, device=device)
    mic = torch.empty((n, 16), device=device).normal_(0.04, 0.2, generator=g).clamp_(min=0)
    x[:, 1600:1728] = mic.repeat_interleave(8, dim=1)
    if d > 1728:
        x[:, 1728:d].normal_(0.0, 0.075, generator=g).clamp_(min=0)
    return x.to(dtype)
