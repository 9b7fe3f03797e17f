"""CPU oracle for the dataset ingest (TabularDataset, utils/data_loaders.py:
233-434) -- the normalisation and re-layout it applies to the sensor streams.

TEST INFRASTRUCTURE ONLY.  Only ``tests/`` may import it; the product
(``icra2021_multimodal_ad_amd.hsr_dataset``) never imports, calls or falls back
to anything here.  Pinned against ``tests/golden/ingest.npz`` (the reference's
own TabularDataset run on the seeded export of ``tests/hsr_fixture.py``,
``tests/golden/gen_ingest_golden.py``) by ``tests/test_hsr_ingest.py``.
"""
import numpy as np


def norm_vec_np(v):
    """utils/data_loaders.py:447-456 with the default ranges: per column
    (v - min) / (max - min) in float64 (integer arrays subtract exactly in
    their own dtype first, as numpy does there), NaN -> 0."""
    v = np.asarray(v)
    lo, hi = v.min(axis=0), v.max(axis=0)
    with np.errstate(invalid="ignore", divide="ignore"):
        out = (1.0 * (v - lo)) / (hi - lo)
    return np.nan_to_num(out)


def image_input(pixels, channels):
    """utils/data_loaders.py:367-378: norm_vec_np of the [N, 24*32*C]
    HWC-flattened pixels, cast to fp32, reinterpreted (view) as [N, C, 24, 32]
    and nearest-upsampled to 32 rows (F.interpolate(size=32): src row =
    floor(y * 24 / 32)) -> [N, C, 32, 32]."""
    n = pixels.shape[0]
    r = norm_vec_np(pixels).astype(np.float32).reshape(n, channels, 24, 32)
    src = (np.arange(32) * 24) // 32
    return r[:, :, src, :]


def flat_input(v):
    """utils/data_loaders.py:380-394 (F/T weight, MFCCs): norm_vec_np -> fp32."""
    return norm_vec_np(v).astype(np.float32)
