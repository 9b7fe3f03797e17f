"""The executor's kernel probe (mmad_ae_probe, the bench's roofline timing):
every kind records one duration per step for the probed launch, and probing
never changes a result bit -- the marker-event kinds (0 / 1, the main-stream
launch started after the side stream's work) and the kernel-attached kinds
(2 / 3, hipExtLaunchKernel start / stop events on the launch itself, which
bench.py leaves on through its timed region)."""
import ctypes

import pytest
import torch

from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd.data import synth_windows

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,layer", [(0, 0), (1, 0), (2, 0), (3, 0), (3, 9)])
def test_probe_records_each_step_and_keeps_bits(kind, layer):
    import types
    from icra2021_multimodal_ad_amd.model_builder import get_model
    lib = _native.load()
    ms = []
    for _ in range(2):
        cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16",
                                    models="ae")
        torch.manual_seed(8)
        ms.append(get_model(cfg))
    ms[1].load_state_dict(ms[0].state_dict())
    for m in ms:
        m._native.sync_shadow(force=True)
    steps = 4
    assert lib.mmad_ae_probe(ms[1]._native._h, kind, layer, steps) == 0
    for s in range(steps):
        x = torch.from_numpy(synth_windows(1024, 2048, seed=70 + s)).cuda()
        la = float(ms[0]._native.train_step_fused(x))
        lb = float(ms[1]._native.train_step_fused(x))
        assert la == lb, (s, la, lb)
    torch.cuda.synchronize()
    buf = (ctypes.c_float * steps)()
    n = lib.mmad_ae_probe_read(ms[1]._native._h, buf, steps)
    assert n == steps
    assert all(0.0 < buf[i] < 50.0 for i in range(n)), list(buf)
    mask = lib.mmad_ae_probe_layers(ms[1]._native._h)
    assert mask > 0 and (mask >> layer) & 1
    assert lib.mmad_ae_probe(ms[1]._native._h, 1, -1, 0) == 0
    a, b = ms[0]._native, ms[1]._native
    for name in ("params", "exp_avg", "exp_avg_sq", "running"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert lib.mmad_ae_probe(ms[1]._native._h, 4, 0, 1) != 0   # no such kind
