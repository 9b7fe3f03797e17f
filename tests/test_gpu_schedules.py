"""Fused-step schedule variants give the same bits as the default schedule:
every schedule knob of the tune table (include/mmad.h knobs 15, 19-31, 33-35, read when
a model handle is created) and the host-side shadow pair only reorder
independent work across streams."""
import pytest
import torch

from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd.data import synth_windows

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("knobs", [
    {"ev_every": 1}, {"ev_every": 3}, {"loss_side": 0}, {"dw_main": 1}, {"dw_main": 3},
    {"pair_rows": 0}, {"pair_rows": 0, "dw_main_ping": 0}, {"shadow_pair": False},
    {"side_prio": 1}, {"event_sysfence": 1}, {"keep_grads": 1}, {"ev_on_kernel": 0},
    {"side_cu_held": 32}, {"pair_rows": 0, "dw_late": 1}, {"pair_rows": 0, "dw_late": 99},
    {"pair_rows": 0, "fork_on_kernel": 0}, {"pair_rows": 0, "fork_on_kernel": 0, "ev_on_kernel": 0},
    {"pair_rows": 0, "fork_pair_below": 4}, {"pair_rows": 0, "fork_pair_below": 9},
    {"pair_rows": 0, "fork_pair_below": 9, "fork_on_kernel": 0}])
def test_schedule_knobs_match_default(knobs):
    """Every schedule knob of the fused step only reorders independent work
    across streams (event coalescing, where the loss is reduced, how many dW
    GEMMs run on the main stream, ping-pong shadows, stream priority, event
    fences, a materialised dW, hand-off events on the launch or behind it, a
    CU-masked side stream): parameters, Adam moments, BN statistics, the
    current bf16 shadow and the losses equal the default schedule's bit for
    bit."""
    import types
    from icra2021_multimodal_ad_amd.model_builder import get_model
    ms = []
    for variant in (True, False):
        cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16",
                                    models="ae")
        torch.manual_seed(8)
        with _native.tune(**(knobs if variant else {})):
            ms.append(get_model(cfg))
    ms[1].load_state_dict(ms[0].state_dict())
    for m in ms:
        m._native.sync_shadow(force=True)
    for s in range(3):
        x = torch.from_numpy(synth_windows(1024, 2048, seed=40 + s)).cuda()
        la, lb = (float(m._native.train_step_fused(x)) for m in ms)
        assert la == lb, (s, la, lb)
    for m in ms:
        m._native.check_status()
    a, b = ms[0]._native, ms[1]._native
    for name in ("params", "exp_avg", "exp_avg_sq", "running"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert torch.equal(a.shadow, b.shadow)
    assert torch.equal(a.shadow, a.params[: a.n_weight].bfloat16())


@pytest.mark.parametrize("tile", [0, 5])
def test_adam_fused_dw_tiles_match_default(tile):
    """The Adam-fused dW GEMM on another tile -- 128x128 with 8 waves (cfg 0)
    or 4 waves (cfg 5) instead of the default shape rule, forced through
    knob 5 for every call -- gives the default schedule's bits: parameters,
    Adam moments, BN statistics, the bf16 shadow and the losses."""
    import types
    from icra2021_multimodal_ad_amd.model_builder import get_model
    cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16",
                                models="ae")
    torch.manual_seed(8)
    ma = get_model(cfg)
    mb = get_model(cfg)
    mb.load_state_dict(ma.state_dict())
    for m in (ma, mb):
        m._native.sync_shadow(force=True)
    for s in range(3):
        x = torch.from_numpy(synth_windows(1024, 2048, seed=40 + s)).cuda()
        la = float(ma._native.train_step_fused(x))
        with _native.tune(tile_adam=tile):
            lb = float(mb._native.train_step_fused(x))
        assert la == lb, (s, la, lb)
    for m in (ma, mb):
        m._native.check_status()
    a, b = ma._native, mb._native
    for name in ("params", "exp_avg", "exp_avg_sq", "running"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert torch.equal(a.shadow, b.shadow)


@pytest.mark.parametrize("dtype,rows", [("bf16", 4096), ("f32", 1024)])
@pytest.mark.parametrize("rb", [1, 4])
def test_bn_apply_slabs_match_default(dtype, rows, rb):
    """The BN-backward apply kernel with 1 / 4 row slabs per block (knob 13,
    read at every launch: the column partials are merged once per block)
    gives the default two-slab kernel's bits: parameters, Adam moments, BN statistics
    and losses.  bf16 at 4096 rows (fold forward, apply backward) and fp32 at
    1024 rows (apply both ways)."""
    import types
    from icra2021_multimodal_ad_amd.model_builder import get_model
    ms = []
    for _ in range(2):
        cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype=dtype,
                                    models="ae")
        torch.manual_seed(8)
        ms.append(get_model(cfg))
    ms[1].load_state_dict(ms[0].state_dict())
    for m in ms:
        m._native.sync_shadow(force=True)
    for s in range(2):
        x = torch.from_numpy(synth_windows(rows, 2048, seed=60 + s)).cuda()
        la = float(ms[0]._native.train_step_fused(x))
        with _native.tune(bn_apply_rb=rb):
            lb = float(ms[1]._native.train_step_fused(x))
            torch.cuda.synchronize()
        assert la == lb, (s, la, lb)
    torch.cuda.synchronize()
    a, b = ms[0]._native, ms[1]._native
    for name in ("params", "exp_avg", "exp_avg_sq", "running"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
