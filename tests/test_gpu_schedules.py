"""Fused-step schedule variants give the same bits as the default schedule.

Streamed Adam on the main-stream tail of the fused step (MMAD_ADAM_STREAM=1:
layers < MMAD_DW_MAIN run a dW GEMM that publishes each fp32 tile through a
per-tile flag, and mmad_adam_stream_kernel applies Adam to the tiles as they
complete, on the tail stream) against the Adam fused into the dW GEMM's
epilogue (MMAD_ADAM_STREAM=0).  The dW accumulation order and the Adam
formula are the same, so parameters, Adam moments, the bf16 weight shadow and
the loss must agree bit for bit, at the C2 and C3 shapes, in bf16 and fp32,
for the plain and the VIB autoencoder, over several steps (flags are reset by
the consumer and reused every step)."""
import pytest
import torch

from icra2021_multimodal_ad_amd.common_utils import init_state_dict
from icra2021_multimodal_ad_amd.data import synth_windows

from tests.test_gpu_parity import _model

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,dtype,models", [(1024, "bf16", "ae"), (4096, "bf16", "vib_ae"),
                                               (256, "f32", "ae"), (1000, "bf16", "ae")])
def test_streamed_adam_matches_fused_epilogue(monkeypatch, rows, dtype, models):
    sd = init_state_dict(2048, 100, 5, seed=21)
    if models == "vib_ae":
        from icra2021_multimodal_ad_amd.model_builder import get_model
        import types
        ms = []
        for st in ("1", "0"):
            monkeypatch.setenv("MMAD_ADAM_STREAM", st)
            cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0,
                                        dtype=dtype, models=models, vib_k=1, beta_kl=1.0)
            torch.manual_seed(3)
            m = get_model(cfg)
            ms.append(m)
        ms[1].load_state_dict(ms[0].state_dict())
    else:
        ms = []
        for st in ("1", "0"):
            monkeypatch.setenv("MMAD_ADAM_STREAM", st)
            m, _ = _model(2048, 100, 5, sd, dtype=dtype)
            ms.append(m)
    for m in ms:
        m._native.sync_shadow(force=True)
    for s in range(3):
        x = torch.from_numpy(synth_windows(rows, 2048, seed=90 + s)).cuda()
        eps = torch.randn(rows, 100, device="cuda") if models == "vib_ae" else None
        la, lb = (float(m._native.train_step_fused(x, eps=eps)) for m in ms)
        assert la == lb, (s, la, lb)
    for m in ms:
        m._native.check_status()
    a, b = ms[0]._native, ms[1]._native
    for name in ("params", "exp_avg", "exp_avg_sq", "running"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    if dtype == "bf16":
        assert torch.equal(a.shadow, b.shadow)


@pytest.mark.parametrize("rows,dtype,models", [(1024, "bf16", "ae"), (4096, "bf16", "vib_ae"),
                                               (256, "f32", "ae")])
def test_tail_pair_launch_matches_two_launches(monkeypatch, rows, dtype, models):
    """The main-stream tail's two Adam-fused dW GEMMs as one launch
    (mmad_gemm_pair_kernel, MMAD_DW_PAIR=1) against two launches
    (MMAD_DW_PAIR=0): each problem keeps its own tile order and partial-sum
    orders, so everything must agree bit for bit over several steps."""
    import types
    from icra2021_multimodal_ad_amd.model_builder import get_model
    ms = []
    for pair in ("1", "0"):
        monkeypatch.setenv("MMAD_DW_PAIR", pair)
        cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype=dtype,
                                    models=models, vib_k=1, beta_kl=1.0)
        torch.manual_seed(4)
        ms.append(get_model(cfg))
    ms[1].load_state_dict(ms[0].state_dict())
    for m in ms:
        m._native.sync_shadow(force=True)
    for s in range(3):
        x = torch.from_numpy(synth_windows(rows, 2048, seed=70 + s)).cuda()
        eps = torch.randn(rows, 100, device="cuda") if models == "vib_ae" else None
        la, lb = (float(m._native.train_step_fused(x, eps=eps)) for m in ms)
        assert la == lb, (s, la, lb)
    for m in ms:
        m._native.check_status()
    a, b = ms[0]._native, ms[1]._native
    for name in ("params", "exp_avg", "exp_avg_sq", "running"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    if dtype == "bf16":
        assert torch.equal(a.shadow, b.shadow)


@pytest.mark.parametrize("env", [
    {"MMAD_EV_EVERY": "1"}, {"MMAD_EV_EVERY": "3"}, {"MMAD_LOSS_SIDE": "0"},
    {"MMAD_DW_MAIN": "1"}, {"MMAD_DW_MAIN": "3"}, {"MMAD_SHADOW_PAIR_ROWS": "0"},
    {"MMAD_SHADOW_PAIR_ROWS": "0", "MMAD_DW_MAIN_PING": "0"}, {"MMAD_SHADOW_PAIR": "0"},
    {"MMAD_SIDE_PRIO": "1"}, {"MMAD_DW_TAIL": "1"}])
def test_schedule_knobs_match_default(monkeypatch, env):
    """Every schedule knob of the fused step only reorders independent work
    across streams (event coalescing, where the loss is reduced, how many dW
    GEMMs run on the main stream, ping-pong shadows, stream priority, the tail
    stream): parameters, Adam moments, BN statistics, the current bf16 shadow
    and the losses equal the default schedule's bit for bit."""
    import types
    from icra2021_multimodal_ad_amd.model_builder import get_model
    ms = []
    for variant in (True, False):
        for k in env:
            monkeypatch.delenv(k, raising=False)
        if variant:
            for k, v in env.items():
                monkeypatch.setenv(k, v)
        cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16",
                                    models="ae")
        torch.manual_seed(8)
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
