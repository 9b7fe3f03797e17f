"""The warp-specialised persistent dW + Adam kernel (mmad_dw_adam_ws_kernel,
tuning knob 12) against the plain Adam-fused dW GEMM: bit-identical
parameters, Adam moments, bf16 shadow and (when materialised) dW, for the
layer operator (mmad_fc_bwd_weight_adam) at bench shapes and for whole fused
train steps in every BN schedule (fold: the BN-producer fix-up in its MMA
epilogue; fused / apply: plain), several steps, several grid caps."""
import pytest
import torch

from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad, BF16
from icra2021_multimodal_ad_amd.common_utils import init_state_dict
from icra2021_multimodal_ad_amd.data import synth_windows

from tests.test_gpu_parity import _model

pytestmark = pytest.mark.gpu


def _dw_adam(ws, M, N, K, blocks=256):
    lib = _native.load()
    dev = torch.device("cuda", 0)
    Mp, Np, Kp = pad(M), pad(N), pad(K)
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    dz = torch.zeros(Mp, Np, device=dev, dtype=torch.bfloat16)
    dz[:M, :N] = torch.randn(M, N, device=dev, generator=g).bfloat16()
    x = torch.zeros(Mp, Kp, device=dev, dtype=torch.bfloat16)
    x[:M, :K] = torch.randn(M, K, device=dev, generator=g).bfloat16()
    p = torch.zeros(Np, Kp, device=dev)
    p[:N, :K] = torch.randn(N, K, device=dev, generator=g) * 0.02
    m = torch.zeros_like(p)
    m[:N, :K] = torch.randn(N, K, device=dev, generator=g) * 1e-3
    v = torch.zeros_like(p)
    v[:N, :K] = torch.rand(N, K, device=dev, generator=g) * 1e-5
    sh = torch.zeros(Np, Kp, device=dev, dtype=torch.bfloat16)
    lib.mmad_tune_set(12, 1 if ws else 0)
    lib.mmad_tune_set(13, blocks)
    try:
        call("mmad_fc_bwd_weight_adam", BF16, Mp, Np, Kp, ptr(dz), ptr(x), ptr(p), ptr(m), ptr(v),
             ptr(sh), None, 0.9, 0.999, 1e-8, 1e-3, 0.97, stream_ptr())
        torch.cuda.synchronize()
    finally:
        lib.mmad_tune_set(12, 0)
        lib.mmad_tune_set(13, 256)
    return p, m, v, sh


@pytest.mark.parametrize("shape", [(1024, 1658, 2048), (1024, 489, 879), (4096, 1268, 1658),
                                   (640, 200, 489)])
@pytest.mark.parametrize("blocks", [256, 64])
def test_ws_kernel_bit_identical_layer_op(shape, blocks):
    a = _dw_adam(False, *shape)
    b = _dw_adam(True, *shape, blocks=blocks)
    for x, y, name in zip(a, b, ("p", "m", "v", "shadow")):
        assert torch.equal(x, y), name


@pytest.mark.parametrize("bn_mode", ["2", "1", "0"])
def test_ws_kernel_bit_identical_train_steps(bn_mode, monkeypatch):
    monkeypatch.setenv("MMAD_BN_MODE", bn_mode)
    lib = _native.load()
    sd = init_state_dict(2048, 100, 5, seed=21)
    outs = []
    try:
        for ws in (0, 1):
            lib.mmad_tune_set(12, ws)
            mdl, _ = _model(2048, 100, 5, sd, dtype="bf16")
            nat = mdl._native
            nat.sync_shadow(force=True)
            for s in range(3):
                x = torch.from_numpy(synth_windows(1024, 2048, seed=80 + s)).cuda()
                loss = nat.train_step_fused(x)
            nat.check_status()
            torch.cuda.synchronize()
            outs.append((float(loss), nat.params.clone(), nat.exp_avg.clone(), nat.exp_avg_sq.clone(),
                         nat.shadow.clone(), nat.running.clone()))
    finally:
        lib.mmad_tune_set(12, 0)
    a, b = outs
    assert a[0] == b[0]
    for x, y in zip(a[1:], b[1:]):
        assert torch.equal(x, y)
