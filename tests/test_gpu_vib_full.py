"""BASELINE C3 at its own size: the VIB-AE (encoder -> mu|logvar -> k-sample
reparameterisation -> decoder, sum-MSE/k + beta*KL) at D=2048 and the
reference's exact 4-modal width D=1728, 4096 windows, k=1, through the HIP
path (C-ABI executor) against the CPU oracle with the same injected noise.

Tolerances (north star, fp32): loss, reconstruction and KL terms rtol 1e-4
against the float64 oracle ('truth').  Gradients: this ten-layer BatchNorm
stack at 4096 windows is ill-conditioned -- both CPU fp32 implementations
(the numpy oracle and the reference's own torch-CPU modules) already sit
~1e-3 (relative Frobenius) from the float64 truth on most tensors -- so
each gradient tensor's relative Frobenius error must stay within 5x the
worse of the two CPU fp32 errors (or 1e-4), and the errors summed over all
tensors within 3x the summed CPU fp32 band.  Every number is printed.
bf16 at full size: finite, bit-deterministic, padding stays zero, and within
the bf16 band of the fp32 run (loss 2 %, gradient cosine > 0.99)."""
import types

import numpy as np
import pytest
import torch

from oracle import ae_oracle as O
from oracle.model_io import model_from_state_dict, grads_to_flat
from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd.common_utils import init_state_dict
from icra2021_multimodal_ad_amd.data import synth_windows

pytestmark = pytest.mark.gpu

B, K_SAMPLES, BETA = 4096, 1, 1.0


def _model(d, sd, dtype):
    from icra2021_multimodal_ad_amd.model_builder import get_model
    cfg = types.SimpleNamespace(input_size=d, btl_size=100, n_layers=5, gpu_id=0, dtype=dtype,
                                models="vib_ae", vib_k=K_SAMPLES, beta_kl=BETA)
    m = get_model(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m


def _grads(m):
    nat = m._native
    out = {}
    layers = [("encoder", i, l) for i, l in enumerate(m.encoder.layer_list)] + \
             [("decoder", i, l) for i, l in enumerate(m.decoder.layer_list)]
    for li, (side, i, layer) in enumerate(layers):
        w, b, g, be = nat.param_views(nat.grads, li)
        p = f"{side}.net.{i}."
        out[p + "layer.weight"] = w.cpu().numpy()
        out[p + "layer.bias"] = b.cpu().numpy()
        if layer.bn is not None:
            out[p + "bn.weight"] = g.cpu().numpy()
            out[p + "bn.bias"] = be.cpu().numpy()
    return out


def _oracle(x, sd, eps, prec):
    O.set_precision(prec)
    try:
        m = model_from_state_dict({k: (np.asarray(v, prec) if np.asarray(v).dtype == np.float32 else v)
                                   for k, v in sd.items()})
        loss, g, aux = O.vib_ae_train_grads(x.astype(prec), m, eps.astype(prec), BETA)
    finally:
        O.set_precision(np.float32)
    return loss, grads_to_flat(g), aux


def _torch_cpu_grads(x, sd, eps):
    """The reference's own CPU fp32 path (stock torch modules, oracle/torch_ref.py)
    with the same injected noise: a second fp32 yardstick next to oracle32."""
    from oracle import torch_ref

    def widths(side):
        shp = sorted((int(k.split(".")[2]), np.asarray(v).shape) for k, v in sd.items()
                     if k.startswith(side + ".net.") and k.endswith("layer.weight"))
        return [shp[0][1][1]] + [s[0] for _, s in shp]
    m = torch_ref.build(sd, widths("encoder"), widths("decoder"), vib=True, k=K_SAMPLES, beta_kl=BETA)
    m.train()
    loss = m.vib_loss(torch.from_numpy(x), eps=torch.from_numpy(eps))
    loss.backward()
    return float(loss.detach()), {n: p.grad.double().numpy() for n, p in m.named_parameters()}


@pytest.mark.parametrize("d,bn_mode", [(2048, None), (1728, None), (2048, "2")])
def test_vib_ae_full_size_fp32_matches_oracle(d, bn_mode, monkeypatch):
    """bn_mode "2": train-mode BN fused into the producing GEMMs (the layers
    whose grid is co-resident; the rest fall back to the apply kernels)."""
    sd = init_state_dict(d, 100, 5, seed=40 + d % 7, enc_out=200)
    x = synth_windows(B, d, seed=41)
    eps = np.random.default_rng(42).standard_normal((K_SAMPLES, B, 100)).astype(np.float32)
    with _native.tune(**({"bn_mode": int(bn_mode)} if bn_mode is not None else {})):
        m = _model(d, sd, "f32")
    xd, ed = torch.from_numpy(x).cuda(), torch.from_numpy(eps).cuda()
    # beta 0 first: the reconstruction term alone (same noise, same bits)
    recon = float(m._native.train_step(xd, k=K_SAMPLES, eps=ed, beta_kl=0.0))
    loss = float(m._native.train_step(xd, k=K_SAMPLES, eps=ed, beta_kl=BETA))
    got = _grads(m)
    l32, g32, aux = _oracle(x, sd, eps, np.float32)
    l64, g64, aux64 = _oracle(x, sd, eps, np.float64)
    assert abs(loss - l64) <= 1e-4 * abs(l64), (loss, l64, l32)
    assert abs(recon - aux64["recon"]) <= 1e-4 * aux64["recon"]
    # the KL term on its own (rounding of the fp32 loss sum allowed for)
    kl_got = (loss - recon) / BETA
    tol = 1e-4 * abs(aux64["kl"]) + 4 * float(np.spacing(np.float32(loss)))
    assert aux64["kl"] > 0 and abs(kl_got - aux64["kl"]) <= tol, (kl_got, aux64["kl"])
    lt, gt = _torch_cpu_grads(x, sd, eps)
    assert abs(lt - l64) <= 1e-4 * abs(l64)
    bad = []
    num = band = 0.0

    def errs(g, t):
        g = g.astype(np.float64)
        return (np.abs(g - t).max() / (np.abs(t).max() + 1e-30),
                np.linalg.norm(g - t) / (np.linalg.norm(t) + 1e-30))
    for k, t in g64.items():
        err, fro = errs(got[k], t)
        o_err, o_fro = errs(g32[k], t)
        t_err, t_fro = errs(gt[k], t)
        print(f"{k:36s} max {err:.2e} (oracle32 {o_err:.2e} torch {t_err:.2e})  "
              f"fro {fro:.2e} (oracle32 {o_fro:.2e} torch {t_fro:.2e})")
        ref = max(o_fro, t_fro)
        if not fro < max(1e-4, 5.0 * ref):
            bad.append((k, fro, o_fro, t_fro))
        num += fro
        band += ref
    # over all 36 tensors: the HIP path's summed error within 3x the CPU fp32 band
    print(f"summed fro error {num:.3e}, CPU fp32 band {band:.3e}, ratio {num / band:.2f}")
    assert num <= 3.0 * band, (num, band)
    assert not bad, bad


def test_vib_ae_full_size_bf16_properties():
    d = 2048
    sd = init_state_dict(d, 100, 5, seed=43, enc_out=200)
    x = torch.from_numpy(synth_windows(B, d, seed=44)).cuda()
    eps = torch.from_numpy(np.random.default_rng(45).standard_normal((1, B, 100)).astype(np.float32)).cuda()
    m16 = _model(d, sd, "bf16")
    nat = m16._native
    l1 = nat.train_step(x, k=1, eps=eps, beta_kl=BETA).clone()
    g1 = nat.grads.clone()
    l2 = nat.train_step(x, k=1, eps=eps, beta_kl=BETA).clone()
    assert torch.isfinite(l1).all() and torch.isfinite(g1).all()
    assert torch.equal(l1, l2) and torch.equal(g1, nat.grads)
    # Philox noise: same (seed, offset) -> same bits; another offset -> another draw
    la = nat.train_step(x, k=1, seed=7, offset=3, beta_kl=BETA).clone()
    lb = nat.train_step(x, k=1, seed=7, offset=3, beta_kl=BETA).clone()
    lc = nat.train_step(x, k=1, seed=7, offset=4, beta_kl=BETA).clone()
    assert torch.equal(la, lb) and not torch.equal(la, lc)
    for l, L in enumerate(nat.layers):
        gw = nat.grads[L["w_off"]: L["w_off"] + L["Np"] * L["Kp"]].view(L["Np"], L["Kp"])
        assert float(gw[L["N"]:].abs().sum() + gw[:, L["K"]:].abs().sum()) == 0.0, l
    m32 = _model(d, sd, "f32")
    l32 = float(m32._native.train_step(x, k=1, eps=eps, beta_kl=BETA))
    assert abs(float(l1) - l32) <= 2e-2 * abs(l32)
    cos = torch.nn.functional.cosine_similarity(m32._native.grads, g1, dim=0).item()
    assert cos > 0.99, cos
    # fused bf16 steps (the C3 bench path) keep the loss finite and falling
    losses = [float(m16.train_step_async(x)) for _ in range(6)]
    assert np.isfinite(losses).all() and losses[-1] < losses[0]
    for l, L in enumerate(nat.layers):
        w = nat.params[L["w_off"]: L["w_off"] + L["Np"] * L["Kp"]].view(L["Np"], L["Kp"])
        assert float(w[L["N"]:].abs().sum() + w[:, L["K"]:].abs().sum()) == 0.0, l
