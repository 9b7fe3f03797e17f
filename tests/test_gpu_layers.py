"""GPU: the plugin surface below the AutoEncoder is differentiable on the HIP
path -- FCLayer (layers/fc_layer.py:23-48) for every element-wise activation
of modules/activation.py:20-45, with and without BatchNorm, and the
variational_info_bottleneck reparameterisation
(decorators/variational_info_bottleneck.py:19-42).

Numerics tests compare against a plain PyTorch fp32 reference of the same op
(torch on the GPU: nn.Linear -> activation -> nn.BatchNorm1d, as the
reference's modules) and, for the VIB encoder, against the CPU oracle:
forward and all gradients within 1e-4 of their max magnitude (fp32)."""
import types

import numpy as np
import pytest
import torch
from torch import nn

from oracle import ae_oracle as O
from oracle.model_io import model_from_state_dict, grads_to_flat
from icra2021_multimodal_ad_amd.common_utils import init_state_dict
from icra2021_multimodal_ad_amd.data import synth_windows

pytestmark = pytest.mark.gpu


def _rel(a, r):
    a = torch.as_tensor(a).double().cpu()
    r = torch.as_tensor(r).double().cpu()
    return float((a - r).abs().max() / (r.abs().max() + 1e-30))


def _torch_ref(layer):
    lin = nn.Linear(layer.layer.in_features, layer.layer.out_features).cuda()
    act = {"leakyrelu": nn.LeakyReLU(0.2), "relu": nn.ReLU(), "sigmoid": nn.Sigmoid(),
           "tanh": nn.Tanh(), None: nn.Identity()}[layer.act_name]
    bn = nn.BatchNorm1d(layer.layer.out_features).cuda() if layer.bn is not None else None
    with torch.no_grad():
        lin.weight.copy_(layer.layer.weight)
        lin.bias.copy_(layer.layer.bias)
        if bn is not None:
            bn.weight.copy_(layer.bn.weight)
            bn.bias.copy_(layer.bn.bias)
    return lin, act, bn


@pytest.mark.parametrize("act", ["leakyrelu", "relu", "sigmoid", "tanh", None])
@pytest.mark.parametrize("bn", [True, False])
def test_fc_layer_forward_backward_matches_torch(act, bn):
    from icra2021_multimodal_ad_amd.fc_module import FCLayer
    torch.manual_seed(3)
    layer = FCLayer(300, 170, act=act, bn=bn).cuda()
    with torch.no_grad():
        if bn:
            layer.bn.weight.uniform_(0.5, 1.5)
            layer.bn.bias.uniform_(-0.2, 0.2)
    lin, a, bnr = _torch_ref(layer)
    x = torch.randn(200, 300, device="cuda", requires_grad=True)
    xr = x.detach().clone().requires_grad_(True)
    layer.train()
    y = layer(x)
    h = a(lin(xr))
    yr = bnr(h) if bnr is not None else h
    assert y.grad_fn is not None
    assert _rel(y.detach(), yr.detach()) < 1e-5
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    assert _rel(x.grad, xr.grad) < 1e-4
    assert _rel(layer.layer.weight.grad, lin.weight.grad) < 1e-4
    if bn and act is None:
        # Linear -> BN: the batch mean removes the bias, its gradient is 0 up
        # to rounding in both implementations
        gw = float(lin.weight.grad.abs().max())
        assert float(layer.layer.bias.grad.abs().max()) < 1e-4 * gw
        assert float(lin.bias.grad.abs().max()) < 1e-4 * gw
    else:
        assert _rel(layer.layer.bias.grad, lin.bias.grad) < 1e-4
    if bn:
        assert _rel(layer.bn.weight.grad, bnr.weight.grad) < 1e-4
        assert _rel(layer.bn.bias.grad, bnr.bias.grad) < 1e-4
        assert _rel(layer.bn.running_var, bnr.running_var) < 1e-5
        assert int(layer.bn.num_batches_tracked) == 1
    # eval forward; a second call reuses the packed weights until they change
    layer.eval()
    bnr.eval() if bnr is not None else None
    with torch.no_grad():
        ye = layer(x)
        he = a(lin(x))
        assert _rel(ye, bnr(he) if bnr is not None else he) < 1e-5
        key = layer._pack[0]
        layer(x)
        assert layer._pack[0] == key
        layer.layer.weight.mul_(1.0)
        layer(x)
        assert layer._pack[0] != key


def test_encoder_vib_decorator_backward_matches_oracle():
    """Backprop through model.encoder(x, distribution='normal', k=2) -- the
    reference's decorator path -- against the oracle's VIB backward."""
    from icra2021_multimodal_ad_amd.model_builder import get_model
    d, btl, nl, B, k = 192, 16, 5, 64, 2
    sd = init_state_dict(d, btl, nl, seed=91, enc_out=2 * btl)
    cfg = types.SimpleNamespace(input_size=d, btl_size=btl, n_layers=nl, gpu_id=0, dtype="f32",
                                models="vib_ae", vib_k=k)
    m = get_model(cfg)
    m.load_state_dict({kk: torch.from_numpy(np.asarray(v)) for kk, v in sd.items()})
    m.train()
    x = synth_windows(B, d, seed=92)
    rng = np.random.default_rng(93)
    eps = rng.standard_normal((k, B, btl)).astype(np.float32)
    R = rng.standard_normal((k, B, btl)).astype(np.float32)
    R2 = rng.standard_normal((B, btl)).astype(np.float32)
    R3 = rng.standard_normal((B, btl)).astype(np.float32)
    out = m.encoder(torch.from_numpy(x).cuda(), distribution="normal", k=k,
                    eps=torch.from_numpy(eps).cuda())
    loss = (out["z"] * torch.from_numpy(R).cuda()).sum() + (out["mu"] * torch.from_numpy(R2).cuda()).sum() \
        + (out["logvar"] * torch.from_numpy(R3).cuda()).sum()
    m.zero_grad()
    loss.backward()
    # oracle
    om = model_from_state_dict(sd)
    enc_out, caches = O.module_forward(x, om["enc"], train=True)
    mu, lv = O.vib_split(enc_out)
    z = O.vib_reparam(mu, lv, eps)
    assert _rel(out["z"].detach(), z) < 1e-5
    sigma = np.exp(np.float32(0.5) * lv)
    dmu = R.sum(0) + R2
    dlv = (R * eps).sum(0) * sigma * np.float32(0.5) + R3
    _, ge = O.module_backward(np.concatenate([dmu, dlv], axis=-1).astype(np.float32), om["enc"], caches)
    ref = grads_to_flat({"enc": ge, "dec": []})
    got = {n: p.grad for n, p in m.named_parameters() if n.startswith("encoder.")}
    for n, r in ref.items():
        assert _rel(got[n], r) < 1e-4, n
    for i, layer in enumerate(m.encoder.layer_list[:-1]):
        assert _rel(layer.bn.running_mean, om["enc"][i]["bn"]["rm"]) < 1e-5


def test_vib_autoencoder_forward_is_differentiable():
    """AutoEncoder.forward of the VIB-AE keeps the autograd graph (k=1:
    dec(z)), so a caller's own loss trains it."""
    from icra2021_multimodal_ad_amd.model_builder import get_model
    cfg = types.SimpleNamespace(input_size=192, btl_size=16, n_layers=5, gpu_id=0, dtype="f32",
                                models="vib_ae", vib_k=1)
    m = get_model(cfg)
    m.train()
    x = torch.from_numpy(synth_windows(64, 192, seed=94)).cuda()
    y = m(x)
    assert y.shape == x.shape and y.grad_fn is not None
    ((y - x) ** 2).sum().backward()
    grads = [p.grad for p in m.parameters()]
    assert all(g is not None and torch.isfinite(g).all() for g in grads)
    assert any(float(g.abs().sum()) > 0 for g in grads[:4])


@pytest.mark.parametrize("act", ["sigmoid", "logsigmoid", "softmax", "logsoftmax", "tanh", "relu",
                                 "leakyrelu", None])
@pytest.mark.parametrize("shape", [(37, 129), (5, 3, 1000), (1, 1)])
def test_standalone_activation_matches_torch(act, shape):
    """modules/activation.py:20-45 standalone (softmax / logsoftmax over dim=-1):
    the native forward and backward against torch's modules, fp32, 1e-6."""
    from icra2021_multimodal_ad_amd.fc_module import Activation
    ref = {"sigmoid": torch.nn.Sigmoid(), "logsigmoid": torch.nn.LogSigmoid(),
           "softmax": torch.nn.Softmax(dim=-1), "logsoftmax": torch.nn.LogSoftmax(dim=-1),
           "tanh": torch.nn.Tanh(), "relu": torch.nn.ReLU(), "leakyrelu": torch.nn.LeakyReLU(0.2),
           None: torch.nn.Identity()}[act]
    g = torch.Generator().manual_seed(hash((act, shape)) & 0xffff)
    x = (torch.randn(*shape, generator=g) * 4.0).cuda().requires_grad_(True)
    gy = torch.randn(*shape, generator=g).cuda()
    y = Activation(act)(x)
    y.backward(gy)
    xr = x.detach().clone().requires_grad_(True)
    yr = ref(xr)
    yr.backward(gy)
    assert torch.allclose(y, yr, rtol=1e-5, atol=1e-6)
    assert torch.allclose(x.grad, xr.grad, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("reduction,shape", [("sum", (1000, 1728)), ("mean", (37, 5)), ("sum", (3,))])
def test_standalone_mse_loss_matches_torch(reduction, shape):
    """fc_module.Loss('mse', reduction) on its own (modules/loss.py:47-52)
    runs the native mmad_mse_loss / mmad_mse_grad: loss within 1e-5 relative
    of torch's MSELoss, both input gradients within 1e-6 (fp32), deterministic
    (same bits twice); odd sizes take the scalar tail."""
    from icra2021_multimodal_ad_amd.fc_module import Loss
    g = torch.Generator().manual_seed(5)
    a = torch.randn(shape, generator=g).cuda().requires_grad_()
    b = torch.randn(shape, generator=g).cuda().requires_grad_()
    crit = Loss("mse", reduction=reduction)
    out = crit(a, b)
    ref_a, ref_b = a.detach().cpu().double().requires_grad_(), b.detach().cpu().double().requires_grad_()
    ref = torch.nn.MSELoss(reduction=reduction)(ref_a, ref_b)
    assert abs(float(out) - float(ref)) <= 1e-5 * abs(float(ref))
    assert torch.equal(out, crit(a, b))
    (out * 3.0).backward()
    (ref * 3.0).backward()
    for got, want in ((a.grad, ref_a.grad), (b.grad, ref_b.grad)):
        assert torch.allclose(got.cpu().double(), want, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("betas,step,lr", [((0.9, 0.999), 1, 1e-3), ((0.9, 0.999), 3, 1e-3),
                                           ((0.8, 0.95), 2, 3e-4)])
def test_public_adam_matches_torch_cpu_adam(betas, step, lr):
    """The public flat optimizer entry mmad_adam (include/mmad.h; the
    reference's optim.Adam step, novelty_detection.py:90) on an odd-length
    buffer with a bf16 shadow: m / v equal torch.optim.Adam's CPU
    single-tensor step from the same state bit for bit, p to the rounding of
    the update (see below), all within 1e-6 of a float64 evaluation of the
    same formulas, and the shadow is bf16(p)."""
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr
    n = 4099
    g_ = torch.Generator().manual_seed(step)
    p0 = torch.randn(n, generator=g_) * 0.05
    g = torch.randn(n, generator=g_) * 1e-2
    m0 = torch.randn(n, generator=g_) * 1e-3 if step > 1 else torch.zeros(n)
    v0 = torch.rand(n, generator=g_) * 1e-5 if step > 1 else torch.zeros(n)
    # torch CPU, foreach=False (_single_tensor_adam), state after step - 1 steps
    prm = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([prm], lr=lr, betas=betas, eps=1e-8, foreach=False)
    opt.state[prm] = {"step": torch.tensor(float(step - 1)), "exp_avg": m0.clone(),
                      "exp_avg_sq": v0.clone()}
    prm.grad = g.clone()
    opt.step()
    st = opt.state[prm]
    # the product: step size / bias correction as the executor forms them
    b1, b2 = betas
    step_size = lr / (1.0 - b1 ** step)
    bc2_sqrt = (1.0 - b2 ** step) ** 0.5
    dp, dg, dm, dv = (t.clone().cuda() for t in (p0, g, m0, v0))
    shadow = torch.zeros(n, device="cuda", dtype=torch.bfloat16)
    call("mmad_adam", n, ptr(dp), ptr(dg), ptr(dm), ptr(dv), b1, b2, 1e-8, step_size, bc2_sqrt,
         ptr(shadow), n, stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dm.cpu(), st["exp_avg"])
    assert torch.equal(dv.cpu(), st["exp_avg_sq"])
    # p: the same formula and order, but torch's CPU sqrt / scalar division
    # depend on the host's SIMD path (the GPU box's torch CPU matches a
    # correctly rounded evaluation on 98.6 % of the elements at step 1, this
    # container's on 99.9 %) and torch's own GPU single-tensor / foreach steps
    # differ from its CPU step by up to 2.9 ulp of max(|p0|, |p|)
    # (tools/adam_probe.py, profiles/r10/r10f_adam_probe.txt): within 4 such ulp
    pg, pt = dp.cpu().double(), prm.detach().double()
    scale = torch.maximum(p0.double().abs(), pt.abs())
    assert bool(((pg - pt).abs() <= scale * 2.0 ** -21).all())
    assert float((pg == pt).double().mean()) >= 0.95
    assert torch.equal(shadow, dp.bfloat16())
    # float64 evaluation of the same update
    pd, gd, md, vd = (t.double() for t in (p0, g, m0, v0))
    md = b1 * md + (1 - b1) * gd
    vd = b2 * vd + (1 - b2) * gd * gd
    pd = pd - step_size * md / (vd.sqrt() / bc2_sqrt + 1e-8)
    assert float((dp.cpu().double() - pd).abs().max()) <= 1e-6 * float(pd.abs().max())
    assert float((dm.cpu().double() - md).abs().max()) <= 1e-6 * float(md.abs().max())
