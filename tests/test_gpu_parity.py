"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle and the
reference's golden vectors.  Tolerances (north star): fp32 path -- loss and
per-window scores within rtol 1e-4; gradients within 1e-4 of their max
magnitude.  bf16 path -- loss within 2 %, gradient cosine > 0.99, per-window
scores within 5 %, AUROC within 0.01 of the fp32 value."""
import types

import numpy as np
import pytest
import torch

from oracle import ae_oracle as O
from oracle.model_io import model_from_state_dict, grads_to_flat
from icra2021_multimodal_ad_amd.common_utils import init_state_dict
from icra2021_multimodal_ad_amd.data import synth_windows

pytestmark = pytest.mark.gpu

CASES = ["c1_ft64", "mm192"]


def _sd(g, prefix):
    return {k[len(prefix):]: g[k] for k in g.files if k.startswith(prefix)}


def _rel(a, r):
    a = np.asarray(a, np.float64)
    return float(np.abs(a - r).max() / (np.abs(r).max() + 1e-30))


def _model(d, btl, nl, sd, dtype="f32", models="ae", k=1, beta_kl=1.0):
    from icra2021_multimodal_ad_amd.model_builder import get_model
    cfg = types.SimpleNamespace(input_size=d, btl_size=btl, n_layers=nl, gpu_id=0, dtype=dtype,
                                models=models, vib_k=k, beta_kl=beta_kl)
    m = get_model(cfg)
    m.load_state_dict({k_: torch.from_numpy(np.asarray(v)) for k_, v in sd.items()})
    return m, cfg


_TRUTH = {}


def _truth_grads(g, name):
    """float64 oracle gradients ('truth') for a golden case."""
    if name not in _TRUTH:
        sd = _sd(g, "init/")
        O.set_precision(np.float64)
        try:
            m = model_from_state_dict({k: (np.asarray(v, np.float64) if np.asarray(v).dtype == np.float32
                                           else v) for k, v in sd.items()})
            _, _, gr = O.ae_train_grads(g["x/0"].astype(np.float64), m)
        finally:
            O.set_precision(np.float32)
        _TRUTH[name] = grads_to_flat(gr)
    return _TRUTH[name]


def assert_grads_close(got, g, name):
    """fp32 bar: within 1e-4 of max|g| of the fp64 truth, or within 2x the
    reference's own fp32 deviation from that truth (near-cancelling BN-layer
    bias gradients are summation-order noise in the reference too)."""
    truth = _truth_grads(g, name)
    for k, t in truth.items():
        ref = g["step1/grad/" + k]
        scale = np.abs(t).max() + 1e-30
        ref_err = np.abs(ref - t).max() / scale
        err = np.abs(np.asarray(got[k], np.float64) - t).max() / scale
        assert err < max(1e-4, 2.0 * ref_err), (k, err, ref_err)


def _grads_flat(model):
    nat = model._native
    out = {}
    names = []
    for side, mod in (("encoder", model.encoder), ("decoder", model.decoder)):
        for i, layer in enumerate(mod.layer_list):
            names.append((f"{side}.net.{i}.", layer.bn is not None))
    for l, (p, has_bn) in enumerate(names):
        w, b, g, be = nat.param_views(nat.grads, l)
        out[p + "layer.weight"] = w.cpu().numpy()
        out[p + "layer.bias"] = b.cpu().numpy()
        if has_bn:
            out[p + "bn.weight"] = g.cpu().numpy()
            out[p + "bn.bias"] = be.cpu().numpy()
    return out


@pytest.mark.parametrize("name", CASES)
def test_train_step_fp32_matches_reference(golden, name):
    g = golden(name)
    d, btl, nl = int(g["meta_d"]), int(g["meta_btl"]), int(g["meta_n_layers"])
    m, _ = _model(d, btl, nl, _sd(g, "init/"))
    x = torch.from_numpy(g["x/0"]).cuda()
    loss = float(m._native.train_step(x))
    assert abs(loss - g["step1/loss"]) <= 1e-4 * g["step1/loss"]
    assert_grads_close(_grads_flat(m), g, name)
    sd = m.state_dict()
    for k in sd:
        if "running" in k:
            assert _rel(sd[k].cpu().numpy(), g["after0/" + k]) < 1e-4, k


@pytest.mark.parametrize("name", CASES)
def test_native_adam_matches_reference(golden, name):
    g = golden(name)
    d, btl, nl = int(g["meta_d"]), int(g["meta_btl"]), int(g["meta_n_layers"])
    m, _ = _model(d, btl, nl, _sd(g, "init/"))
    nat = m._native
    # inject the reference's own step-1 gradients, then one native Adam step
    for l, layer in enumerate(list(m.encoder.layer_list) + list(m.decoder.layer_list)):
        side = "encoder" if l < len(m.encoder.layer_list) else "decoder"
        i = l if side == "encoder" else l - len(m.encoder.layer_list)
        p = f"step1/grad/{side}.net.{i}."
        w, b, gg, be = nat.param_views(nat.grads, l)
        w.copy_(torch.from_numpy(g[p + "layer.weight"]))
        b.copy_(torch.from_numpy(g[p + "layer.bias"]))
        if layer.bn is not None:
            gg.copy_(torch.from_numpy(g[p + "bn.weight"]))
            be.copy_(torch.from_numpy(g[p + "bn.bias"]))
    nat.adam(lr=1e-3)
    sd = m.state_dict()
    for k, v in sd.items():
        if "running" in k or "num_batches" in k:
            continue
        assert np.abs(v.cpu().numpy().astype(np.float64) - g["after0/" + k]).max() < 1e-6, k


@pytest.mark.parametrize("name", CASES)
def test_reference_step_api_and_trajectory(golden, name):
    """AutoEncoder.step with a torch Adam optimizer (novelty_detection.py:90):
    step-1 loss exact, later steps within the sign(g) amplification band."""
    g = golden(name)
    d, btl, nl = int(g["meta_d"]), int(g["meta_btl"]), int(g["meta_n_layers"])
    m, cfg = _model(d, btl, nl, _sd(g, "init/"))
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    eng = types.SimpleNamespace(model=m, optimizer=opt, config=cfg)
    B = int(g["meta_batch"])
    losses = [m.step(eng, (torch.from_numpy(g[f"x/{s}"]), torch.zeros(B)))[0] for s in range(3)]
    assert abs(losses[0] - g["loss/0"]) <= 1e-4 * g["loss/0"]
    assert abs(losses[1] - g["loss/1"]) <= 5e-3 * g["loss/1"]
    assert abs(losses[2] - g["loss/2"]) <= 2e-2 * g["loss/2"]
    st = opt.state_dict()["state"]
    assert len(st) == len(list(m.parameters()))
    assert int(m.state_dict()["encoder.net.0.bn.num_batches_tracked"]) == 3


@pytest.mark.parametrize("name", CASES)
def test_eval_forward_validate_and_scores(golden, name):
    g = golden(name)
    d, btl, nl = int(g["meta_d"]), int(g["meta_btl"]), int(g["meta_n_layers"])
    steps = int(g["meta_steps"])
    m, cfg = _model(d, btl, nl, _sd(g, f"after{steps - 1}/"))
    m.eval()
    with torch.no_grad():
        xh = m(torch.from_numpy(g["x/0"]).cuda()).detach().cpu().numpy()
    assert _rel(xh, g["eval/x_hat"]) < 1e-4
    eng = types.SimpleNamespace(model=m, optimizer=None, config=cfg)
    (vl,) = m.validate(eng, (torch.from_numpy(g["x/0"]), None))
    assert abs(vl - g["eval/loss"]) <= 1e-4 * g["eval/loss"]
    from icra2021_multimodal_ad_amd.reconstruction_aggregation import (
        get_diffs, score_windows, base_from_layer_sq, sap_from_layer_sq)
    diffs = get_diffs(g["score/test_x"], m)
    for i, dd in enumerate(diffs):
        ref = g[f"score/test_diff{i}"]
        assert dd.shape == ref.shape
        assert np.abs(dd - ref).max() <= 1e-4 * max(1.0, np.abs(ref).max()), i
    lsq = score_windows(torch.from_numpy(g["score/test_x"]), m, batch_size=256).cpu().numpy()
    widths = m._native.diff_widths()
    base = base_from_layer_sq(lsq, widths)
    sap = sap_from_layer_sq(lsq, widths)
    assert _rel(base, g["score/base"]) < 1e-4
    assert _rel(sap, g["score/sap"]) < 1e-4
    lab = g["score/test_label"]
    assert abs(O.auroc(base, lab) - g["score/base_auroc"]) < 2e-3
    assert abs(O.auroc(sap, lab) - g["score/sap_auroc"]) < 2e-3


def test_fc_layer_standalone_matches_oracle(golden):
    g = golden("mm192")
    from icra2021_multimodal_ad_amd.fc_module import FCLayer
    sd = _sd(g, "after2/")
    om = model_from_state_dict(sd)
    layer = FCLayer(192, om["enc"][0]["W"].shape[0], act="leakyrelu", bn=True).cuda()
    with torch.no_grad():
        layer.layer.weight.copy_(torch.from_numpy(om["enc"][0]["W"]))
        layer.layer.bias.copy_(torch.from_numpy(om["enc"][0]["b"]))
        layer.bn.weight.copy_(torch.from_numpy(om["enc"][0]["bn"]["gamma"]))
        layer.bn.bias.copy_(torch.from_numpy(om["enc"][0]["bn"]["beta"]))
        layer.bn.running_mean.copy_(torch.from_numpy(om["enc"][0]["bn"]["rm"]))
        layer.bn.running_var.copy_(torch.from_numpy(om["enc"][0]["bn"]["rv"]))
    x = g["x/1"]
    layer.eval()
    y = layer(torch.from_numpy(x).cuda()).detach().cpu().numpy()
    ye, _ = O.fc_forward(x, om["enc"][0], train=False)
    assert _rel(y, ye) < 1e-5
    layer.train()
    y = layer(torch.from_numpy(x).cuda()).detach().cpu().numpy()
    yt, _ = O.fc_forward(x, om["enc"][0], train=True)
    assert _rel(y, yt) < 1e-4
    assert _rel(layer.bn.running_var.cpu().numpy(), om["enc"][0]["bn"]["rv"]) < 1e-5


def test_autograd_forward_backward_matches(golden):
    g = golden("mm192")
    m, _ = _model(192, 16, 5, _sd(g, "init/"))
    m.train()
    x = torch.from_numpy(g["x/0"]).cuda()
    loss = m.get_loss_value(x, x)
    assert abs(loss.item() - g["step1/loss"]) <= 1e-4 * g["step1/loss"]
    m.zero_grad()
    loss.backward()
    assert_grads_close({n: p.grad.cpu().numpy() for n, p in m.named_parameters()}, g, "mm192")


def test_d1728_reference_width_fp32(golden):
    g = golden("d1728")
    m, _ = _model(1728, 100, 5, init_state_dict(1728, 100, 5, seed=2))
    loss = float(m._native.train_step(torch.from_numpy(g["x/0"]).cuda()))
    assert abs(loss - g["step1/loss"]) <= 1e-4 * g["step1/loss"]
    for k, v in _grads_flat(m).items():
        v = v.astype(np.float64)
        sq = g["step1/gradsq/" + k]
        assert abs((v ** 2).sum() - sq) <= 1e-3 * sq, k


def test_bf16_train_step_tracks_fp32():
    sd = init_state_dict(2048, 100, 5, seed=4)
    x = torch.from_numpy(synth_windows(1024, 2048, seed=5)).cuda()
    m32, _ = _model(2048, 100, 5, sd, dtype="f32")
    m16, _ = _model(2048, 100, 5, sd, dtype="bf16")
    l32 = float(m32._native.train_step(x))
    l16 = float(m16._native.train_step(x))
    assert abs(l16 - l32) <= 2e-2 * l32
    g32, g16 = m32._native.grads, m16._native.grads
    cos = torch.nn.functional.cosine_similarity(g32, g16, dim=0).item()
    assert cos > 0.99, cos
    # a few bf16 steps reduce the loss
    losses = []
    for s in range(5):
        losses.append(float(m16.train_step_async(x)))
    assert losses[-1] < losses[0]
    assert np.isfinite(losses).all()


def test_vib_train_step_matches_oracle():
    d, btl, nl, B, k, beta = 192, 16, 5, 64, 2, 0.5
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict as isd
    sd = isd(d, btl, nl, seed=21, enc_out=2 * btl)
    m, _ = _model(d, btl, nl, sd, models="vib_ae", k=k, beta_kl=beta)
    x = synth_windows(B, d, seed=22)
    eps = np.random.default_rng(23).standard_normal((k, B, btl)).astype(np.float32)
    loss = float(m._native.train_step(torch.from_numpy(x).cuda(), k=k,
                                      eps=torch.from_numpy(eps).cuda(), beta_kl=beta))
    rl, rg, _ = O.vib_ae_train_grads(x, model_from_state_dict(sd), eps, beta)
    assert abs(loss - rl) <= 1e-4 * abs(rl)
    got = _grads_flat(m)
    for kk, v in grads_to_flat(rg).items():
        assert _rel(got[kk], v) < 1e-4, kk


def test_vib_decorator_reparam(golden):
    g = golden("vib")
    from icra2021_multimodal_ad_amd.fc_module import reparameterize
    mu = torch.from_numpy(g["mu"]).cuda()
    lv = torch.from_numpy(g["logvar"]).cuda()
    z = reparameterize(mu, lv, 3, True, eps=torch.from_numpy(g["eps"]).cuda()).cpu().numpy()
    assert _rel(z, g["z"]) < 1e-5
    with torch.no_grad():
        zd = reparameterize(mu, lv, 2, False).cpu().numpy()
    assert np.array_equal(zd, np.broadcast_to(g["mu"], zd.shape))
    zr = reparameterize(mu, lv, 256, True).cpu().numpy()   # Philox draw
    e = (zr - g["mu"][None]) / np.exp(0.5 * g["logvar"])[None]
    n = e.size                                             # 5-sigma bounds for N(0, 1)
    assert abs(e.mean()) < 5 / np.sqrt(n) and abs(e.std() - 1) < 5 * np.sqrt(0.5 / n)


def test_full_size_properties_bf16():
    """BASELINE C2 shape: D=2048, B=1024 bf16 -- finite loss, deterministic
    (same inputs -> bit-identical loss and grads), padded regions stay zero."""
    sd = init_state_dict(2048, 100, 5, seed=6)
    m, _ = _model(2048, 100, 5, sd, dtype="bf16")
    x = torch.from_numpy(synth_windows(1024, 2048, seed=7)).cuda()
    l1 = m._native.train_step(x).clone()
    g1 = m._native.grads.clone()
    l2 = m._native.train_step(x).clone()
    assert torch.equal(l1, l2)
    assert torch.equal(g1, m._native.grads)
    nat = m._native
    for l, L in enumerate(nat.layers):
        w = nat.params[L["w_off"]: L["w_off"] + L["Np"] * L["Kp"]].view(L["Np"], L["Kp"])
        gw = nat.grads[L["w_off"]: L["w_off"] + L["Np"] * L["Kp"]].view(L["Np"], L["Kp"])
        assert float(w[L["N"]:].abs().sum() + w[:, L["K"]:].abs().sum()) == 0.0
        assert float(gw[L["N"]:].abs().sum() + gw[:, L["K"]:].abs().sum()) == 0.0


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_fused_step_equals_unfused(dtype):
    """mmad_ae_train_step (per-layer Adam on the side stream, overlapped with
    the backward) == train_fwd_bwd followed by one flat Adam."""
    sd = init_state_dict(192, 16, 5, seed=31)
    ma, _ = _model(192, 16, 5, sd, dtype=dtype)
    mb, _ = _model(192, 16, 5, sd, dtype=dtype)
    for s in range(3):
        x = torch.from_numpy(synth_windows(200, 192, seed=40 + s)).cuda()
        la = ma._native.train_step_fused(x)
        lb = mb._native.train_step(x)
        mb._native.adam()
        assert float(la) == float(lb)
    torch.cuda.synchronize()
    nat = ma._native
    for l, L in enumerate(nat.layers):
        for name, off, n in (("W", L["w_off"], L["Np"] * L["Kp"]),
                             ("small", L["b_off"], (3 if L["bn"] else 1) * L["Np"])):
            d = (ma._native.params[off:off + n] - mb._native.params[off:off + n]).abs().max().item()
            assert d <= 1e-6, (l, name, d)
    assert torch.equal(ma._native.running, mb._native.running)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_tile_configs_bit_identical(dtype):
    """Every GEMM tile configuration (forced through the tuning knob) yields
    bit-identical gradients and BN statistics: the K accumulation order and all
    epilogue partial-sum orders are tile-independent, so the autotuner's pick
    can never change a result.  (A forced configuration that does not divide a
    GEMM's output falls back to the tuned one for that GEMM.)"""
    from icra2021_multimodal_ad_amd import _native
    lib = _native.load()
    sd = init_state_dict(500, 40, 3, seed=17)
    x = torch.from_numpy(synth_windows(512, 500, seed=18)).cuda()
    ref = None
    try:
        for cfg in (-1, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9):
            lib.mmad_tune_set(0, cfg)
            m, _ = _model(500, 40, 3, sd, dtype=dtype)
            loss = float(m._native.train_step(x))
            out = (m._native.grads.cpu().numpy(), m._native.running.cpu().numpy(), loss)
            if ref is None:
                ref = out
                continue
            assert np.array_equal(out[0], ref[0]), cfg
            assert np.array_equal(out[1], ref[1]), cfg
            assert abs(out[2] - ref[2]) <= 1e-5 * abs(ref[2]), cfg   # loss partials are per tile
    finally:
        lib.mmad_tune_set(0, -1)


def test_nap_run_native_matches_reference_fit(golden):
    """NAP run through mmad_nap_score (GEMM + standardise/square-mean epilogue)
    with the reference's own fit state: scores within 1e-4 (fp32 path), and the
    on-device fit reproduces the reference's scores on the well-conditioned
    case."""
    from icra2021_multimodal_ad_amd.reconstruction_aggregation import NapScorer
    g = golden("nap")
    W = g["train"].shape[1]
    m, _ = _model(W, 8, 2, init_state_dict(W, 8, 2, seed=5), dtype="f32")
    nap = NapScorer(m)
    nap.sel = slice(0, 1)
    fit = {k: g[k] for k in ("mu_r", "v", "mu_s", "var")}
    nap.fit(fit_state=fit)
    got = nap.score(torch.from_numpy(g["test"])).cpu().numpy()
    assert _rel(got, g["score"]) < 1e-4
    nap2 = NapScorer(m)
    nap2.sel = slice(0, 1)
    nap2.fit(train_diffs=torch.from_numpy(g["train"]))
    got2 = nap2.score(torch.from_numpy(g["test"])).cpu().numpy()
    assert _rel(got2, g["score"]) < 1e-4


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_nap_on_autoencoder_diffs(golden, name, dtype):
    """NAP (utils/metric.py:183-238) on the AE's own get_diffs, with the
    reference's fit state (score/nap_*): the reference's diffs through the
    native NAP run give score/nap to 1e-4 for either model dtype (the NAP GEMM
    is fp32 always); the fp32 model's own GPU diffs do too, with the NAP AUROC
    (The NAP AUROC of these fits is not compared: the synthetic diffs make
    them near-singular, var ~ 1e-12 on some components, so the scores there
    are rounding noise times 1e12 in the reference as much as here -- NAP AUROC
    parity is pinned on a full-rank fit in tests/test_gpu_e2e.py.)"""
    from icra2021_multimodal_ad_amd.reconstruction_aggregation import NapScorer, get_diffs
    g = golden(name)
    d, btl, nl = int(g["meta_d"]), int(g["meta_btl"]), int(g["meta_n_layers"])
    steps = int(g["meta_steps"])
    m, _ = _model(d, btl, nl, _sd(g, f"after{steps - 1}/"), dtype=dtype)
    nap = NapScorer(m).fit(fit_state={k: g["score/nap_" + k] for k in ("mu_r", "v", "mu_s", "var")})
    n_layers = len(m._native.diff_widths())
    ref_diffs = [g[f"score/test_diff{i}"] for i in range(n_layers)]
    got = nap.score(ref_diffs).cpu().numpy()
    assert _rel(got, g["score/nap"]) < 1e-4
    if dtype == "f32":
        own = nap.score(get_diffs(g["score/test_x"], m)).cpu().numpy()
        assert _rel(own, g["score/nap"]) < 1e-4


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_score_stream_graph_matches_per_batch(golden, dtype):
    """mmad_ae_score_stream (BASELINE C5 streaming pass, hipGraph replay) ==
    per-batch mmad_ae_score bit for bit, ragged last batch included; a replay
    after a train step sees the new weights and BN running statistics; fp32
    scores match the reference's golden BASE/SAP."""
    from icra2021_multimodal_ad_amd.reconstruction_aggregation import (
        score_windows, base_from_layer_sq, sap_from_layer_sq)
    g = golden("mm192")
    d, btl, nl = int(g["meta_d"]), int(g["meta_btl"]), int(g["meta_n_layers"])
    steps = int(g["meta_steps"])
    m, _ = _model(d, btl, nl, _sd(g, f"after{steps - 1}/"), dtype=dtype)
    nat = m._native
    x = torch.from_numpy(g["score/test_x"]).cuda()
    n, bs = x.shape[0], 48          # ragged: n is not a multiple of 48

    def per_batch():
        m.eval()
        parts = [nat.score(x[s:s + bs])[0] for s in range(0, n, bs)]
        return torch.cat(parts, dim=1)

    out = torch.full((nat.n_enc + 1, n + 5), float("nan"), device="cuda")
    eager = score_windows(x, m, batch_size=bs, out=out[:, :n], graph=False).clone()
    ref = per_batch()
    assert torch.equal(eager, ref)
    assert nat._lib.mmad_ae_graph_count(nat._h) == 0
    first = score_windows(x, m, batch_size=bs, out=out[:, :n]).clone()   # eager + capture
    assert nat._lib.mmad_ae_graph_count(nat._h) == 1
    out[:, :n].fill_(float("nan"))
    replay = score_windows(x, m, batch_size=bs, out=out[:, :n]).clone()
    assert nat._lib.mmad_ae_graph_count(nat._h) == 1
    assert torch.equal(first, ref) and torch.equal(replay, ref)
    assert torch.isnan(out[:, n:]).all()          # nothing written past N
    if dtype == "f32":
        widths = nat.diff_widths()
        lsq = replay.cpu().numpy()
        assert _rel(base_from_layer_sq(lsq, widths), g["score/base"]) < 1e-4
        assert _rel(sap_from_layer_sq(lsq, widths), g["score/sap"]) < 1e-4
    # train in between: the captured pass reads the updated weights/BN stats
    m.train()
    m.train_step_async(x[:64])
    ref2 = per_batch()
    assert not torch.equal(ref2, ref)
    again = score_windows(x, m, batch_size=bs, out=out[:, :n]).clone()
    assert torch.equal(again, ref2)
    assert nat._lib.mmad_ae_clear_graphs(nat._h) == 0
    assert nat._lib.mmad_ae_graph_count(nat._h) == 0


def test_bf16_shadow_follows_load_state_dict_and_torch_optim():
    """The bf16 weight shadow must follow every write of the fp32 master made
    through the reference-shaped parameters: load_state_dict after native
    steps (best-on-valid restore, novelty_detection.py:125) and a torch
    optimizer step on model.parameters()."""
    sd = init_state_dict(700, 40, 5, seed=61)
    x = torch.from_numpy(synth_windows(256, 700, seed=62)).cuda()
    m, _ = _model(700, 40, 5, sd, dtype="bf16")
    m.eval()
    with torch.no_grad():
        y0 = m(x).clone()
    m.train()
    for _ in range(2):
        m.train_step_async(x)                      # native Adam: shadow updated in place
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    m.eval()
    with torch.no_grad():
        y1 = m(x)
    assert torch.equal(y0, y1)
    fresh, _ = _model(700, 40, 5, sd, dtype="bf16")
    fresh.eval()
    with torch.no_grad():
        assert torch.equal(fresh(x), y1)
    # in-place writes through the parameters (what a torch optimizer does)
    with torch.no_grad():
        for p in m.parameters():
            p.mul_(0.5)
    with torch.no_grad():
        y2 = m(x)
    fresh.load_state_dict(m.state_dict())
    with torch.no_grad():
        assert torch.equal(fresh(x), y2)
    assert not torch.equal(y2, y1)


def test_differentiable_forward_guards_its_saved_activations(golden):
    """model(x1); model(x2); backward of the first must not silently use the
    second forward's activations (one shared native workspace)."""
    g = golden("mm192")
    m, _ = _model(192, 16, 5, _sd(g, "init/"))
    m.train()
    x = torch.from_numpy(g["x/0"]).cuda()
    l1 = m.get_loss_value(x, x)
    l2 = m.get_loss_value(x[:32], x[:32])
    with pytest.raises(RuntimeError, match="another native pass"):
        l1.backward()
    l2.backward()                                   # the latest forward is fine
    with pytest.raises(RuntimeError):
        m.zero_grad()
        l3 = m.get_loss_value(x, x)
        l3.backward(retain_graph=True)
        l3.backward()                               # a second backward reuses consumed state


@pytest.mark.parametrize("dtype,models", [("f32", "ae"), ("bf16", "ae"), ("bf16", "vib_ae")])
def test_graph_step_equals_eager_step(dtype, models, monkeypatch):
    """mmad_ae_train_step_graph (whole step captured once, replayed with the
    per-call values copied in) == the eager mmad_ae_train_step, bit for bit,
    over steps with changing inputs, Adam step counts and VIB noise offsets."""
    from icra2021_multimodal_ad_amd import _native
    d, btl, nl = 700, 40, 5
    enc_out = 2 * btl if models == "vib_ae" else None
    sd = init_state_dict(d, btl, nl, seed=71, enc_out=enc_out)
    xs = [torch.from_numpy(synth_windows(384, d, seed=80 + i)).cuda() for i in range(4)]
    res = {}
    for graph in (False, True):
        m, _ = _model(d, btl, nl, sd, dtype=dtype, models=models)
        m._native.use_graph = graph
        losses = [float(m.train_step_async(xs[i % 4])) for i in range(7)]
        nat = m._native
        res[graph] = (losses, nat.params.clone(), nat.exp_avg.clone(), nat.exp_avg_sq.clone(),
                      nat.running.clone())
        if graph:
            assert nat._lib.mmad_ae_train_graph_count(nat._h) == 1
    for a, b in zip(res[False][1:], res[True][1:]):
        assert torch.equal(a, b)
    assert res[False][0] == res[True][0]


@pytest.mark.parametrize("shape", [(3000, 48), (40, 300), (5000, 700)])
def test_nap_fit_native_matches_reference_and_oracle(golden, shape):
    """mmad_nap_fit (Rotater.fit + Standardizer.fit, utils/normalize.py:25-70)
    against the reference's own fit state on nap.npz (mu_r 1e-6, var rtol 1e-4,
    each V column parallel to the reference's up to sign: |cos| >= 1 - 1e-5 --
    the nap.npz spectrum is well separated), and against the float64 oracle
    (oracle.nap_fit) on seeded data, including N < W (rank-deficient: only the
    N - 1 informative directions are compared; the rest are an arbitrary
    orthonormal completion in either implementation).  Repeat runs are
    bit-identical."""
    from icra2021_multimodal_ad_amd.reconstruction_aggregation import nap_fit
    N, W = shape
    if shape == (3000, 48):
        g = golden("nap")
        x = g["train"]
        ref = {k: g[k] for k in ("mu_r", "v", "mu_s", "var")}
    else:
        rng = np.random.default_rng(N + W)
        x = (rng.standard_normal((N, W)) * np.linspace(3.0, 0.2, W) + 0.5).astype(np.float32)
        ref = O.nap_fit(x)
    got = nap_fit(torch.from_numpy(x).cuda())
    again = nap_fit(torch.from_numpy(x).cuda())
    for k in got:
        assert torch.equal(got[k], again[k]), k
    got = {k: t.cpu().numpy().astype(np.float64) for k, t in got.items()}
    R = min(N, W)
    assert got["v"].shape == (W, R)
    assert np.abs(got["mu_r"] - ref["mu_r"]).max() <= 1e-6 * max(1.0, np.abs(ref["mu_r"]).max())
    keep = R if N > W else N - 1
    v, rv = got["v"][:, :keep], np.asarray(ref["v"], np.float64)[:, :keep]
    cos = np.abs((v * rv).sum(0)) / (np.linalg.norm(v, axis=0) * np.linalg.norm(rv, axis=0))
    assert cos.min() >= 1 - 1e-5, cos.min()
    assert np.abs(got["var"][:keep] - ref["var"][:keep]).max() <= 1e-4 * ref["var"][:keep].max()
    assert np.abs(got["mu_s"][:keep]).max() <= 1e-4 * np.sqrt(ref["var"][:keep].max())
    vtv = got["v"].T @ got["v"]
    assert np.abs(vtv - np.eye(R)).max() < 1e-5
