"""Generate golden vectors by running the REFERENCE implementation on CPU.

Runs only in the build container (it needs /root/reference); the .npz files it
writes are committed and travel instead of the reference.  Usage:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

Shims applied (reference rot listed in SURVEY.md §0): ``collections.Iterable``
for Python>=3.10 (models/abstract_model.py:25); ignite is absent, so
``AutoEncoder.step`` / ``validate`` are driven with a duck-typed engine
(``.model``, ``.optimizer``, ``.config.gpu_id``), exactly the attributes
models/auto_encoder.py:57-91 reads.  Weights come from the build's seeded
``init_state_dict`` and are loaded with ``load_state_dict``; inputs from the
build's seeded synthetic generator.
"""
import collections
import collections.abc
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True
collections.Iterable = collections.abc.Iterable
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(1, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from icra2021_multimodal_ad_amd.common_utils import init_state_dict  # noqa: E402
from icra2021_multimodal_ad_amd.data import synth_windows, synth_split  # noqa: E402

torch.set_num_threads(8)


def ref_model(d, btl, n_layers, seed, enc_out=None):
    from model_builder import get_model
    cfg = types.SimpleNamespace(input_size=d, btl_size=btl, n_layers=n_layers, gpu_id=-1)
    m = get_model(cfg)
    sd = init_state_dict(d, btl, n_layers, seed=seed)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m


def sd_numpy(m, prefix):
    return {prefix + k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}


def grads_numpy(m, prefix):
    return {prefix + k: p.grad.detach().cpu().numpy().copy() for k, p in m.named_parameters()}


def engine_for(m, opt):
    return types.SimpleNamespace(model=m, optimizer=opt, config=types.SimpleNamespace(gpu_id=-1))


def train_case(name, d, btl, n_layers, batch, seed, steps=3, keep_params=True):
    """Fixture: init params, per-step batches, loss/x_hat/grads of step 1,
    running stats + params after each Adam step, eval x_hat after training."""
    from models.auto_encoder import AutoEncoder
    m = ref_model(d, btl, n_layers, seed)
    out = {"meta_d": np.int64(d), "meta_btl": np.int64(btl), "meta_n_layers": np.int64(n_layers),
           "meta_batch": np.int64(batch), "meta_seed": np.int64(seed), "meta_steps": np.int64(steps),
           "meta_torch": np.array(torch.__version__)}
    if keep_params:
        out.update(sd_numpy(m, "init/"))
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    eng = engine_for(m, opt)
    xs = [synth_windows(batch, d, seed=seed * 100 + s + 1) for s in range(steps)]
    # step-1 forward/backward recorded separately (no optimiser step)
    m.train()
    x0 = torch.from_numpy(xs[0])
    xh = m(x0)
    loss = m.recon_loss(xh, x0)
    m.zero_grad()
    loss.backward()
    out["step1/x_hat"] = xh.detach().numpy()
    out["step1/loss"] = np.float64(loss.item())
    g = grads_numpy(m, "step1/grad/")
    if keep_params:
        out.update(g)
    else:
        for k, v in g.items():
            out[k.replace("/grad/", "/gradsum/")] = np.float64(v.astype(np.float64).sum())
            out[k.replace("/grad/", "/gradsq/")] = np.float64((v.astype(np.float64) ** 2).sum())
    # restore pristine state (the forward above touched running stats)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in
                       init_state_dict(d, btl, n_layers, seed=seed).items()})
    for s in range(steps):
        out[f"x/{s}"] = xs[s]
        (lv,) = AutoEncoder.step(eng, (torch.from_numpy(xs[s]), torch.zeros(batch)))
        out[f"loss/{s}"] = np.float64(lv)
        if keep_params:
            out.update(sd_numpy(m, f"after{s}/"))
    m.eval()
    with torch.no_grad():
        out["eval/x_hat"] = m(torch.from_numpy(xs[0])).numpy()
        (vl,) = AutoEncoder.validate(eng, (torch.from_numpy(xs[0]), torch.zeros(batch)))
    out["eval/loss"] = np.float64(vl)
    return m, out


def scoring_case(m, out, d, seed, n_normal, n_anom):
    """get_diffs + BASE/SAP/NAP scores and AUROCs (reconstruction_aggregation.py,
    utils/metric.py) on a seeded split, with the trained model ``m``."""
    from reconstruction_aggregation import get_diffs
    from utils import metric
    sp = synth_split(n_normal, n_anom, d, seed=seed + 7)
    out["score/train_x"] = sp["train"]
    out["score/valid_x"] = sp["valid"]
    out["score/test_x"] = sp["test"]
    out["score/test_label"] = sp["test_label"]
    with torch.no_grad():
        tr = get_diffs(sp["train"], m, batch_size=64)
        va = get_diffs(sp["valid"], m)
        te = get_diffs(sp["test"], m)
    for i, dd in enumerate(te):
        out[f"score/test_diff{i}"] = dd
    base, base_auc, *_ = metric.get_recon_loss(va[0], te[0], sp["test_label"], f1_quantiles=[.90])
    sap, sap_auc, *_ = metric.get_d_loss(tr, va, te, sp["test_label"], start_layer_index=0,
                                         end_layer_index=len(te) + 1, norm_type=2, f1_quantiles=[.90])
    with tempfile.TemporaryDirectory() as td:
        cfg = types.SimpleNamespace(train_diffs=os.path.join(td, "td.pt"))
        nap, nap_auc, *_ = metric.get_d_norm_loss(tr, va, te, sp["test_label"], cfg, start_layer_index=0,
                                                  end_layer_index=len(te) + 1, norm_type=2,
                                                  f1_quantiles=[.90])
    # the NAP fit itself (utils/metric.py:213-217 with the reference classes), so
    # the score formula can be pinned independently of the SVD's conditioning
    from utils.normalize import Rotater, Standardizer
    trc = np.concatenate(tr, axis=1)
    rot, std = Rotater(), Standardizer()
    rot.fit(trc, gpu_id=-1)
    std.fit(rot.run(trc, gpu_id=-1))
    out["score/nap_mu_r"] = rot.mu.numpy()
    out["score/nap_v"] = rot.v.numpy()
    out["score/nap_mu_s"] = std.mu.numpy()
    out["score/nap_var"] = std.var.numpy()
    out["score/base"] = np.asarray(base, np.float64)
    out["score/sap"] = np.asarray(sap, np.float64)
    out["score/nap"] = np.asarray(nap, np.float64)
    out["score/base_auroc"] = np.float64(base_auc)
    out["score/sap_auroc"] = np.float64(sap_auc)
    out["score/nap_auroc"] = np.float64(nap_auc)


def nap_case(seed=5):
    """Well-conditioned NAP fit/run (utils/normalize.py:20-103) on gaussian
    'diffs' with distinct per-direction scales (N_train >> dims)."""
    from utils.normalize import Rotater, Standardizer
    rng = np.random.Generator(np.random.PCG64(seed))
    dims = 48
    mix = rng.normal(size=(dims, dims)) * np.geomspace(3.0, 0.3, dims)[None, :]
    train = (rng.normal(size=(3000, dims)) @ mix.T + rng.normal(size=dims)).astype(np.float32)
    test = (rng.normal(size=(200, dims)) * 1.3 @ mix.T).astype(np.float32)
    rot, std = Rotater(), Standardizer()
    rot.fit(train, gpu_id=-1)
    std.fit(rot.run(train, gpu_id=-1))
    score = (np.abs(std.run(rot.run(test, gpu_id=-1))) ** 2).mean(axis=1)
    return {"train": train, "test": test, "score": score.astype(np.float64),
            "mu_r": rot.mu.numpy(), "v": rot.v.numpy(), "mu_s": std.mu.numpy(), "var": std.var.numpy()}


def vib_case(seed=3):
    """Reference VIB decorator (decorators/variational_info_bottleneck.py) on an
    FCModule with output 2*btl; eps recovered as (z-mu)/sigma."""
    from modules import FCModule
    from utils.common_utils import get_hidden_layer_sizes
    d, btl, b, k = 64, 8, 16, 3
    torch.manual_seed(seed)
    enc = FCModule(d, 2 * btl, get_hidden_layer_sizes(d, 2 * btl, 2), use_batch_norm=True,
                   act="leakyrelu", last_act=None)
    dec = FCModule(btl, d, get_hidden_layer_sizes(btl, d, 2), use_batch_norm=True,
                   act="leakyrelu", last_act=None)
    x = torch.from_numpy(synth_windows(b, d, seed=seed))
    out = {"x": x.numpy()}
    out.update({"enc/" + k2: v.detach().numpy().copy() for k2, v in enc.state_dict().items()})
    out.update({"dec/" + k2: v.detach().numpy().copy() for k2, v in dec.state_dict().items()})
    enc.train()
    dec.train()
    r = enc(x, distribution="normal", k=k)
    sigma = (r["logvar"] * 0.5).exp()
    out["mu"] = r["mu"].detach().numpy()
    out["logvar"] = r["logvar"].detach().numpy()
    out["z"] = r["z"].detach().numpy()
    out["eps"] = ((r["z"] - r["mu"]) / sigma).detach().numpy()
    xh = dec(r["z"])
    out["x_hat"] = xh.detach().numpy()
    enc.eval()
    with torch.no_grad():
        r2 = enc(x, distribution="normal", k=2, stochastic_inference=False)
    out["det_z"] = r2["z"].numpy()
    try:
        enc(x, distribution="normal", k=0)
        out["k0_raises"] = np.bool_(False)
    except ValueError:
        out["k0_raises"] = np.bool_(True)
    return out


def main():
    torch.use_deterministic_algorithms(False)
    os.makedirs(HERE, exist_ok=True)
    m, out = train_case("c1_ft64", d=64, btl=100, n_layers=5, batch=32, seed=0)
    scoring_case(m, out, d=64, seed=0, n_normal=2000, n_anom=100)
    np.savez_compressed(os.path.join(HERE, "c1_ft64.npz"), **out)
    print("c1_ft64", out["loss/0"], out["score/sap_auroc"])

    m, out = train_case("mm192", d=192, btl=16, n_layers=5, batch=64, seed=1)
    scoring_case(m, out, d=192, seed=1, n_normal=2000, n_anom=100)
    np.savez_compressed(os.path.join(HERE, "mm192.npz"), **out)
    print("mm192", out["loss/0"], out["score/sap_auroc"])

    m, out = train_case("d1728", d=1728, btl=100, n_layers=5, batch=64, seed=2, steps=2,
                        keep_params=False)
    # big case: keep x_hat only for a few rows to stay small
    out["step1/x_hat"] = out["step1/x_hat"][:8]
    out["eval/x_hat"] = out["eval/x_hat"][:8]
    for s in range(2):
        out[f"x/{s}"] = out[f"x/{s}"]  # 64 x 1728 inputs: ~440 KB each, compressed
    np.savez_compressed(os.path.join(HERE, "d1728.npz"), **out)
    print("d1728", out["loss/0"], out["loss/1"])

    np.savez_compressed(os.path.join(HERE, "vib.npz"), **vib_case())
    np.savez_compressed(os.path.join(HERE, "nap.npz"), **nap_case())
    print("vib done")


if __name__ == "__main__":
    main()
