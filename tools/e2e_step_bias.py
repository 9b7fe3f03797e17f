"""Where along the trajectory the product's fp32 training loss leaves the
reference ensemble (the loss-EMA offset): per seed, the
product's 288 AutoEncoder.step losses (tests/golden/e2e.npz configuration,
fp32, Adam lr 1e-3, the seeded loaders) against the five members' per-step
losses in the fixture (reference at 8 / 1 / 2 / 4 threads + the CPU oracle):
z(t) = (L_product - mean) / std over the members, averaged over 24-step
(two-epoch) windows and over seeds; the same statistic for each member
against the other four (leave-one-out) as the yardstick.
Usage: python tools/e2e_step_bias.py [seeds=0,1,...,7|all] [knob=value ...]
(knobs: _native.tune names, e.g. splitk=4: every GEMM's K loop in 4 slices
summed in slice order -- a more accurate fp32 summation -- to test whether the
offset follows the fp32 GEMMs' rounding noise)"""
import sys
import types

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import numpy as np  # noqa: E402
import torch  # noqa: E402

g = np.load("tests/golden/e2e.npz")
all_seeds = sorted({int(k.split("/")[0][1:]) for k in g.files if k.startswith("s") and k.endswith("/step_loss")})
seeds = [int(s) for s in sys.argv[1].split(",")] if len(sys.argv) > 1 and sys.argv[1] != "all" else all_seeds
knobs = dict(a.split("=") for a in sys.argv[2:])
members = ["", "ref1/", "ref2/", "ref4/", "oracle/"]


def cfg_for(seed):
    skip = ("meta/torch", "meta/seeds", "meta/floor_threads")
    c = types.SimpleNamespace(**{k[len("meta/"):]: g[k].item() for k in g.files
                                 if k.startswith("meta/") and k not in skip})
    c.gpu_id = 0
    c.dtype = "f32"
    c.data_seed, c.sampler_seed, c.model_seed = 100 + seed, 200 + seed, 300 + seed
    return c


def product_losses(seed, n):
    from icra2021_multimodal_ad_amd.auto_encoder import AutoEncoder
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict
    from icra2021_multimodal_ad_amd.data_loaders import get_loaders
    from icra2021_multimodal_ad_amd.model_builder import get_model
    from icra2021_multimodal_ad_amd import _native
    cfg = cfg_for(seed)
    with _native.tune(**{k: int(v) for k, v in knobs.items()}):
        return _train(cfg, n)


def _train(cfg, n):
    from icra2021_multimodal_ad_amd.auto_encoder import AutoEncoder
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict
    from icra2021_multimodal_ad_amd.data_loaders import get_loaders
    from icra2021_multimodal_ad_amd.model_builder import get_model
    model = get_model(cfg)
    sd0 = init_state_dict(cfg.input_size, cfg.btl_size, cfg.n_layers, seed=cfg.model_seed)
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd0.items()})
    _, tr, _, _ = get_loaders(cfg)
    eng = types.SimpleNamespace(model=model, optimizer=torch.optim.Adam(model.parameters(), lr=1e-3),
                                config=cfg)
    out = []
    while len(out) < n:
        for batch in tr:
            out.append(AutoEncoder.step(eng, batch)[0])
            if len(out) == n:
                break
    return np.asarray(out, np.float64)


W = 24
zs, loo = [], {m or "ref8/": [] for m in members}
for s in seeds:
    ens = np.stack([np.asarray(g[f"s{s}/{m}step_loss"], np.float64) for m in members])
    n = ens.shape[1]
    ours = product_losses(s, n)
    mu, sd = ens.mean(0), np.maximum(ens.std(0, ddof=1), 1e-12)
    z = (ours - mu) / sd
    zs.append(z)
    for i, m in enumerate(members):
        rest = np.delete(ens, i, axis=0)
        loo[m or "ref8/"].append((ens[i] - rest.mean(0)) / np.maximum(rest.std(0, ddof=1), 1e-12))
    win = [float(z[a:a + W].mean()) for a in range(0, n, W)]
    print(f"seed {s}: product z per {W}-step window " + " ".join(f"{v:+.2f}" for v in win), flush=True)
Z = np.stack(zs)
n = Z.shape[1]
print(f"knobs {knobs}")
print("all seeds, product: " + " ".join(f"{Z[:, a:a + W].mean():+.2f}" for a in range(0, n, W)))
print(f"all seeds, product: steps 2-288 mean z {Z[:, 1:].mean():+.3f}, fraction > 0 {(Z[:, 1:] > 0).mean():.3f}")
for m, lst in loo.items():
    L = np.stack(lst)
    print(f"leave-one-out {m:8s}: steps 2-288 mean z {L[:, 1:].mean():+.3f}, fraction > 0 {(L[:, 1:] > 0).mean():.3f}; "
          "windows " + " ".join(f"{L[:, a:a + W].mean():+.2f}" for a in range(0, n, W)))
