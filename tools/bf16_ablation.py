"""Which bf16 tensor of the throughput path moves the trained model's SAP /
NAP AUROC?  An ablation on the reference's own architecture (the modules of
oracle/torch_ref.py, restated here with explicit rounding points), trained
in torch fp32 on the GPU with bf16 rounding emulated at exactly the places
the product's bf16 step rounds:

  act : the stored activations -- the input x, every layer's post-activation
        a (BatchNorm statistics are taken from the rounded a) and post-BN y,
        the bottleneck z: everything a later GEMM reads as an operand;
  dz  : the stored gradients at every Linear output (the MSE epilogue's
        2(x_hat - x), the fused BN-backward's dz): the dW / bwd-data operands;
  w   : the weight operand of every GEMM (the bf16 shadow of the fp32 master;
        gradients flow to the fp32 master, biases / gamma / beta stay fp32);
  all : the three together (= the product's bf16 path);
  fp32: none (another fp32 implementation: the ablation's own floor);
  <v>_sr: variant v with stochastic instead of round-to-nearest rounding.

Every variant trains the e2e configuration (tests/golden/e2e.npz meta: D=1728,
btl 100, 24 epochs of 12 batches of 500) from the seed's initial weights on
the seed's batches (the build's loaders), keeps the best-on-valid state,
and is scored in fp32 (BASE / SAP every epoch, NAP at a few epochs: torch
fp32 SVD as utils/normalize.py does); each score is compared with the
REFERENCE's AUROC at the same epoch (e2e.npz, 8-thread run).  Prints one JSON
line per (seed, variant) and a summary per variant.
Usage: python tools/bf16_ablation.py [seeds=0+1+2] [variants=fp32+act+dz+w+all] [nap_epochs=6+12+18+24]
       python tools/bf16_ablation.py wc [seeds=0+1+2] [variants=fp32+act+w+all+all_sr]
         (the well-conditioned NAP fixture, tests/golden/nap_wc.npz: NAP per resolvable layer range)
"""
import json
import sys
import types

sys.path.insert(0, ".")
import numpy as np
import torch
import torch.nn.functional as F
from sklearn import metrics as skm

from icra2021_multimodal_ad_amd.common_utils import ae_widths, init_state_dict
from icra2021_multimodal_ad_amd.data_loaders import get_loaders

dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False
G = np.load("tests/golden/e2e.npz")
nap_epochs = [6, 12, 18, 24]


SR = {"on": False}


def bf(x):
    """fp32 -> bf16 -> fp32: round to nearest even, or (SR["on"]) stochastic
    rounding: uniform random low 16 bits added before truncation."""
    if not SR["on"]:
        return x.bfloat16().float()
    i = x.contiguous().view(torch.int32)
    r = torch.randint(0, 1 << 16, i.shape, device=i.device, dtype=torch.int32)
    return ((i + r) & ~0xFFFF).view(torch.float32)


class RoundAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return bf(x)

    @staticmethod
    def backward(ctx, g):
        return g


class RoundGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return bf(g)


class AE(torch.nn.Module):
    """FC-AE of the reference (Linear -> LeakyReLU(0.2) -> BatchNorm1d per
    hidden layer, plain Linear last in each module), with the rounding
    points of the product's bf16 step."""

    def __init__(self, enc, dec, mode):
        super().__init__()
        self.mode = mode
        self.lin, self.bn, self.last = torch.nn.ModuleList(), torch.nn.ModuleList(), []
        for widths in (enc, dec):
            n = len(widths) - 1
            for i in range(n):
                self.lin.append(torch.nn.Linear(widths[i], widths[i + 1]))
                self.bn.append(torch.nn.BatchNorm1d(widths[i + 1]) if i < n - 1 else torch.nn.Identity())
                self.last.append(i == n - 1)
        self.n_enc = len(enc) - 1

    def load_ref(self, sd):
        """The reference's 60 state_dict keys -> these modules."""
        i = 0
        for mod, widths in (("encoder", None), ("decoder", None)):
            j = 0
            while f"{mod}.net.{j}.layer.weight" in sd:
                self.lin[i].weight.data.copy_(torch.as_tensor(sd[f"{mod}.net.{j}.layer.weight"]))
                self.lin[i].bias.data.copy_(torch.as_tensor(sd[f"{mod}.net.{j}.layer.bias"]))
                if f"{mod}.net.{j}.bn.weight" in sd:
                    b = self.bn[i]
                    b.weight.data.copy_(torch.as_tensor(sd[f"{mod}.net.{j}.bn.weight"]))
                    b.bias.data.copy_(torch.as_tensor(sd[f"{mod}.net.{j}.bn.bias"]))
                    b.running_mean.copy_(torch.as_tensor(sd[f"{mod}.net.{j}.bn.running_mean"]))
                    b.running_var.copy_(torch.as_tensor(sd[f"{mod}.net.{j}.bn.running_var"]))
                i += 1
                j += 1

    def layer(self, i, h, train_round):
        m = self.mode if train_round else ()
        w = self.lin[i].weight
        if "w" in m:
            w = RoundAct.apply(w)                 # bf16 shadow; the gradient reaches the fp32 master
        z = F.linear(h, w, self.lin[i].bias)
        if "dz" in m:
            z = RoundGrad.apply(z)
        if self.last[i]:
            if "act" in m and i == self.n_enc - 1:
                z = RoundAct.apply(z)             # the bottleneck is a GEMM operand
            return z
        a = F.leaky_relu(z, 0.2)
        if "act" in m:
            a = RoundAct.apply(a)
        y = self.bn[i](a)
        if "act" in m:
            y = RoundAct.apply(y)
        return y

    def forward(self, x, train_round=False):
        h = RoundAct.apply(x) if train_round and "act" in self.mode else x
        for i in range(len(self.lin)):
            h = self.layer(i, h, train_round)
        return h


def diffs(model, x, bs=698):
    """get_diffs (reconstruction_aggregation.py:6-37), eval mode, fp32."""
    model.eval()
    out = []
    with torch.no_grad():
        for s in range(0, x.shape[0], bs):
            xb = x[s:s + bs]
            xt = model(xb)
            d = [xt - xb]
            a, b = xb, xt
            for i in range(model.n_enc):
                a, b = model.layer(i, a, False), model.layer(i, b, False)
                d.append(b - a)
            out.append(d)
    return [torch.cat(c, 0) for c in zip(*out)]


def auroc(score, lab):
    fpr, tpr, _ = skm.roc_curve(lab, score)
    return float(skm.auc(fpr, tpr))


def nap_auroc(tr, te, lab):
    """utils/normalize.py Rotater (torch fp32 SVD) + Standardizer, utils/metric.py:183-238."""
    x = torch.cat(tr, 1)
    mu = x.mean(0)
    xc = x - mu
    v = torch.linalg.svd(xc, full_matrices=False)[2].T
    rt = xc @ v
    ms, var = rt.mean(0), rt.var(0, unbiased=True)
    st = ((torch.cat(te, 1) - mu) @ v - ms) / var.sqrt()
    return auroc((st ** 2).mean(1).cpu().numpy(), lab)


def run(seed, mode, override=None):
    c = types.SimpleNamespace(**{k[5:]: G[k].item() for k in G.files
                                 if k.startswith("meta/") and k not in ("meta/torch", "meta/seeds",
                                                                        "meta/floor_threads")})
    c.__dict__.update(override or {})
    c.gpu_id, c.dtype = 0, "f32"
    c.data_seed, c.sampler_seed, c.model_seed = 100 + seed, 200 + seed, 300 + seed
    enc, dec = ae_widths(c.input_size, c.btl_size, c.n_layers)
    torch.manual_seed(0)
    SR["on"] = mode.endswith("_sr")
    base_mode = mode[:-3] if SR["on"] else mode
    m = AE(enc, dec, set() if base_mode == "fp32" else
           ({"act", "dz", "w"} if base_mode == "all" else {base_mode})).to(dev)
    m.load_ref(init_state_dict(c.input_size, c.btl_size, c.n_layers, seed=c.model_seed))
    dset, trl, val, tel = get_loaders(c, device=dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    # reading the train split in sampler order draws a permutation: keep the
    # train sampler's generator where it was, so the batch order is the reference's
    st = trl.sampler.rng.bit_generator.state
    tr_x, _ = dset.get_transformed_data(trl)
    trl.sampler.rng.bit_generator.state = st
    va_x, _ = dset.get_transformed_data(val)
    te_x, te_y = dset.get_transformed_data(tel)
    lab = np.isin(np.asarray(te_y.cpu() if torch.is_tensor(te_y) else te_y), [c.target_class])
    ref = {k: np.asarray(G[f"s{seed}/epoch_auroc/{k}"]) for k in ("base", "sap", "nap")
           if f"s{seed}/epoch_auroc/{k}" in G.files}
    rows, best, lowest = [], None, np.inf
    for ep in range(1, c.n_epochs + 1):
        m.train()
        for x, _ in trl:
            opt.zero_grad()
            loss = ((m(x, train_round=True) - x) ** 2).sum()
            loss.backward()
            opt.step()
        m.eval()
        with torch.no_grad():
            vema = None
            for x, _ in val:
                lv = float(((m(x) - x) ** 2).sum())
                vema = lv if vema is None else 0.98 * vema + 0.02 * lv
        te = diffs(m, te_x)
        r = {"epoch": ep, "valid": vema, "base": auroc((te[0] ** 2).mean(1).cpu().numpy(), lab),
             "sap": auroc((torch.cat(te, 1) ** 2).mean(1).cpu().numpy(), lab)}
        if ep in nap_epochs and "nap" in ref:
            r["nap"] = nap_auroc(diffs(m, tr_x, c.batch_size), te, lab)
        rows.append(r)
        if vema < lowest:
            lowest, best = vema, ep
    out = {"seed": seed, "variant": mode, "best_epoch": best}
    for k in ("base", "sap", "nap"):
        d = [r[k] - ref[k][r["epoch"] - 1] for r in rows if k in r]
        out[f"{k}_mean_abs_delta_same_epoch"] = float(np.mean(np.abs(d))) if d else None
        out[f"{k}_deltas"] = [round(v, 5) for v in d]
    return out


def run_wc(seed, mode):
    """The well-conditioned NAP fixture (tests/golden/nap_wc.npz, D=256):
    train the variant for the fixture's epochs from the seed's initial
    weights, keep the best-on-valid state, and score NAP on every
    well-conditioned layer range; |AUROC - reference (8 threads)| per range
    next to the reference's own |ref1 - ref8|."""
    W = np.load("tests/golden/nap_wc.npz")
    skip = ("meta/torch", "meta/seeds", "meta/min_var_ratio", "meta/members")
    c = types.SimpleNamespace(**{k[5:]: W[k].item() for k in W.files if k.startswith("meta/") and k not in skip})
    c.gpu_id, c.dtype = 0, "f32"
    c.data_seed, c.sampler_seed, c.model_seed = 500 + seed, 600 + seed, 700 + seed
    enc, dec = ae_widths(c.input_size, c.btl_size, c.n_layers)
    torch.manual_seed(0)
    SR["on"] = mode.endswith("_sr")
    base_mode = mode[:-3] if SR["on"] else mode
    m = AE(enc, dec, set() if base_mode == "fp32" else
           ({"act", "dz", "w"} if base_mode == "all" else {base_mode})).to(dev)
    m.load_ref(init_state_dict(c.input_size, c.btl_size, c.n_layers, seed=c.model_seed))
    dset, trl, val, tel = get_loaders(c, device=dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    st = trl.sampler.rng.bit_generator.state
    tr_x, _ = dset.get_transformed_data(trl)
    trl.sampler.rng.bit_generator.state = st
    te_x, te_y = dset.get_transformed_data(tel)
    lab = np.isin(np.asarray(te_y.cpu() if torch.is_tensor(te_y) else te_y), [c.target_class])
    best, lowest = None, np.inf
    for ep in range(1, c.n_epochs + 1):
        m.train()
        for x, _ in trl:
            opt.zero_grad()
            ((m(x, train_round=True) - x) ** 2).sum().backward()
            opt.step()
        m.eval()
        with torch.no_grad():
            vema = None
            for x, _ in val:
                lv = float(((m(x) - x) ** 2).sum())
                vema = lv if vema is None else 0.98 * vema + 0.02 * lv
        if vema < lowest:
            lowest, best = vema, {k: v.clone() for k, v in m.state_dict().items()}
    m.load_state_dict(best)
    tr, te = diffs(m, tr_x, c.batch_size), diffs(m, te_x)
    out, d, f = {"fixture": "nap_wc", "seed": seed, "variant": mode}, [], []
    for s_, e_ in np.asarray(W[f"s{seed}/ranges"]).reshape(-1, 2):
        a = nap_auroc(tr[s_:e_], te[s_:e_], lab)
        r8 = float(W[f"s{seed}/nap_{s_}_{e_}/auroc"])
        r1 = float(W[f"s{seed}/ref1/nap_{s_}_{e_}/auroc"])
        d.append(abs(a - r8))
        f.append(abs(r1 - r8))
    out.update(nap_mean_abs_delta=float(np.mean(d)), nap_p90=float(np.quantile(d, 0.9)),
               ref_floor_mean=float(np.mean(f)), ref_floor_p90=float(np.quantile(f, 0.9)))
    return out


def main():
    global nap_epochs
    if len(sys.argv) > 1 and sys.argv[1] == "wc":
        seeds = [int(s) for s in (sys.argv[2] if len(sys.argv) > 2 else "0+1+2").split("+")]
        variants = (sys.argv[3] if len(sys.argv) > 3 else "fp32+act+w+all+all_sr").split("+")
        agg = {}
        for v in variants:
            for s in seeds:
                o = run_wc(s, v)
                print(json.dumps(o), flush=True)
                agg.setdefault(v, []).append(o["nap_mean_abs_delta"])
            print(json.dumps({"fixture": "nap_wc", "variant": v, "nap_mean_abs_delta": float(np.mean(agg[v])),
                              "seeds": seeds}), flush=True)
        return
    seeds = [int(s) for s in (sys.argv[1] if len(sys.argv) > 1 else "0+1+2").split("+")]
    variants = (sys.argv[2] if len(sys.argv) > 2 else "fp32+act+dz+w+all").split("+")
    if len(sys.argv) > 3:
        nap_epochs = [int(e) for e in sys.argv[3].split("+")]
    summary = {}
    for s in seeds:
        for v in variants:
            o = run(s, v)
            print(json.dumps(o), flush=True)
            for k in ("base", "sap", "nap"):
                summary.setdefault(v, {}).setdefault(k, []).append(o[f"{k}_mean_abs_delta_same_epoch"])
    for v, d in summary.items():
        print(json.dumps({"variant": v, **{f"{k}_mean_abs_delta": float(np.mean(x)) for k, x in d.items()},
                          "seeds": seeds}), flush=True)


if __name__ == "__main__":
    main()
