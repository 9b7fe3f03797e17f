"""CPU oracle for the autoencoder train-and-score hot path.

TEST INFRASTRUCTURE ONLY.  This module is the checker: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``icra2021_multimodal_ad_amd``) never imports, calls or
falls back to anything here.

It is a plain-numpy restatement (fp32 storage, fp32 BLAS matmuls, fp64 where
the reference itself uses fp64) of the reference's algorithm.  Every function
cites the reference file:line it restates (paths relative to the reference
repo root).  It is pinned against golden vectors produced by importing the
reference itself in the build container (``tests/golden/gen_golden.py``);
``tests/test_oracle_golden.py`` checks the pin.

Model representation: a model is ``{"enc": [layer...], "dec": [layer...]}``;
a layer is a dict with ``W`` [out,in], ``b`` [out], ``act`` ("leakyrelu" or
None) and ``bn`` (None or dict with ``gamma``, ``beta``, ``rm``, ``rv``,
``nbt``).  This mirrors ``FCModule.layer_list`` (modules/fc_module.py:34-51).
"""
import math

import numpy as np

F32 = np.float32


class _Precision:
    """Storage precision of the oracle (fp32 = reference numerics; fp64 is
    used by the tests as 'truth' to size fp32 summation-order tolerances)."""
    ft = np.float32


_P = _Precision()


def set_precision(dtype):
    _P.ft = np.dtype(dtype).type


LEAKY_SLOPE = 0.2      # modules/activation.py:37-38 (nn.LeakyReLU(.2))
BN_EPS = 1e-5          # nn.BatchNorm1d default, layers/fc_layer.py:33
BN_MOMENTUM = 0.1      # nn.BatchNorm1d default


# --------------------------------------------------------------------------
# shapes
# --------------------------------------------------------------------------
def get_hidden_layer_sizes(start_size, end_size, n_hidden_layers):
    """utils/common_utils.py:22-31 -- float step, truncation toward zero."""
    diff = (start_size - end_size) / (n_hidden_layers + 1)
    return [int(start_size - diff * (i + 1)) for i in range(n_hidden_layers)]


def ae_layer_sizes(input_size, btl_size, n_layers, enc_out=None):
    """model_builder.py:6-45.  Returns (encoder widths, decoder widths) as
    full lists [in, hidden..., out].  ``enc_out`` overrides the encoder output
    width (2*btl for the VIB head)."""
    if not isinstance(input_size, int):
        c, h, w = input_size
        input_size = c * h * w
    eo = btl_size if enc_out is None else enc_out
    enc = [input_size] + get_hidden_layer_sizes(input_size, eo, n_layers - 1) + [eo]
    dec = [btl_size] + get_hidden_layer_sizes(btl_size, input_size, n_layers - 1) + [input_size]
    return enc, dec


# --------------------------------------------------------------------------
# forward
# --------------------------------------------------------------------------
def leaky(z, slope=LEAKY_SLOPE):
    """modules/activation.py:37-45 (LeakyReLU forward)."""
    return np.where(z > 0, z, z * _P.ft(slope)).astype(_P.ft)


def apply_act(z, act):
    """modules/activation.py:20-45.  Only the activations the AE uses plus the
    elementwise ones the surface exposes."""
    if act is None:
        return z
    if act == "leakyrelu":
        return leaky(z)
    if act == "relu":
        return np.maximum(z, 0).astype(_P.ft)
    if act == "sigmoid":
        return (1.0 / (1.0 + np.exp(-z.astype(np.float64)))).astype(_P.ft)
    if act == "tanh":
        return np.tanh(z).astype(_P.ft)
    raise NotImplementedError(act)


def fc_forward(x, layer, train):
    """layers/fc_layer.py:37-48: y = BN(act(x W^T + b)); activation BEFORE BN.

    Train-mode BN (torch native_batch_norm): biased batch variance for
    normalisation, unbiased for the running update, momentum 0.1, eps 1e-5.
    Returns (y, cache); running stats are updated in place in train mode."""
    x = x.astype(_P.ft, copy=False)
    z = (x @ layer["W"].T + layer["b"]).astype(_P.ft)
    a = apply_act(z, layer["act"])
    cache = {"x": x, "z": z, "a": a}
    bn = layer.get("bn")
    if bn is None:
        return a, cache
    if train:
        n = a.shape[0]
        mu = a.mean(axis=0, dtype=np.float64)
        var = ((a - mu) ** 2).mean(axis=0, dtype=np.float64)
        rstd = 1.0 / np.sqrt(var + BN_EPS)
        xhat = ((a - mu) * rstd).astype(_P.ft)
        y = (xhat * bn["gamma"] + bn["beta"]).astype(_P.ft)
        unbiased = var * n / max(n - 1, 1)
        bn["rm"] = ((1 - BN_MOMENTUM) * bn["rm"] + BN_MOMENTUM * mu).astype(_P.ft)
        bn["rv"] = ((1 - BN_MOMENTUM) * bn["rv"] + BN_MOMENTUM * unbiased).astype(_P.ft)
        bn["nbt"] = int(bn.get("nbt", 0)) + 1
        cache.update(xhat=xhat, rstd=rstd.astype(_P.ft), mu=mu.astype(_P.ft))
    else:
        rstd = 1.0 / np.sqrt(bn["rv"].astype(np.float64) + BN_EPS)
        y = ((a - bn["rm"]) * rstd * bn["gamma"] + bn["beta"]).astype(_P.ft)
    return y, cache


def module_forward(x, layers, train):
    """modules/fc_module.py:59-61 (nn.Sequential over layer_list).  Rank>2
    inputs are flattened for BN exactly as layers/fc_layer.py:40-43."""
    shape = x.shape
    h = x.reshape(-1, shape[-1])
    caches = []
    for layer in layers:
        h, c = fc_forward(h, layer, train)
        caches.append(c)
    return h.reshape(*shape[:-1], h.shape[-1]), caches


def ae_forward(x, model, train):
    """models/auto_encoder.py:36-50: z = enc(x).view(B,-1); x_hat = dec(z)."""
    z, ce = module_forward(x, model["enc"], train)
    xh, cd = module_forward(z, model["dec"], train)
    return xh, {"enc": ce, "dec": cd, "z": z}


def mse_sum(xh, x):
    """modules/loss.py:31-32,47-52 with reduction='sum' (model_builder.py:42)."""
    d = (xh.astype(np.float64) - x.astype(np.float64))
    return float((d * d).sum())


# --------------------------------------------------------------------------
# backward (autograd of the forward above, as torch computes it)
# --------------------------------------------------------------------------
def fc_backward(dy, layer, cache):
    """Backward of layers/fc_layer.py:37-48.  Returns (dx, grads)."""
    g = {}
    bn = layer.get("bn")
    if bn is not None:
        xhat, rstd = cache["xhat"], cache["rstd"]
        n = dy.shape[0]
        dbeta = dy.sum(axis=0, dtype=np.float64)
        dgamma = (dy * xhat).sum(axis=0, dtype=np.float64)
        da = (bn["gamma"] * rstd / n) * (n * dy - dbeta - xhat * dgamma)
        da = da.astype(_P.ft)
        g["gamma"] = dgamma.astype(_P.ft)
        g["beta"] = dbeta.astype(_P.ft)
    else:
        da = dy
    if layer["act"] == "leakyrelu":
        dz = np.where(cache["z"] > 0, da, da * _P.ft(LEAKY_SLOPE)).astype(_P.ft)
    elif layer["act"] is None:
        dz = da
    else:
        raise NotImplementedError(layer["act"])
    g["W"] = (dz.T @ cache["x"]).astype(_P.ft)
    g["b"] = dz.sum(axis=0, dtype=np.float64).astype(_P.ft)
    dx = (dz @ layer["W"]).astype(_P.ft)
    return dx, g


def module_backward(dout, layers, caches):
    shape = dout.shape
    d = dout.reshape(-1, shape[-1]).astype(_P.ft)
    grads = [None] * len(layers)
    for i in range(len(layers) - 1, -1, -1):
        d, grads[i] = fc_backward(d, layers[i], caches[i])
    return d, grads


def ae_train_grads(x, model):
    """One AutoEncoder.step forward+backward (models/auto_encoder.py:57-77)
    without the optimiser: returns (loss, x_hat, grads{"enc","dec"})."""
    xh, cache = ae_forward(x, model, train=True)
    loss = mse_sum(xh, x)
    dxh = (_P.ft(2.0) * (xh - x)).astype(_P.ft)
    dz, gd = module_backward(dxh, model["dec"], cache["dec"])
    _, ge = module_backward(dz, model["enc"], cache["enc"])
    return loss, xh, {"enc": ge, "dec": gd}


# --------------------------------------------------------------------------
# Adam (novelty_detection.py:90, torch.optim.Adam defaults, lr 1e-3)
# --------------------------------------------------------------------------
PARAM_NAMES = ("W", "b", "gamma", "beta")


def iter_params(model):
    for side in ("enc", "dec"):
        for li, layer in enumerate(model[side]):
            for name in ("W", "b"):
                yield (side, li, name), layer, None
            if layer.get("bn") is not None:
                for name in ("gamma", "beta"):
                    yield (side, li, name), layer, "bn"


def adam_step(model, grads, state, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam single-tensor step (amsgrad=False, weight_decay=0):
    m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
    p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)."""
    state["t"] = state.get("t", 0) + 1
    t = state["t"]
    b1, b2 = betas
    bc1 = 1 - b1 ** t
    bc2 = 1 - b2 ** t
    for key, layer, where in iter_params(model):
        side, li, name = key
        g = grads[side][li][name].astype(_P.ft)
        holder = layer["bn"] if where == "bn" else layer
        pname = name
        p = holder[pname]
        m = state.setdefault(("m",) + key, np.zeros_like(p))
        v = state.setdefault(("v",) + key, np.zeros_like(p))
        m[...] = (b1 * m + (1 - b1) * g).astype(_P.ft)
        v[...] = (b2 * v + (1 - b2) * g * g).astype(_P.ft)
        denom = (np.sqrt(v) / _P.ft(math.sqrt(bc2)) + _P.ft(eps)).astype(_P.ft)
        holder[pname] = (p - _P.ft(lr / bc1) * m / denom).astype(_P.ft)
    return state


def train_step(x, model, state, lr=1e-3):
    """AutoEncoder.step (models/auto_encoder.py:57-77) + Adam: returns loss."""
    loss, _, grads = ae_train_grads(x, model)
    adam_step(model, grads, state, lr=lr)
    return loss


# --------------------------------------------------------------------------
# VIB head (decorators/variational_info_bottleneck.py:19-42) + KL (build-defined)
# --------------------------------------------------------------------------
def vib_split(out):
    """decorators/variational_info_bottleneck.py:34: mu, logvar = split(D//2)."""
    h = out.shape[-1] // 2
    return out[..., :h], out[..., h:]


def vib_reparam(mu, logvar, eps_noise):
    """decorators/variational_info_bottleneck.py:22-24,37:
    sigma = exp(0.5*logvar); z[k] = eps[k]*sigma + mu.  ``eps_noise`` is
    [k, B, btl] (injected noise; the reference draws randn_like)."""
    sigma = np.exp(_P.ft(0.5) * logvar).astype(_P.ft)
    return (eps_noise * sigma[None] + mu[None]).astype(_P.ft)


def kl_normal(mu, logvar):
    """Build-defined KL term (SURVEY §8 a10'): -1/2 sum(1 + lv - mu^2 - e^lv)."""
    mu = mu.astype(np.float64)
    lv = logvar.astype(np.float64)
    return float(-0.5 * (1.0 + lv - mu * mu - np.exp(lv)).sum())


def vib_ae_train_grads(x, model, eps_noise, beta_kl):
    """Build-defined VIB-AE step (SURVEY §8 a10'): loss = sum_k,b,d
    (dec(z_k)-x)^2 / k + beta*KL; returns (loss, grads, aux)."""
    k = eps_noise.shape[0]
    out, ce = module_forward(x, model["enc"], train=True)
    mu, logvar = vib_split(out)
    z = vib_reparam(mu, logvar, eps_noise)                 # [k,B,btl]
    xh, cd = module_forward(z, model["dec"], train=True)    # [k,B,D]
    d = xh.astype(np.float64) - x[None].astype(np.float64)
    recon = float((d * d).sum()) / k
    kl = kl_normal(mu, logvar)
    loss = recon + beta_kl * kl
    dxh = (_P.ft(2.0 / k) * (xh - x[None])).astype(_P.ft)
    dz, gd = module_backward(dxh, model["dec"], cd)
    dz = dz.reshape(z.shape)
    sigma = np.exp(_P.ft(0.5) * logvar).astype(_P.ft)
    dmu = dz.sum(axis=0) + _P.ft(beta_kl) * mu
    dlv = (dz * eps_noise).sum(axis=0) * sigma * _P.ft(0.5) + _P.ft(0.5 * beta_kl) * (np.exp(logvar) - 1)
    dout = np.concatenate([dmu, dlv], axis=-1).astype(_P.ft)
    _, ge = module_backward(dout, model["enc"], ce)
    return loss, {"enc": ge, "dec": gd}, {"mu": mu, "logvar": logvar, "z": z, "x_hat": xh,
                                          "recon": recon, "kl": kl}


# --------------------------------------------------------------------------
# scoring (reconstruction_aggregation.py + utils/metric.py + utils/normalize.py)
# --------------------------------------------------------------------------
def get_diffs(x, model, batch_size=698):
    """reconstruction_aggregation.py:6-37 (eval mode): d0 = x_hat - x and, for
    each encoder layer l, d_l = enc_l(x_hat_{l-1}) - enc_l(x_{l-1})."""
    out = None
    for s in range(0, x.shape[0], batch_size):
        xb = x[s:s + batch_size].astype(_P.ft)
        xh, _ = ae_forward(xb, model, train=False)
        diffs = [xh - xb]
        h, ht = xb, xh
        for layer in model["enc"]:
            h, _ = fc_forward(h, layer, train=False)
            ht, _ = fc_forward(ht, layer, train=False)
            diffs.append(ht - h)
        if out is None:
            out = [[d] for d in diffs]
        else:
            for o, d in zip(out, diffs):
                o.append(d)
    return [np.concatenate(o, axis=0).astype(_P.ft) for o in out]


def layer_sq_sums(diffs):
    """Per-window sum of squared diffs per layer: the reduction the scoring
    kernels emit ([n_diff_layers, N], float64 here)."""
    return np.stack([(d.astype(np.float64) ** 2).sum(axis=1) for d in diffs])


def _clamp_layers(n, start, end):
    """utils/metric.py:155-162 (start/end clamping of get_d_loss)."""
    if end is None:
        end = n + 1
    if start > n - 1:
        start = n - 1
    if end - start < 1:
        end = start + 1
    return start, end


def base_score(diffs):
    """utils/metric.py:133: mean(d0^2, axis=1)."""
    return (diffs[0].astype(np.float64) ** 2).mean(axis=1)


def sap_score(diffs, start_layer_index=0, end_layer_index=None):
    """utils/metric.py:155-171: mean of squares over concatenated diffs."""
    s, e = _clamp_layers(len(diffs), start_layer_index, end_layer_index)
    cat = np.concatenate(diffs[s:e], axis=-1).astype(np.float64)
    return (cat ** 2).mean(axis=1)


def nap_fit(train_cat):
    """utils/normalize.py:52-70 (Rotater.fit: mu, V from SVD of centred train
    diffs) + :20-34 (Standardizer.fit on the rotated train diffs; var is the
    ddof=1 np.cov diagonal)."""
    x = train_cat.astype(_P.ft)
    mu_r = x.mean(axis=0, dtype=np.float64).astype(_P.ft)
    _, _, vt = np.linalg.svd((x - mu_r).astype(np.float64), full_matrices=False)
    v = vt.T.astype(_P.ft)
    rot = ((x - mu_r) @ v).astype(_P.ft)
    mu_s = rot.mean(axis=0, dtype=np.float64).astype(_P.ft)
    c = rot - mu_s
    var = ((c.astype(np.float64) ** 2).sum(axis=0) / max(c.shape[0] - 1, 1)).astype(_P.ft)
    return {"mu_r": mu_r, "v": v, "mu_s": mu_s, "var": var}


def nap_score(cat, fit):
    """utils/metric.py:219-222 + utils/normalize.py:36-45,72-103:
    mean_j(((x-mu_r) V - mu_s)_j^2 / var_j)."""
    rot = ((cat.astype(_P.ft) - fit["mu_r"]) @ fit["v"]).astype(np.float64)
    st = (rot - fit["mu_s"]) / np.sqrt(fit["var"].astype(np.float64))
    return (st ** 2).mean(axis=1)


def auroc(score, label):
    """utils/metric.py:29-44 (sklearn roc_curve + auc) == Mann-Whitney U with
    ties counted one half."""
    score = np.asarray(score, dtype=np.float64)
    label = np.asarray(label).astype(bool)
    npos, nneg = int(label.sum()), int((~label).sum())
    if npos == 0 or nneg == 0:
        return 0.0
    order = np.argsort(score, kind="mergesort")
    s = score[order]
    ranks = np.empty(len(s), dtype=np.float64)
    i = 0
    while i < len(s):
        j = i
        while j + 1 < len(s) and s[j + 1] == s[i]:
            j += 1
        ranks[i:j + 1] = 0.5 * (i + j) + 1.0
        i = j + 1
    r = np.empty_like(ranks)
    r[order] = ranks
    u = r[label].sum() - npos * (npos + 1) / 2.0
    return float(u / (npos * nneg))


def f1_at_quantile(valid_score, test_score, test_label, q=0.90):
    """utils/metric.py:118-130 (quantile overridden to 0.90 at :120)."""
    thr = np.quantile(valid_score, q)
    pred = test_score > thr
    lab = np.asarray(test_label).astype(bool)
    tp = (pred & lab).sum()
    p = tp / float(pred.sum()) if pred.sum() else 0.0
    r = tp / float(lab.sum()) if lab.sum() else 0.0
    return (2 * p * r / (p + r) if (p + r) else 0.0), thr
