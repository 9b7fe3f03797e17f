"""get_diffs and the fused per-window scoring (reconstruction_aggregation.py:6-37
of the reference, plus the score reductions of utils/metric.py:133,167-171).

``get_diffs(x, model, batch_size)`` keeps the reference contract (a list of
n_enc+1 numpy arrays: d0 = x_hat - x, then d_l = enc_l(x_hat_{l-1}) -
enc_l(x_{l-1})), computed by one native call per batch (mmad_ae_score: the
encoder activations of x are reused from the AE forward instead of being
recomputed).  ``score_windows`` is the streaming form the scoring benchmark
uses: per-window squared-diff sums per layer, diffs never materialised.
"""
import numpy as np
import torch


def _device_of(model):
    return model._native.device


def get_diffs(x, model, batch_size=698):
    model.eval()
    if isinstance(x, np.ndarray):
        x = torch.tensor(x)
    dev = _device_of(model)
    widths = model._native.diff_widths()
    cuts = np.cumsum([0] + widths)
    out = [[] for _ in widths]
    with torch.no_grad():
        for xb in x.split(batch_size):
            xb = xb.to(dev).float().reshape(xb.shape[0], -1)
            _, diffs = model._native.score(xb, want_diffs=True)
            d = diffs.cpu().numpy()
            for i in range(len(widths)):
                out[i].append(d[:, cuts[i]:cuts[i + 1]])
    return [np.concatenate(o, axis=0) for o in out]


def score_windows(x, model, batch_size=16384, out=None):
    """Per-window sum of squared diffs per layer, [n_enc+1, N] fp32 on the
    device.  x: [N, D] tensor (any device; streamed in batches)."""
    model.eval()
    dev = _device_of(model)
    n = x.shape[0]
    nl = model._native.n_enc + 1
    if out is None:
        out = torch.empty((nl, n), device=dev)
    with torch.no_grad():
        for s in range(0, n, batch_size):
            xb = x[s:s + batch_size].to(dev, non_blocking=True)
            lsq, _ = model._native.score(xb)
            out[:, s:s + xb.shape[0]] = lsq
    return out


def base_from_layer_sq(layer_sq, widths):
    """utils/metric.py:133: mean_d(d0^2)."""
    return layer_sq[0] / float(widths[0])


def sap_from_layer_sq(layer_sq, widths, start_layer_index=0, end_layer_index=None):
    """utils/metric.py:155-171: mean of d^2 over the concatenated layers
    [start, end) with the reference's clamping."""
    n = len(widths)
    if end_layer_index is None:
        end_layer_index = n + 1
    if start_layer_index > n - 1:
        start_layer_index = n - 1
    if end_layer_index - start_layer_index < 1:
        end_layer_index = start_layer_index + 1
    sel = slice(start_layer_index, end_layer_index)
    return layer_sq[sel].sum(0) / float(sum(widths[sel]))
