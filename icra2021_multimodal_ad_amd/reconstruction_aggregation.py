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
    model._native.check_status()
    return [np.concatenate(o, axis=0) for o in out]


def score_windows(x, model, batch_size=65536, out=None, graph=True):
    """Per-window sum of squared diffs per layer, [n_enc+1, N] fp32 on the
    device.  x: [N, D] tensor.  Resident on the model's device: ONE native call
    for the whole pass (mmad_ae_score_stream), replayed as a captured hipGraph
    from the second call on (graph=True); elsewhere: streamed in batches."""
    model.eval()
    dev = _device_of(model)
    n = x.shape[0]
    nl = model._native.n_enc + 1
    if out is None:
        out = torch.empty((nl, n), device=dev)
    with torch.no_grad():
        if x.device == dev and x.dtype == torch.float32 and x.dim() == 2 and x.stride(1) == 1 \
                and out.stride(1) == 1:
            return model._native.score_stream(x, batch_size, out, graph=graph)
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


def nap_fit(x, device=None):
    """Rotater.fit + Standardizer.fit (utils/normalize.py:52-70, :25-34) of the
    NAP score on train diffs x [N, W] -> {'mu_r', 'v', 'mu_s', 'var'} (device
    fp32; v is [W, min(N, W)]) through mmad_nap_fit: fp64 Gram of the centred
    diffs + rocSOLVER eigensolve (V = right singular vectors, descending), fp32
    rotation with fp64 statistics."""
    from ._native import call, load, ptr, stream_ptr, require_gpu
    dev = torch.device(device) if device is not None else x.device
    x = torch.as_tensor(x).to(dev, torch.float32).contiguous()
    require_gpu(x)
    if x.dim() != 2 or x.shape[0] < 2:
        raise ValueError("NAP fit needs [N >= 2, W] train diffs, got %s" % (tuple(x.shape),))
    N, W = x.shape
    R = min(N, W)
    ws_b = int(load().mmad_nap_fit_ws_bytes(N, W))
    ws = torch.empty(ws_b, device=dev, dtype=torch.uint8)
    out = {"mu_r": torch.empty(W, device=dev), "v": torch.empty((W, R), device=dev),
           "mu_s": torch.empty(R, device=dev), "var": torch.empty(R, device=dev)}
    call("mmad_nap_fit", N, W, ptr(x), x.stride(0), ptr(out["mu_r"]), ptr(out["v"]),
         ptr(out["mu_s"]), ptr(out["var"]), ptr(ws), ws_b, stream_ptr())
    return out


class NapScorer:
    """NAP score (utils/metric.py:183-238 get_d_norm_loss with Rotater
    utils/normalize.py:47-103 and Standardizer :20-45).

    fit: the rotation (mu_r, V) from the SVD of the centred train diffs and the
    standardiser (mu_s, ddof=1 variance of the rotated train diffs), on the
    device through mmad_nap_fit (see nap_fit).
    run: ONE native GEMM per batch (mmad_nap_score): the concatenated diffs
    times V^T with the centring/standardising folded into a bias and a
    per-column weight, squared-mean reduced in the epilogue -- the rotated
    diffs are never materialised.  The run is always the exact-fp32 GEMM,
    whatever the model's dtype: the centring is folded in AFTER the product,
    and near-zero ``var`` columns (rank-deficient fits)
    multiply any rounding of (x V) by 1/var, which bf16 operands would turn
    into noise.
    """

    def __init__(self, model=None, start_layer_index=0, end_layer_index=None, widths=None,
                 device=None):
        import torch as _t
        if model is not None:
            widths = model._native.diff_widths()
            device = model._native.device
        if widths is None:
            raise ValueError("NapScorer needs a model or the diff widths")
        self.model = model
        self.device = _t.device(device) if device is not None else \
            _t.device("cuda", _t.cuda.current_device())
        n = len(widths)
        if end_layer_index is None:
            end_layer_index = n + 1
        if start_layer_index > n - 1:                  # utils/metric.py:197-202 clamping
            start_layer_index = n - 1
        if end_layer_index - start_layer_index < 1:
            end_layer_index = start_layer_index + 1
        self.sel = slice(start_layer_index, end_layer_index)
        cuts = np.cumsum([0] + list(widths))
        self.c0, self.c1 = int(cuts[self.sel.start]), int(cuts[min(self.sel.stop, n)])
        self.fit_state = None

    @classmethod
    def standalone(cls, width, device=None):
        """A scorer over already-concatenated [N, width] diffs."""
        return cls(widths=[int(width)], device=device)

    def _cat(self, diffs):
        if isinstance(diffs, (list, tuple)):
            parts = [torch.as_tensor(d) for d in diffs[self.sel]]
            return torch.cat([p.to(parts[0].device, torch.float32) for p in parts], dim=1)
        return torch.as_tensor(diffs)

    def fit(self, train_diffs=None, fit_state=None):
        """train_diffs: list of per-layer arrays (get_diffs) or [N, W]; or a
        ready fit_state {'mu_r','v','mu_s','var'} (e.g. the reference's)."""
        dev = self.device
        if fit_state is None:
            fit_state = nap_fit(self._cat(train_diffs), dev)
        fit_state = {k: torch.as_tensor(np.asarray(v) if not torch.is_tensor(v) else v).to(dev)
                     for k, v in fit_state.items()}
        self.fit_state = fit_state
        from ._native import pad
        W, R = fit_state["v"].shape
        Kp, Rp = pad(W), pad(R)
        vt = torch.zeros((Rp, Kp), device=dev, dtype=torch.float32)
        vt[:R, :W] = fit_state["v"].T.float()
        # (x - mu_r) V - mu_s = x V + bias, bias = -(mu_r V + mu_s)  (float64 fold)
        bias = torch.zeros(Rp, device=dev)
        bias[:R] = (-(fit_state["mu_r"].double() @ fit_state["v"].double())
                    - fit_state["mu_s"].double()).float()
        w = torch.zeros(Rp, device=dev)
        w[:R] = (1.0 / fit_state["var"].double()).float()
        self._dev = (W, R, Kp, Rp, vt, bias, w)
        return self

    def score(self, diffs):
        """diffs: list of per-layer arrays or [N, W] (host or device) -> [N]
        NAP scores (device fp32)."""
        from ._native import call, ptr, stream_ptr, pad, F32, require_gpu
        W, R, Kp, Rp, vt, bias, w = self._dev
        x = self._cat(diffs).to(self.device, torch.float32).contiguous()
        require_gpu(x)
        N = x.shape[0]
        assert x.shape[1] == W, (x.shape, W)
        Mp = pad(N)
        xp = torch.empty((Mp, Kp), device=self.device, dtype=torch.float32)
        dt = F32
        s = stream_ptr()
        call("mmad_pack_input", dt, N, W, Mp, Kp, ptr(x), x.stride(0), ptr(xp), s)
        rowsq = torch.empty((Rp // 128, Mp), device=self.device)
        out = torch.empty(N, device=self.device)
        call("mmad_nap_score", dt, N, W, R, Mp, Kp, Rp, ptr(xp), ptr(vt), ptr(bias), ptr(w),
             ptr(rowsq), ptr(out), s)
        return out
