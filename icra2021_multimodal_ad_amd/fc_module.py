"""FCLayer / FCModule / Activation / Loss / variational_info_bottleneck.

Mirrors the reference's module surface (names, constructor arguments, error
behaviour, ``layer_list``, state_dict keys) so callers are drop-in:

* Activation  -- modules/activation.py:20-45
* Loss        -- modules/loss.py:20-53
* FCLayer     -- layers/fc_layer.py:23-48 (Linear -> Activation -> BN, dropout)
* FCModule    -- modules/fc_module.py:23-61 (layer_list + registered ``net``)
* variational_info_bottleneck -- decorators/variational_info_bottleneck.py:19-42

Parameters are held in ``nn.Linear`` / ``nn.BatchNorm1d`` containers purely so
the state_dict layout is byte-for-byte the reference's; their torch
``forward`` is never called.  FCLayer.forward runs the fused HIP kernel
(``mmad_fc_fwd``: GEMM + bias + activation + BatchNorm) through the C-ABI;
there is no CPU / eager fallback.
"""
import torch
from torch import nn

from . import _native
from ._native import call, ptr, stream_ptr, pad

ACT_NAMES = ("sigmoid", "logsigmoid", "softmax", "logsoftmax", "tanh", "relu", "leakyrelu")
LEAKY_SLOPE = 0.2  # modules/activation.py:37-38


# MMAD_ACT_* (include/mmad.h)
ACT_ENUM = {None: 0, "leakyrelu": 1, "relu": 2, "sigmoid": 3, "tanh": 4, "logsigmoid": 5,
            "softmax": 6, "logsoftmax": 7}


class _ActivationFn(torch.autograd.Function):
    """Standalone activation on the device (mmad_activation_fwd / _bwd): the
    backward works from the saved OUTPUT (every supported form's derivative
    is a function of it)."""

    @staticmethod
    def forward(ctx, x, act):
        _native.require_gpu(x)
        shape, dtype = x.shape, x.dtype
        n = shape[-1] if x.dim() > 0 else 1
        x2 = x.reshape(-1, n).float().contiguous()
        y = torch.empty_like(x2)
        call("mmad_activation_fwd", act, LEAKY_SLOPE, x2.shape[0], n, ptr(x2), n, ptr(y), n,
             stream_ptr())
        ctx.save_for_backward(y)
        ctx.act, ctx.dtype = act, dtype
        return y.view(shape).to(dtype)

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        g2 = gy.reshape(y.shape).float().contiguous()
        dx = torch.empty_like(g2)
        n = y.shape[1]
        call("mmad_activation_bwd", ctx.act, LEAKY_SLOPE, y.shape[0], n, ptr(y), n, ptr(g2), n,
             ptr(dx), n, stream_ptr())
        return dx.view(gy.shape).to(ctx.dtype), None


class Activation(nn.Module):
    """modules/activation.py:20-45.  ``name`` selects the nonlinearity; unknown
    names (incl. None) are the identity.  Element-wise activations are fused
    into the FC kernel epilogue inside an FCLayer; called standalone, every
    form (softmax / logsoftmax over dim=-1 included) runs the native
    activation kernels, differentiably.  ``act`` keeps the torch module the
    reference holds (surface parity: printing, state); it is never called."""

    def __init__(self, act):
        super().__init__()
        self.name = act if act in ACT_NAMES else None
        if act == "sigmoid":
            self.act = nn.Sigmoid()
        elif act == "logsigmoid":
            self.act = nn.LogSigmoid()
        elif act == "softmax":
            self.act = nn.Softmax(dim=-1)
        elif act == "logsoftmax":
            self.act = nn.LogSoftmax(dim=-1)
        elif act == "tanh":
            self.act = nn.Tanh()
        elif act == "relu":
            self.act = nn.ReLU()
        elif act == "leakyrelu":
            self.act = nn.LeakyReLU(LEAKY_SLOPE)
        else:
            self.act = None

    @property
    def fusable(self):
        return self.name in (None, "leakyrelu", "relu", "sigmoid", "tanh")

    def forward(self, x):
        if self.act is None:
            return x
        return _ActivationFn.apply(x, ACT_ENUM[self.name])


class _MSEFn(torch.autograd.Function):
    """modules/loss.py:47-52 sum / mean reduction of (y_hat - y)^2 on the
    device (mmad_mse_loss: deterministic two-level reduction; backward
    mmad_mse_grad)."""

    @staticmethod
    def forward(ctx, y_hat, y, mean):
        _native.require_gpu(y_hat)
        a = y_hat.detach().float().contiguous()
        b = y.detach().to(a.device).float().contiguous()
        if a.shape != b.shape:
            raise ValueError(f"mse: y_hat {tuple(a.shape)} and y {tuple(b.shape)} differ")
        out = torch.empty((), device=a.device, dtype=torch.float32)
        work = torch.empty(int(_native.load().mmad_mse_loss_ws_floats()), device=a.device)
        call("mmad_mse_loss", a.numel(), ptr(a), ptr(b), 1 if mean else 0, ptr(out), ptr(work),
             stream_ptr())
        ctx.save_for_backward(a, b)
        ctx.mean = mean
        ctx.dtypes = (y_hat.dtype, y.dtype)
        return out.to(y_hat.dtype)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.detach().float().reshape(1).contiguous()
        need_a, need_b = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        da = torch.empty_like(a) if need_a else None
        db = torch.empty_like(b) if need_b else None
        if need_a or need_b:
            call("mmad_mse_grad", a.numel(), ptr(a), ptr(b), ptr(g), 1 if ctx.mean else 0, ptr(da),
                 ptr(db), stream_ptr())
        return (da.to(ctx.dtypes[0]) if da is not None else None,
                db.to(ctx.dtypes[1]) if db is not None else None, None)


class Loss(nn.Module):
    """modules/loss.py:20-53 (same names/reductions).  The AE's
    ``Loss('mse', reduction='sum')`` is fused into the last decoder GEMM by the
    native train step; called on its own the MSE (sum / mean) runs the native
    mmad_mse_loss / mmad_mse_grad (differentiable); the other criteria, which
    the autoencoder path never uses, are torch's modules as in the reference."""

    def __init__(self, loss, weight=None, reduction="sum"):
        self.reduction = reduction
        super().__init__()
        self.name = loss
        if loss == "bce":
            self.loss = nn.BCELoss(weight=weight, reduction=reduction)
        elif loss == "bce_with_logit":
            self.loss = nn.BCEWithLogitsLoss(weight=weight, reduction=reduction)
        elif loss == "mse":
            self.loss = nn.MSELoss(reduction=reduction)
        elif loss == "l1":
            self.loss = nn.L1Loss(reduction=reduction)
        elif loss == "ce":
            self.loss = nn.CrossEntropyLoss(weight=weight, reduction=reduction)
        elif loss == "nll":
            self.loss = nn.NLLLoss(weight=weight, reduction=reduction)
        else:
            self.loss = None

    def is_classification_task(self):
        return isinstance(self.loss, (nn.NLLLoss, nn.CrossEntropyLoss))

    def forward(self, y_hat, y):
        if self.loss is not None:
            if self.is_classification_task():
                y = y.long()
            if self.name == "mse" and self.reduction in ("sum", "mean"):
                return _MSEFn.apply(y_hat, y, self.reduction == "mean")
            return self.loss(y_hat, y)
        return y_hat.mean()


class FCLayer(nn.Module):
    """layers/fc_layer.py:23-48: y = BN(act(x W^T + b)) [-> dropout].

    forward runs the fused HIP layer (mmad_fc_fwd [+ mmad_bn_train_apply]) and
    is differentiable: backward is mmad_bn_act_bwd / mmad_act_bwd +
    mmad_fc_bwd_weight + mmad_fc_bwd_data.  Inside an AutoEncoder the packed
    operands are the executor's own padded buffers (no copy); a standalone
    layer packs W/b once per parameter version."""

    def __init__(self, input_size, output_size=1, bias=True, act="relu", bn=False, dropout_p=0):
        super().__init__()
        self.layer = nn.Linear(input_size, output_size, bias)
        self.bn = nn.BatchNorm1d(output_size) if bn else None
        self.dropout = nn.Dropout(dropout_p) if dropout_p else None
        self.act = Activation(act) if act else None
        self.mmad_dtype = "f32"
        self._flat = None        # (NativeAE, layer index) when owned by an AutoEncoder
        self._pack = None        # standalone: (key, w_packed, b_packed, g_packed, be_packed)

    @property
    def act_name(self):
        return self.act.name if self.act is not None else None

    def forward(self, x):
        if self.dropout is not None or (self.act is not None and not self.act.fusable) \
                or self.layer.bias is None:
            raise NotImplementedError("FCLayer HIP path supports bias=True, element-wise "
                                      "activations and no dropout (the AE configuration)")
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        params = [self.layer.weight, self.layer.bias]
        if self.bn is not None:
            params += [self.bn.weight, self.bn.bias]
        if torch.is_grad_enabled() and (x2.requires_grad or any(p.requires_grad for p in params)):
            y = _FCLayerFn.apply(x2, self, self.training, *params)
        else:
            y = fc_layer_forward(self, x2, self.training)[0]
        return y.reshape(*shape[:-1], y.shape[-1])

    # packed operands -------------------------------------------------------
    def packed(self, dev, dt):
        """(w [Np][Kp] dtype, bias [Np], gamma [Np] | None, beta [Np] | None) fp32
        padded device buffers holding the current parameter values."""
        if self._flat is not None:
            nat, l = self._flat
            L = nat.layers[l]
            nat.sync_shadow()
            wsrc = nat.shadow if dt == _native.BF16 else nat.params
            w = wsrc[L["w_off"]: L["w_off"] + L["Np"] * L["Kp"]]
            b = nat.params[L["b_off"]: L["b_off"] + L["Np"]]
            g = nat.params[L["g_off"]: L["g_off"] + L["Np"]] if L["bn"] else None
            be = nat.params[L["be_off"]: L["be_off"] + L["Np"]] if L["bn"] else None
            return w, b, g, be
        lin, bn = self.layer, self.bn
        src = [lin.weight, lin.bias] + ([bn.weight, bn.bias] if bn is not None else [])
        key = (dt, str(dev)) + tuple((p._version, p.data_ptr()) for p in src)
        if self._pack is None or self._pack[0] != key:
            N, K = lin.out_features, lin.in_features
            Np, Kp = pad(N), pad(K)
            tdt = torch.bfloat16 if dt == _native.BF16 else torch.float32
            with torch.no_grad():
                w = torch.zeros((Np, Kp), device=dev, dtype=tdt)
                w[:N, :K] = lin.weight.detach()
                vecs = []
                for p in src[1:]:
                    v = torch.zeros(Np, device=dev)
                    v[:N] = p.detach()
                    vecs.append(v)
            self._pack = (key, w, vecs[0], vecs[1] if bn is not None else None,
                          vecs[2] if bn is not None else None)
        return self._pack[1:]


def fc_layer_forward(layer, x2, training):
    """Run one FCLayer through ``mmad_fc_fwd`` (+ ``mmad_bn_train_apply`` in
    train mode, which also updates the running statistics in place).  Returns
    (y [M, N] fp32, saved) with saved = what the backward needs."""
    _native.require_gpu(x2)
    lin, bn = layer.layer, layer.bn
    dev = x2.device
    dt = _native.BF16 if layer.mmad_dtype == "bf16" else _native.F32
    tdt = torch.bfloat16 if dt == _native.BF16 else torch.float32
    M, K = x2.shape
    N = lin.out_features
    Mp, Kp, Np = pad(M), pad(K), pad(N)
    x2 = x2.detach().float().contiguous()
    s = stream_ptr()
    xin = torch.empty((Mp, Kp), device=dev, dtype=tdt)
    call("mmad_pack_input", dt, M, K, Mp, Kp, ptr(x2), K, ptr(xin), s)
    w, b, g, be = layer.packed(dev, dt)
    out = torch.empty((Mp, Np), device=dev, dtype=tdt)
    act = _native.ACT[layer.act_name]
    saved = dict(dt=dt, M=M, N=N, K=K, Mp=Mp, Np=Np, Kp=Kp, xin=xin, w=w, g=g, act=act,
                 bn_train=False, bn_eval=False)
    if bn is None:
        call("mmad_fc_fwd", dt, M, N, K, Mp, Np, Kp, ptr(xin), ptr(w), ptr(b), act,
             LEAKY_SLOPE, None, None, ptr(out), None, s)
        saved["a"] = out
    elif training:
        stats = torch.empty((Mp // 32, 2, Np), device=dev)
        a = torch.empty((Mp, Np), device=dev, dtype=tdt)
        call("mmad_fc_fwd", dt, M, N, K, Mp, Np, Kp, ptr(xin), ptr(w), ptr(b), act,
             LEAKY_SLOPE, None, None, ptr(a), ptr(stats), s)
        sm = torch.empty(Np, device=dev)
        sr = torch.empty(Np, device=dev)
        # running statistics are updated in place (valid columns only)
        call("mmad_bn_train_apply", dt, M, N, Mp, Np, ptr(a), ptr(stats), ptr(g), ptr(be),
             ptr(bn.running_mean), ptr(bn.running_var), float(bn.momentum), float(bn.eps), ptr(sm),
             ptr(sr), ptr(out), s)
        with torch.no_grad():
            bn.num_batches_tracked.add_(1)
        saved.update(a=a, sm=sm, sr=sr, bn_train=True)
    else:
        sc = torch.empty(Np, device=dev)
        sh = torch.empty(Np, device=dev)
        rm = torch.zeros(Np, device=dev)
        rv = torch.ones(Np, device=dev)
        rm[:N] = bn.running_mean
        rv[:N] = bn.running_var
        call("mmad_bn_eval_affine", N, Np, ptr(g), ptr(be), ptr(rm), ptr(rv), float(bn.eps),
             ptr(sc), ptr(sh), s)
        call("mmad_fc_fwd", dt, M, N, K, Mp, Np, Kp, ptr(xin), ptr(w), ptr(b), act,
             LEAKY_SLOPE, ptr(sc), ptr(sh), ptr(out), None, s)
        saved["bn_eval"] = True
    y = torch.empty((M, N), device=dev)
    call("mmad_unpack_output", dt, M, N, Np, ptr(out), ptr(y), N, s)
    return y, saved


class _FCLayerFn(torch.autograd.Function):
    """Autograd of FCLayer (layers/fc_layer.py:37-48) on the native kernels."""

    @staticmethod
    def forward(ctx, x2, layer, training, *params):
        y, saved = fc_layer_forward(layer, x2, training)
        ctx.saved = saved
        ctx.n_params = len(params)
        return y

    @staticmethod
    def backward(ctx, dy):
        sv = ctx.saved
        if sv["bn_eval"]:
            raise NotImplementedError("FCLayer backward through eval-mode BatchNorm is not supported "
                                      "on the HIP path (train() the layer to differentiate it)")
        dt, M, N, K, Mp, Np, Kp = sv["dt"], sv["M"], sv["N"], sv["K"], sv["Mp"], sv["Np"], sv["Kp"]
        dev = dy.device
        tdt = torch.bfloat16 if dt == _native.BF16 else torch.float32
        s = stream_ptr()
        dy = dy.detach().float().contiguous()
        dyp = torch.empty((Mp, Np), device=dev, dtype=tdt)
        call("mmad_pack_input", dt, M, N, Mp, Np, ptr(dy), N, ptr(dyp), s)
        dz = torch.empty((Mp, Np), device=dev, dtype=tdt)
        dbpart = torch.empty((Mp // 128, Np), device=dev)
        dgamma = dbeta = None
        if sv["bn_train"]:
            dgamma = torch.empty(Np, device=dev)
            dbeta = torch.empty(Np, device=dev)
            ws = torch.empty(int(_native.load().mmad_bn_act_bwd_ws(Mp, Np)), dtype=torch.uint8, device=dev)
            call("mmad_bn_act_bwd", dt, sv["act"], LEAKY_SLOPE, M, N, Mp, Np, ptr(dyp), ptr(sv["a"]),
                 ptr(sv["sm"]), ptr(sv["sr"]), ptr(sv["g"]), ptr(dz), ptr(dgamma), ptr(dbeta),
                 ptr(dbpart), ptr(ws), s)
        else:
            call("mmad_act_bwd", dt, sv["act"], LEAKY_SLOPE, M, Mp, Np, ptr(dyp), ptr(sv["a"]), ptr(dz),
                 ptr(dbpart), s)
        db = torch.empty(Np, device=dev)
        call("mmad_colsum", Mp // 128, N, Np, ptr(dbpart), Np, 1.0, ptr(db), s)
        dw = torch.empty((Np, Kp), device=dev)
        call("mmad_fc_bwd_weight", dt, Mp, Np, Kp, ptr(dz), ptr(sv["xin"]), ptr(dw), s)
        dxp = torch.empty((Mp, Kp), device=dev, dtype=tdt)
        call("mmad_fc_bwd_data", dt, M, N, K, Mp, Np, Kp, ptr(dz), ptr(sv["w"]), ptr(dxp), None, s)
        dx = torch.empty((M, K), device=dev)
        call("mmad_unpack_output", dt, M, K, Kp, ptr(dxp), ptr(dx), K, s)
        grads = [dw[:N, :K], db[:N]]
        if ctx.n_params == 4:
            grads += [dgamma[:N], dbeta[:N]]
        return (dx, None, None, *grads)


class _ReparamFn(torch.autograd.Function):
    """decorators/variational_info_bottleneck.py:22-26,37 with its autograd:
    dmu = sum_k dz, dlogvar = 1/2 sigma sum_k dz eps (mmad_vib_reparam_bwd)."""

    @staticmethod
    def forward(ctx, mu, logvar, k, det, eps, seed):
        _native.require_gpu(mu)
        B, btl = mu.shape
        dev = mu.device
        enc = torch.cat([mu.detach(), logvar.detach()], dim=-1).float().contiguous()
        Mpz, Kpz = pad(k * B), pad(btl)
        z = torch.empty((Mpz, Kpz), device=dev)
        eps_used = torch.empty((k, B, btl), device=dev)
        if eps is not None:
            eps = eps.float().contiguous()
        call("mmad_vib_reparam_fwd", _native.F32, B, btl, k, ptr(enc), 2 * btl, ptr(eps),
             ptr(eps_used) if not det else None, int(seed), 0, int(det), ptr(z), Kpz, None, stream_ptr())
        if det:
            eps_used.zero_()              # z = mu: no noise term in the gradient
        ctx.save_for_backward(enc, eps_used)
        ctx.k, ctx.B, ctx.btl = k, B, btl
        return z[:k * B, :btl].reshape(k, B, btl)

    @staticmethod
    def backward(ctx, dz):
        enc, eps_used = ctx.saved_tensors
        k, B, btl = ctx.k, ctx.B, ctx.btl
        dz = dz.detach().float().contiguous().reshape(k * B, btl)
        denc = torch.empty((pad(B), 2 * btl), device=dz.device)
        call("mmad_vib_reparam_bwd", _native.F32, B, btl, k, ptr(enc), 2 * btl, ptr(eps_used), ptr(dz),
             btl, 0.0, ptr(denc), 2 * btl, None, stream_ptr())
        return denc[:B, :btl], denc[:B, btl:], None, None, None, None


def reparameterize(mu, logvar, k, stochastic_inference, eps=None, seed=None):
    """decorators/variational_info_bottleneck.py:22-26,37 on the GPU through
    ``mmad_vib_reparam_fwd`` (differentiable via ``mmad_vib_reparam_bwd``):
    z[k,B,btl] = eps*exp(0.5*logvar) + mu, or mu expanded when grad is
    disabled and stochastic_inference is False."""
    det = not (torch.is_grad_enabled() or stochastic_inference)
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    return _ReparamFn.apply(mu, logvar, int(k), det, eps, seed)


def variational_info_bottleneck(forward_fn):
    """decorators/variational_info_bottleneck.py:19-42: distribution=None ->
    pass-through; 'normal' -> split mu|logvar, reparameterise k samples."""
    def decorated_forward(self, x, distribution=None, k=1, stochastic_inference=True, eps=None):
        output = forward_fn(self, x)
        if distribution is None:
            return output
        elif distribution == "normal":
            mu, logvar = output.split(output.size(-1) // 2, dim=-1)
            if k < 1:
                raise ValueError("k should be >= 1")
            z = reparameterize(mu, logvar, k, stochastic_inference, eps=eps)
            return {"z": z, "mu": mu, "logvar": logvar}
        else:
            raise NotImplementedError(
                "Wrong distribution for information bottleneck: {}".format(distribution))
    return decorated_forward


vib = variational_info_bottleneck


class FCModule(nn.Module):
    """modules/fc_module.py:23-61."""

    def __init__(self, input_size, output_size, hidden_sizes=None, use_batch_norm=True,
                 dropout_p=0, act="leakyrelu", last_act=None):
        super().__init__()
        self.layer_list = []
        if use_batch_norm and dropout_p > 0:
            raise Exception("Either batch_norm or dropout is allowed, not both")
        hidden_sizes = list(hidden_sizes or [])
        layer_sizes = [input_size] + hidden_sizes + [output_size]
        for idx, (in_size, out_size) in enumerate(zip(layer_sizes[:-1], layer_sizes[1:])):
            if idx < len(hidden_sizes):
                layer = FCLayer(input_size=in_size, output_size=out_size, act=act,
                                bn=use_batch_norm, dropout_p=dropout_p)
            else:
                layer = FCLayer(input_size=in_size, output_size=out_size, act=last_act)
            self.layer_list.append(layer)
        self.net = nn.Sequential(*self.layer_list)

    @property
    def widths(self):
        return [self.layer_list[0].layer.in_features] + [l.layer.out_features for l in self.layer_list]

    @vib
    def forward(self, x):
        return self.net(x)
