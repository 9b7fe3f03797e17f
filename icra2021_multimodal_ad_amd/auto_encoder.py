"""AbstractModel / AutoEncoder -- the reference's model plugin surface
(models/abstract_model.py:20-40, models/auto_encoder.py:21-123) on top of the
native executor.

``AutoEncoder.step`` / ``validate`` keep the reference's static signatures
``(engine, mini_batch) -> (float,)`` with a duck-typed engine (``.model``,
``.optimizer``, ``.config.gpu_id``); the step runs the whole forward, sum-MSE,
backward and Adam update as HIP kernels (mmad_ae_train_fwd_bwd + mmad_ae_adam)
with no per-op Python dispatch.  ``forward`` runs the fused native forward and
is differentiable (mmad_ae_backward) for callers that build their own loss.
"""
from collections.abc import Iterable

import torch
import torch.nn as nn

from . import _native
from .engine import NativeAE


class AbstractModel(nn.Module):
    """models/abstract_model.py:20-40."""

    def __init__(self, *model_and_opts):
        super().__init__()
        for model_and_opt in model_and_opts:
            if not (model_and_opt is None or isinstance(model_and_opt, Iterable)):
                raise Exception("model_and_opt arg should be None or iterable objects")
        self.optimizer_list = []

    def forward(self):
        raise NotImplementedError

    def get_loss_value(self, x, y, *args, **kwargs):
        raise NotImplementedError

    def get_all_optimizers_state_dicts(self):
        return [opt.state_dict() for opt in self.optimizer_list]


class _AEFunction(torch.autograd.Function):
    """Differentiable fused forward: activations stay in the native workspace,
    backward runs the native backward sequence and returns parameter grads."""

    @staticmethod
    def forward(ctx, x, model, *params):
        nat = model._native
        xh, _ = nat.forward(x, train_bn=True)
        model._count_bn_step()
        ctx.model = model
        ctx.B = x.shape[0]
        ctx.gen = nat.gen
        return xh

    @staticmethod
    def backward(ctx, dxh):
        model = ctx.model
        nat = model._native
        if nat.gen != ctx.gen:
            # the saved activations live in the model's one workspace: any
            # native call since this forward (another forward, validate,
            # score, step) has overwritten them
            raise RuntimeError("AutoEncoder backward: the model ran another native pass after this "
                               "forward; call backward() before the next forward/validate/score")
        nat.backward(dxh.contiguous().float(), ctx.B)
        nat.gen += 1          # the backward consumed (and overwrote) the saved activations
        grads = [g.clone() for g in model._grad_views()]
        return (None, None, *grads)


# under data parallelism the status flag is exchanged every STATUS_EVERY calls
# (and at every epoch end, dist.DataParallel.epoch_end), not per step: the
# exchange is one more collective plus a host round trip on a sub-millisecond
# step.  A timed-out barrier only invalidates results -- every rank still
# issues the same collectives -- so deferring the check cannot hang a rank.
STATUS_EVERY = 16


def _check_status_all(model, force=False):
    """model._native.check_status() (a kernel barrier / split-K combine that
    timed out leaves that call's outputs unwritten).  Under data parallelism
    the failure is local to one GPU, so the flag is MAX-all-reduced and every
    rank raises together instead of one rank stopping alone; that exchange
    runs every STATUS_EVERY-th call (or when ``force``d), the same count on
    every rank."""
    d = getattr(model, "dist", None)
    if d is None or getattr(d, "world", 1) <= 1:
        model._native.check_status()
        return
    n = model.__dict__.get("_status_calls", 0) + 1
    model.__dict__["_status_calls"] = n
    if not force and n % STATUS_EVERY:
        return
    import torch.distributed as tdist
    err = None
    try:
        model._native.check_status()
    except Exception as e:   # noqa: BLE001 -- re-raised on every rank below
        err = e
    dev = "cuda" if tdist.get_backend(d.group) == "nccl" else "cpu"
    flag = torch.tensor([0.0 if err is None else 1.0], device=dev)
    tdist.all_reduce(flag, op=tdist.ReduceOp.MAX, group=d.group)
    if float(flag.item()) != 0.0:
        raise err if err is not None else _native.NativeError(
            "a kernel barrier timed out on another rank; this step's results are invalid")


class AutoEncoder(AbstractModel):
    """models/auto_encoder.py:21-123.

    Extra (build) arguments: ``dtype`` ('f32' exact parity path, 'bf16'
    throughput path), ``vib`` (encoder emits mu|logvar, decoder consumes a
    k-sample reparameterised z; SURVEY §8 a10/a10'), ``k``, ``beta_kl``."""

    def __init__(self, encoder, decoder, recon_loss, dtype="f32", vib=False, k=1, beta_kl=1.0):
        super().__init__()
        self.encoder = encoder
        self.decoder = decoder
        self.recon_loss = recon_loss
        self.vib = bool(vib)
        self.k = int(k)
        self.beta_kl = float(beta_kl)
        self.mmad_dtype = dtype
        dev = next(encoder.parameters()).device
        self._native = NativeAE(encoder.widths, decoder.widths, vib=vib, dtype=dtype, device=dev)
        self._nbt_pending = 0
        self._rng_offset = 0
        self.dist = None  # set by icra2021_multimodal_ad_amd.dist.attach_data_parallel
        self._adopt()
        self._native.version_fn = self._param_version

    # ------------------------------------------------------------ plumbing
    def _layers(self):
        return list(self.encoder.layer_list) + list(self.decoder.layer_list)

    def _adopt(self):
        """Copy the modules' current values into the flat native buffers and
        re-point every parameter / running buffer at a view of them."""
        nat = self._native
        with torch.no_grad():
            for l, layer in enumerate(self._layers()):
                w, b, g, be = nat.param_views(nat.params, l)
                w.copy_(layer.layer.weight)
                b.copy_(layer.layer.bias)
                if layer.bn is not None:
                    g.copy_(layer.bn.weight)
                    be.copy_(layer.bn.bias)
                    rm, rv = nat.running_views(l)
                    rm.copy_(layer.bn.running_mean)
                    rv.copy_(layer.bn.running_var)
        self._rebind()

    def _rebind(self):
        nat = self._native
        self.__dict__.pop("_plist_cache", None)
        for l, layer in enumerate(self._layers()):
            layer.mmad_dtype = self.mmad_dtype
            layer._flat = (nat, l)          # standalone layer calls use the padded buffers
            w, b, g, be = nat.param_views(nat.params, l)
            gw, gb, gg, gbe = nat.param_views(nat.grads, l)
            layer.layer.weight.data = w
            layer.layer.bias.data = b
            if layer.bn is not None:
                layer.bn.weight.data = g
                layer.bn.bias.data = be
                rm, rv = nat.running_views(l)
                layer.bn._buffers["running_mean"] = rm
                layer.bn._buffers["running_var"] = rv
                nbt = layer.bn.num_batches_tracked
                layer.bn._buffers["num_batches_tracked"] = nbt.to(nat.device)

    def _grad_views(self):
        nat = self._native
        out = []
        for l, layer in enumerate(self._layers()):
            w, b, g, be = nat.param_views(nat.grads, l)
            out += [w, b] + ([g, be] if layer.bn is not None else [])
        return out

    def _param_list(self):
        out = []
        for layer in self._layers():
            out += [layer.layer.weight, layer.layer.bias]
            if layer.bn is not None:
                out += [layer.bn.weight, layer.bn.bias]
        return out

    def _param_version(self):
        """Sum of the version counters the fp32 master can be written through
        (each nn.Parameter view has its own; the flat buffer has one more)."""
        plist = self.__dict__.get("_plist_cache")
        if plist is None:
            plist = self._param_list()
            self.__dict__["_plist_cache"] = plist
        return sum(p._version for p in plist) + self._native.params._version

    def _count_bn_step(self):
        self._nbt_pending += 1

    def _flush_counters(self):
        if self._nbt_pending:
            with torch.no_grad():
                for layer in self._layers():
                    if layer.bn is not None:
                        layer.bn.num_batches_tracked.add_(self._nbt_pending)
            self._nbt_pending = 0

    def _apply(self, fn, recurse=True):
        probe = fn(torch.zeros(1))
        if probe.dtype != torch.float32:
            raise NotImplementedError("the fp32 master parameters cannot change dtype; "
                                      "pick dtype='bf16' at construction for the bf16 path")
        self._flush_counters()
        self._native.to(probe.device)
        for layer in self._layers():
            if layer.bn is not None:
                layer.bn._buffers["num_batches_tracked"] = fn(layer.bn.num_batches_tracked)
        self._rebind()
        return self

    def state_dict(self, *args, **kwargs):
        """Reference key layout (60 keys for n_layers=5), contiguous copies.
        After sharded data-parallel steps the master weights are current only
        on their owning ranks: call ``model.dist.epoch_end(model)`` (or
        ``model._native.sync_master()``) on EVERY rank first -- doing it here
        would put a collective into a call one rank may make alone."""
        if getattr(self, "_native", None) is not None and self._native.master_stale:
            raise RuntimeError("state_dict: the master weights are sharded over the data-parallel "
                               "ranks; call model.dist.epoch_end(model) on every rank first")
        self._flush_counters()
        sd = super().state_dict(*args, **kwargs)
        if not kwargs.get("keep_vars", False):
            for k in list(sd.keys()):
                sd[k] = sd[k].detach().clone()
        return sd

    def load_state_dict(self, state_dict, strict=True, **kwargs):
        self._nbt_pending = 0
        res = super().load_state_dict(state_dict, strict=strict, **kwargs)
        # the bf16 weight shadow must follow the restored master at once
        self._native.sync_shadow(force=True)
        return res

    # ---------------------------------------------------- reference surface
    def encode(self, x):
        """models/auto_encoder.py:36-39."""
        z = self.encoder(x)
        return z.view(x.size(0), -1)

    def decode(self, z):
        """models/auto_encoder.py:41-44."""
        return self.decoder(z)

    def forward(self, x):
        """models/auto_encoder.py:46-50 (x_hat = dec(enc(x))) as one fused
        native pass; differentiable in train mode."""
        x2 = x.reshape(x.size(0), -1)
        if self.training and torch.is_grad_enabled():
            params = self._param_list()
            if any(p.requires_grad for p in params):
                if not self.vib:
                    return _AEFunction.apply(x2, self, *params).view(x.size(0), -1)
                # VIB-AE: layer by layer through the differentiable FCLayer /
                # reparameterisation ops; the reconstruction of the k samples
                # is averaged (k = 1: dec(z))
                out = self.encoder(x2, distribution="normal", k=self.k)
                xh = self.decoder(out["z"])
                return xh.mean(dim=0).view(x.size(0), -1)
        xh, _ = self._native.forward(x2, train_bn=self.training)
        if self.training:
            self._count_bn_step()
        return xh.view(x.size(0), -1)

    def get_loss_value(self, x, y, *args, **kwargs):
        """models/auto_encoder.py:52-55."""
        output = self(x)
        return self.recon_loss(output, x)

    # ------------------------------------------------------- fused training
    def train_step_async(self, x, optimizer=None, eps=None):
        """One AutoEncoder.step worth of work (train mode, fwd + sum-MSE +
        bwd [+ grad all-reduce] + Adam) with the loss left on the device."""
        if not self.training:
            self.train()
        nat = self._native
        # a step enters collectives whenever the executor holds a communicator
        # (whatever model.dist says) or the torch exchange is attached
        if getattr(nat, "_comm", None) is not None or (self.dist is not None and self.dist.world > 1):
            from .dist import assert_collective_context
            assert_collective_context("train_step_async with the data-parallel exchange attached")
        seed = 0x9E3779B97F4A7C15 & ((1 << 63) - 1)
        if self.dist is None or self.dist.native:
            # single process, or data parallel with the native RCCL exchange
            # (per-layer all-reduce + Adam inside the executor's step)
            lr, betas, aeps = self._adam_hyper(optimizer)
            loss = nat.train_step_fused(x, lr=lr, betas=betas, adam_eps=aeps, k=self.k, eps=eps,
                                        seed=seed, offset=self._rng_offset, beta_kl=self.beta_kl)
            self._rng_offset += 1
            self._count_bn_step()
            if optimizer is not None:
                self._mirror_optimizer_state(optimizer)
            return loss
        # torch exchange: the backward records per-layer dW events so that each
        # bucket's all-reduce + Adam starts while the lower layers still run
        lr, betas, aeps = self._adam_hyper(optimizer)
        if self.dist.overlapped and not getattr(nat, "_dw_events", False):
            nat.dw_events(True)
            nat._dw_events = True
        loss = nat.train_step(x, k=self.k, eps=eps, seed=seed, offset=self._rng_offset,
                              beta_kl=self.beta_kl)
        self._rng_offset += 1
        self._count_bn_step()
        self.dist.exchange_and_adam(nat, loss, lr, betas, aeps)
        if optimizer is not None:
            self._mirror_optimizer_state(optimizer)
        return loss

    @staticmethod
    def _adam_hyper(optimizer):
        lr, betas, eps = 1e-3, (0.9, 0.999), 1e-8
        if optimizer is not None:
            if not isinstance(optimizer, torch.optim.Adam):
                raise NotImplementedError("native step supports torch.optim.Adam "
                                          "(novelty_detection.py:90)")
            grp = optimizer.param_groups[0]
            if grp.get("weight_decay", 0) or grp.get("amsgrad", False) or grp.get("maximize", False):
                raise NotImplementedError("native Adam: weight_decay/amsgrad/maximize unsupported")
            lr, betas, eps = float(grp["lr"]), tuple(grp["betas"]), float(grp["eps"])
        return lr, betas, eps

    def _mirror_optimizer_state(self, optimizer):
        """Expose the native m/v as the torch optimizer's state (views)."""
        nat = self._native
        if getattr(optimizer, "_mmad_mirrored", None) is self:
            # every parameter's state shares one step tensor
            optimizer._mmad_step.fill_(float(nat.adam_step_count))
            return
        ms, vs = [], []
        for l, layer in enumerate(self._layers()):
            w, b, g, be = nat.param_views(nat.exp_avg, l)
            w2, b2, g2, be2 = nat.param_views(nat.exp_avg_sq, l)
            ms += [w, b] + ([g, be] if layer.bn is not None else [])
            vs += [w2, b2] + ([g2, be2] if layer.bn is not None else [])
        step = torch.tensor(float(nat.adam_step_count))
        for p, m, v in zip(self._param_list(), ms, vs):
            optimizer.state[p] = {"step": step, "exp_avg": m, "exp_avg_sq": v}
        optimizer._mmad_step = step
        optimizer._mmad_mirrored = self

    @staticmethod
    def step(engine, mini_batch):
        """models/auto_encoder.py:57-77."""
        model = engine.model
        model.train()
        x, _ = mini_batch
        if engine.config.gpu_id >= 0:
            x = x.cuda(engine.config.gpu_id)
        x = x.view(x.size(0), -1)
        loss = model.train_step_async(x, engine.optimizer)
        loss = float(loss)
        _check_status_all(model)
        return (loss,)

    @staticmethod
    def validate(engine, mini_batch):
        """models/auto_encoder.py:79-91 (eval mode, no grad, sum-MSE)."""
        model = engine.model
        model.eval()
        with torch.no_grad():
            x, _ = mini_batch
            if engine.config.gpu_id >= 0:
                x = x.cuda(engine.config.gpu_id)
            x = x.view(x.size(0), -1)
            _, loss = model._native.forward(x, train_bn=False, want_xhat=False, want_loss=True)
            if model.dist is not None:
                # data parallel: the whole batch's sum-MSE = sum of the shards'
                model.dist.all_reduce_sum(loss)
        loss = float(loss)
        _check_status_all(model)
        return (loss,)

    @staticmethod
    def attach(trainer, evaluator, config):
        """models/auto_encoder.py:93-123 with the build's ignite-free engine."""
        from .engine_loop import Events, RunningAverage
        RunningAverage(output_transform=lambda x: x[0]).attach(trainer, "recon")
        if getattr(config, "verbose", 0) >= 1:
            @trainer.on(Events.EPOCH_COMPLETED)
            def print_train_logs(engine):
                print("Epoch {} - loss={:.4e}".format(engine.state.epoch,
                                                      engine.state.metrics["recon"]))
        RunningAverage(output_transform=lambda x: x[0]).attach(evaluator, "recon")
        if getattr(config, "verbose", 0) >= 1:
            @evaluator.on(Events.EPOCH_COMPLETED)
            def print_valid_logs(engine):
                print("Validation - recon={:.4e} lowest_recon={:.4e}".format(
                    engine.state.metrics["recon"], engine.lowest_loss))
