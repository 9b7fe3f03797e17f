"""NativeAE: owner of the device buffers of one autoencoder and the handle of
the native executor (``mmad_ae_*`` in include/mmad.h).

Memory layout (DESIGN.md "Data layout in HBM"): one flat fp32 parameter
buffer (all weights [Np][Kp] first, then per-layer bias/gamma/beta, every
dimension zero-padded to 128), same-shaped flat grads and Adam m/v, a bf16
shadow of the weight region for the bf16 path, and a [2][n_bn] running-stat
buffer.  The reference-shaped ``nn.Parameter``s of the plugin surface are
strided views into these buffers, so ``state_dict`` / ``load_state_dict`` /
``torch.optim`` all see the same memory the kernels use.
"""
import ctypes

import torch

from . import _native
from ._native import call, ptr, stream_ptr

DTYPES = {"f32": _native.F32, "fp32": _native.F32, "float32": _native.F32,
          "bf16": _native.BF16, "bfloat16": _native.BF16}


class NativeAE:
    def __init__(self, enc_widths, dec_widths, vib=False, dtype="bf16", device=None,
                 slope=0.2, bn_eps=1e-5, bn_momentum=0.1):
        lib = _native.load()
        self.dtype_name = "bf16" if DTYPES[dtype] == _native.BF16 else "f32"
        self.dt = DTYPES[dtype]
        self.enc_widths = [int(w) for w in enc_widths]
        self.dec_widths = [int(w) for w in dec_widths]
        self.vib = bool(vib)
        self.n_enc, self.n_dec = len(enc_widths) - 1, len(dec_widths) - 1
        self.btl = self.dec_widths[0]
        self.bn_eps, self.bn_momentum = bn_eps, bn_momentum
        h = ctypes.c_void_p()
        ea = (ctypes.c_int * len(enc_widths))(*self.enc_widths)
        da = (ctypes.c_int * len(dec_widths))(*self.dec_widths)
        call("mmad_ae_create", ctypes.byref(h), self.dt, self.n_enc, ea, self.n_dec, da,
             int(self.vib), float(slope), float(bn_eps), float(bn_momentum))
        self._h = h
        self._lib = lib
        n_l = self.n_enc + self.n_dec
        info = (ctypes.c_int64 * (7 * n_l))()
        tot = (ctypes.c_int64 * 4)()
        call("mmad_ae_layout", h, info, tot)
        self.n_params, self.n_weight, self.n_bn = int(tot[0]), int(tot[1]), int(tot[2])
        widths = [(self.enc_widths[i], self.enc_widths[i + 1], True) for i in range(self.n_enc)] + \
                 [(self.dec_widths[i], self.dec_widths[i + 1], False) for i in range(self.n_dec)]
        self.layers = []
        for i, (k, n, enc) in enumerate(widths):
            r = [int(v) for v in info[7 * i: 7 * i + 7]]
            self.layers.append(dict(K=k, N=n, enc=enc, w_off=r[0], b_off=r[1], g_off=r[2],
                                    be_off=r[3], Kp=r[4], Np=r[5], bn_off=r[6], bn=r[2] >= 0))
        device = torch.device(device) if device is not None else torch.device("cpu")
        self.device = device
        self._alloc(device)
        self._ws = None
        self._synced_version = None
        # version of the fp32 master as the plugin surface sees it: the
        # reference-shaped nn.Parameters are views with their OWN version
        # counters (load_state_dict / a torch optimizer bump those, not
        # params._version), so the owner installs a callable summing them
        self.version_fn = None
        # bumped by every native call that rewrites the workspace; a
        # differentiable forward records it and its backward checks it
        self.gen = 0
        self.adam_step_count = 0
        self.use_graph = bool(_native.SCHEDULE["train_graph"])

    # ------------------------------------------------------------------ memory
    def _alloc(self, device, src=None):
        kw = dict(device=device, dtype=torch.float32)
        self.params = torch.zeros(self.n_params, **kw)
        self.grads = torch.zeros(self.n_params, **kw)
        self.exp_avg = torch.zeros(self.n_params, **kw)
        self.exp_avg_sq = torch.zeros(self.n_params, **kw)
        self.running = torch.zeros(2 * self.n_bn, **kw)
        self.running[self.n_bn:] = 1.0
        # bf16: two weight shadows (mmad_ae_set_shadow_pair), ping-ponged by
        # the fused step on large calls (the executor picks per call: knob
        # pair_rows); _native.SCHEDULE["shadow_pair"] = False keeps one
        self._pair = self.dt == _native.BF16 and bool(_native.SCHEDULE["shadow_pair"])
        self._shadow_buf = (torch.zeros((2 if self._pair else 1) * self.n_weight, device=device,
                                        dtype=torch.bfloat16)
                            if self.dt == _native.BF16 else None)
        if src is not None:
            for name in ("params", "grads", "exp_avg", "exp_avg_sq", "running"):
                getattr(self, name).copy_(getattr(src, name))
        self._bind()

    def _bind(self):
        self._synced_version = None
        if self.device.type != "cuda":
            return
        sb = self._shadow_buf
        call("mmad_ae_bind", self._h, ptr(self.params), ptr(self.grads), ptr(self.exp_avg),
             ptr(self.exp_avg_sq), ptr(sb[: self.n_weight] if sb is not None else None),
             ptr(self.running))
        if self._pair:
            call("mmad_ae_set_shadow_pair", self._h, ptr(sb[self.n_weight:]))
        if getattr(self, "_grad_bf16", None) is not None:
            # the bf16 exchange scratch follows the buffers to their new device
            self.set_grad_bf16(True)

    @property
    def shadow(self):
        """The bf16 weight shadow the kernels read next (None for fp32)."""
        sb = self._shadow_buf
        if sb is None:
            return None
        if not self._pair or self.device.type != "cuda":
            return sb[: self.n_weight]
        cur = self._lib.mmad_ae_current_shadow(self._h) or 0
        return sb[self.n_weight:] if cur != sb.data_ptr() else sb[: self.n_weight]

    def to(self, device):
        device = torch.device(device)
        if device == self.device:
            return self
        old = _Snapshot(self)
        self.device = device
        self._alloc(device, src=old)
        self._ws = None
        self._dw_streams = None   # the torch exchange's bucket streams belong to the old device
        return self

    def set_comm(self, comm):
        """Attach a dist.NativeComm (or None): mmad_ae_train_step then exchanges
        the weight gradients in buckets of consecutive layers (tune knob
        dp_bucket_mib) on the executor's comm stream before their Adam
        (sharded: reduce-scatter, Adam on this rank's 1/N, all-gather).
        Detaching first all-gathers the sharded master weights / Adam moments
        (sync_master: collective, so detach on every rank at the same point)."""
        if comm is None and getattr(self, "_comm", None) is not None:
            self.sync_master()
        self._comm = comm        # keep the communicator alive as long as the handle uses it
        call("mmad_ae_set_comm", self._h, comm.handle if comm is not None else None)

    def set_grad_bf16(self, on=True):
        """Optional bf16 gradient exchange of the sharded DP buckets
        (mmad_ae_set_grad_bf16): this object owns the bf16 scratch buffer."""
        self._grad_bf16 = (torch.empty(self.n_weight, device=self.device, dtype=torch.bfloat16)
                           if on else None)
        call("mmad_ae_set_grad_bf16", self._h, ptr(self._grad_bf16))

    @property
    def master_stale(self):
        """True while the sharded DP step has left the fp32 master weights (bf16
        model) / the Adam moments current only on their owning rank."""
        return bool(self._lib.mmad_ae_dp_master_stale(self._h))

    def sync_master(self):
        """All-gather the shards of the master weights and Adam moments after
        sharded DP steps (collective: every rank, same point; a no-op when
        nothing is stale)."""
        if self.master_stale:
            call("mmad_ae_dp_sync_master", self._h, stream_ptr())

    def __del__(self):
        try:
            if getattr(self, "_h", None) is not None:
                self._lib.mmad_ae_destroy(self._h)
                self._h = None
        except Exception:
            pass

    # ---------------------------------------------------------------- views
    def _vec(self, buf, off, n):
        return buf[off: off + n]

    def weight_view(self, buf, l):
        L = self.layers[l]
        return buf[L["w_off"]: L["w_off"] + L["Np"] * L["Kp"]].view(L["Np"], L["Kp"])[:L["N"], :L["K"]]

    def param_views(self, buf, l):
        """Reference-shaped views of layer ``l`` in flat buffer ``buf``:
        (weight[N,K], bias[N], gamma[N] | None, beta[N] | None)."""
        L = self.layers[l]
        w = self.weight_view(buf, l)
        b = self._vec(buf, L["b_off"], L["N"])
        g = self._vec(buf, L["g_off"], L["N"]) if L["bn"] else None
        be = self._vec(buf, L["be_off"], L["N"]) if L["bn"] else None
        return w, b, g, be

    def running_views(self, l):
        L = self.layers[l]
        if not L["bn"]:
            return None, None
        o, n = L["bn_off"], L["N"]
        return self.running[o: o + n], self.running[self.n_bn + o: self.n_bn + o + n]

    # -------------------------------------------------------------- helpers
    def _require(self, x):
        _native.require_gpu(x)
        if self.device.type != "cuda":
            raise _native.NativeUnavailable("model buffers are on the CPU; call .cuda() first")

    def master_version(self):
        return self.version_fn() if self.version_fn is not None else self.params._version

    def sync_shadow(self, force=False):
        """Refresh the bf16 weight shadow if the fp32 master was written by
        anything other than the native Adam (load_state_dict, torch optim)."""
        if self.shadow is None or self.device.type != "cuda":
            return
        v = self.master_version()
        if force or v != self._synced_version:
            call("mmad_ae_sync_shadow", self._h, stream_ptr())
            self._synced_version = v

    def _mark_synced(self):
        """The native Adam just wrote the master AND the shadow."""
        if self.shadow is not None:
            self._synced_version = self.master_version()

    def check_status(self):
        """Raise NativeError if a split-K GEMM combine of the calls since the
        last check timed out (a no-op unless split-K is enabled)."""
        if self._ws is None or self.device.type != "cuda":
            return
        base = self._ws.data_ptr()
        aligned = (base + 255) // 256 * 256
        call("mmad_ae_status", self._h, ctypes.c_void_p(aligned), self._ws.numel() - (aligned - base),
             stream_ptr())

    def workspace(self, B, k=1):
        need = int(self._lib.mmad_ae_workspace_bytes(self._h, int(B), int(k)))
        if need < 0:
            raise _native.NativeError("workspace size query failed")
        if self._ws is None or self._ws.numel() < need:
            # zeroed: the split-K control words must start at zero
            self._ws = torch.zeros(need + 256, dtype=torch.uint8, device=self.device)
        base = self._ws.data_ptr()
        aligned = (base + 255) // 256 * 256
        return ctypes.c_void_p(aligned), need

    @staticmethod
    def _as_input(x, width):
        x = x.reshape(x.shape[0], -1)
        if x.dtype != torch.float32:
            x = x.float()
        if x.stride(-1) != 1:
            x = x.contiguous()
        if x.shape[1] != width:
            raise ValueError(f"input width {x.shape[1]} != model input size {width}")
        return x

    # ----------------------------------------------------------------- ops
    def train_step(self, x, k=1, eps=None, seed=0, offset=0, beta_kl=0.0, loss_out=None):
        """AutoEncoder.step forward+backward: grads into self.grads; returns the
        device loss tensor [1] (no host sync)."""
        self._require(x)
        x = self._as_input(x, self.enc_widths[0])
        B = x.shape[0]
        self.sync_shadow()
        ws, nb = self.workspace(B, k)
        if loss_out is None:
            loss_out = torch.empty(1, device=self.device, dtype=torch.float32)
        if eps is not None:
            eps = eps.contiguous().float()
            assert eps.numel() == k * B * self.btl
        self.gen += 1
        call("mmad_ae_train_fwd_bwd", self._h, ptr(x), x.stride(0), B, int(k), ptr(eps),
             int(seed), int(offset), float(beta_kl), ptr(loss_out), ws, nb, stream_ptr())
        return loss_out

    def train_step_fused(self, x, lr=1e-3, betas=(0.9, 0.999), adam_eps=1e-8, k=1, eps=None,
                         seed=0, offset=0, beta_kl=0.0, loss_out=None):
        """Whole step with per-layer Adam overlapped on the side stream
        (mmad_ae_train_step); returns the device loss tensor [1]."""
        self._require(x)
        x = self._as_input(x, self.enc_widths[0])
        B = x.shape[0]
        self.sync_shadow()
        ws, nb = self.workspace(B, k)
        if loss_out is None:
            loss_out = torch.empty(1, device=self.device, dtype=torch.float32)
        if eps is not None:
            eps = eps.contiguous().float()
            assert eps.numel() == k * B * self.btl
        self.adam_step_count += 1
        self.gen += 1
        # eager multi-stream schedule by default.  SCHEDULE["train_graph"] replays
        # one captured hipGraph per step instead (mmad_ae_train_step_graph);
        # measured slower on ROCm 7 (profiles/r02e_host.log: host 377 vs 325
        # us/step, GPU 675 vs 524 us/step at C2), so it stays opt-in
        fn = "mmad_ae_train_step_graph" if self.use_graph else "mmad_ae_train_step"
        call(fn, self._h, ptr(x), x.stride(0), B, int(k), ptr(eps), int(seed),
             int(offset), float(beta_kl), float(lr), float(betas[0]), float(betas[1]),
             float(adam_eps), int(self.adam_step_count), ptr(loss_out), ws, nb, stream_ptr())
        self._mark_synced()
        return loss_out

    def backward(self, dxh, B):
        """loss.backward() after forward(train_bn=True) on the same workspace."""
        self._require(dxh)
        ws, nb = self.workspace(B, 1)
        call("mmad_ae_backward", self._h, ptr(dxh), dxh.stride(0), int(B), ws, nb, stream_ptr())

    def adam(self, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, step=None):
        if step is None:
            self.adam_step_count += 1
            step = self.adam_step_count
        call("mmad_ae_adam", self._h, float(lr), float(betas[0]), float(betas[1]), float(eps),
             int(step), stream_ptr())
        self._mark_synced()

    def adam_range(self, off, n, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, step=1):
        """Adam on the parameter range [off, off + n) (mmad_ae_adam_range) on
        the current stream; the caller counts the step."""
        call("mmad_ae_adam_range", self._h, float(lr), float(betas[0]), float(betas[1]), float(eps),
             int(step), int(off), int(n), stream_ptr())

    def dw_events(self, on=True):
        call("mmad_ae_dw_events", self._h, int(bool(on)))

    def wait_dw(self, layer, stream):
        """`stream` waits for the last train_step's dW GEMM of `layer` and its
        bwd-data GEMM (needs dw_events(True) before that step)."""
        call("mmad_ae_wait_dw", self._h, int(layer), stream_ptr(stream))

    def dw_plan(self):
        """Weight buckets in backward order: [(offset, length, lowest layer)]."""
        cap = len(self.enc_widths) + len(self.dec_widths)
        off, n, lo = (ctypes.c_int64 * cap)(), (ctypes.c_int64 * cap)(), (ctypes.c_int * cap)()
        cnt = _native.load().mmad_ae_dw_plan(self._h, cap, off, n, lo)
        if cnt < 0:
            _native.check(cnt, "mmad_ae_dw_plan")
        return [(int(off[i]), int(n[i]), int(lo[i])) for i in range(cnt)]

    def forward(self, x, train_bn=False, want_xhat=True, want_loss=False):
        self._require(x)
        x = self._as_input(x, self.enc_widths[0])
        B = x.shape[0]
        self.sync_shadow()
        ws, nb = self.workspace(B, 1)
        xh = torch.empty((B, self.dec_widths[-1]), device=self.device) if want_xhat else None
        loss = torch.empty(1, device=self.device) if want_loss else None
        self.gen += 1
        call("mmad_ae_forward", self._h, ptr(x), x.stride(0), B, int(bool(train_bn)), ptr(xh),
             self.dec_widths[-1], ptr(loss), ws, nb, stream_ptr())
        return xh, loss

    def score(self, x, want_diffs=False):
        """Per-window squared-diff sums [n_enc+1, B] (and the concatenated diffs
        [B, sum widths] if asked) -- reconstruction_aggregation.get_diffs."""
        self._require(x)
        x = self._as_input(x, self.enc_widths[0])
        B = x.shape[0]
        self.sync_shadow()
        ws, nb = self.workspace(B, 1)
        lsq = torch.empty((self.n_enc + 1, B), device=self.device)
        diffs = None
        if want_diffs:
            diffs = torch.empty((B, self.diff_width()), device=self.device)
        self.gen += 1
        call("mmad_ae_score", self._h, ptr(x), x.stride(0), B, ptr(lsq), ptr(diffs), ws, nb,
             stream_ptr())
        return lsq, diffs

    def score_stream(self, x, batch, out, graph=True):
        """Whole-dataset scoring pass (mmad_ae_score_stream): x [N, D] fp32 on
        this device, out [n_enc+1, >=N] fp32 with unit column stride.  With
        graph=True the pass is captured once and replayed as one hipGraph."""
        self._require(x)
        x = self._as_input(x, self.enc_widths[0])
        N = x.shape[0]
        if out.device != self.device or out.dtype != torch.float32 or out.stride(1) != 1 \
                or out.shape[0] != self.n_enc + 1 or out.shape[1] < N:
            raise ValueError("score_stream: out must be fp32 [n_enc+1, >=N] on the model device")
        self.sync_shadow()
        B = min(int(batch), N)
        ws, nb = self.workspace(B, 1)
        self.gen += 1
        call("mmad_ae_score_stream", self._h, ptr(x), x.stride(0), N, B, ptr(out), out.stride(0),
             ws, nb, 1 if graph else 0, stream_ptr())
        return out

    def diff_widths(self):
        return [self.enc_widths[0]] + self.enc_widths[1:]

    def diff_width(self):
        return sum(self.diff_widths())


class _Snapshot:
    """CPU/host copy of the flat buffers used while moving devices."""

    def __init__(self, ae):
        for name in ("params", "grads", "exp_avg", "exp_avg_sq", "running"):
            setattr(self, name, getattr(ae, name).detach().clone())
