"""Data parallelism for the train step: one process per GPU, windows sharded by
rows, BatchNorm statistics per shard (DDP semantics).  Sum, not
mean: the reference loss is sum-reduced (model_builder.py:42), so the global
gradient of the concatenated batch is the sum of the shard gradients.

Two exchange paths:
* native (GPU, 'nccl' process group, the default): an RCCL communicator of our
  own (mmad_comm_*, unique id broadcast over the torch process group) attached
  to the executor.  The backward's weight gradients are grouped into buckets
  of >= 8 MiB (consecutive layers, one contiguous range each); as soon as a
  bucket's dW GEMMs complete, the comm stream REDUCE-SCATTERS its fp32
  gradient, runs Adam on this rank's 1/N slice of p / m / v only (ZeRO-1:
  optimizer state sharded, the bf16 weight shadow written for that slice), and
  ALL-GATHERS the updated shadow -- overlapped with the rest of the backward.
  Biases / gamma / beta + the loss follow in one small all-reduced bucket.  A
  bucket the ranks do not divide into 16-B slices keeps all-reduce + full
  Adam.  The fp32 master and m / v are then current only on their owner:
  ``epoch_end`` all-gathers them (mmad_ae_dp_sync_master) before anything
  reads the state_dict.  One host call per step, no host sync.
* torch (gloo / fallback): train_fwd_bwd, one torch.distributed all-reduce
  of the flat gradient, the flat Adam; or (DataParallel.overlap, opt-in) each
  weight bucket of the native plan all-reduced on its own stream as soon as
  the executor's dW events say its GEMMs are done and Adam-updated there
  (mmad_ae_adam_range), overlapping the rest of the backward.  Weights and
  Adam state replicated.

Around the step (NoveltyDetecter under data parallelism): each
rank trains on its rows of every global batch (data_loaders.BatchLoader with
rank / world), validation losses are summed over the ranks so every rank
keeps the same best-on-valid state, BatchNorm running statistics are averaged
at every epoch end, and scoring is sharded by rows with the per-window scores
all-gathered (shard_rows / gather_rows) before AUROC."""
import contextlib
import os
import threading

import torch
import torch.distributed as dist


def shard_rows(n, rank, world):
    """Contiguous row range [lo, hi) of `rank`'s shard of n rows: the first
    n % world ranks take one row more (rank order = row order)."""
    q, r = divmod(int(n), int(world))
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def gather_rows(local, n, group=None):
    """All-gather row shards cut by shard_rows back into the [n, ...] tensor
    (rank order), on every rank.  Shards are padded to the largest for the
    collective (all_gather needs equal sizes) and trimmed after."""
    world = dist.get_world_size(group)
    m = -(-int(n) // world)
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    out = []
    for r in range(world):
        lo, hi = shard_rows(n, r, world)
        out.append(parts[r][:hi - lo])
    return torch.cat(out, dim=0)


_LOCAL = threading.local()


@contextlib.contextmanager
def rank_local():
    """Marks code that only SOME ranks run (e.g. rank 0's kernel probe in
    bench.py).  Inside it, any call that would enter a collective exchange
    raises (assert_collective_context) instead of blocking forever in a
    collective the other ranks never join (round 2's r02zf bench hang)."""
    prev = getattr(_LOCAL, "depth", 0)
    _LOCAL.depth = prev + 1
    try:
        yield
    finally:
        _LOCAL.depth = prev


def assert_collective_context(what):
    if getattr(_LOCAL, "depth", 0) > 0:
        raise RuntimeError(f"{what} inside a rank-local region (dist.rank_local): the other ranks "
                           f"would never join its collectives; detach the exchange first")


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env vars.
    Returns (rank, world_size, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend)
    return rank, world, local


class NativeComm:
    """An RCCL communicator owned by libmmad (include/mmad.h, mmad_comm_*).

    Construction is collective and agreed in stages over the torch process
    group, so one rank's failure never leaves the others blocked in RCCL:
    rank 0 broadcasts the unique id together with a success flag (a failed id
    query makes every rank raise before any RCCL call); mmad_comm_create is
    then entered by every rank once all have agreed they are ready.  ``fail_stage`` (tests) makes this rank fail
    at 'uid' (rank 0's id query) or 'create'."""

    def __init__(self, group=None, fail_stage=None):
        import ctypes
        from . import _native
        self._lib = _native.load()
        self.handle = None
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        n = self._lib.mmad_comm_unique_id_bytes()
        uid = (ctypes.c_char * n)()
        ok = 1
        if self.rank == 0:
            try:
                if fail_stage == "uid":
                    raise RuntimeError("injected unique-id failure")
                _native.check(self._lib.mmad_comm_get_unique_id(uid), "mmad_comm_get_unique_id")
            except Exception:   # noqa: BLE001 -- every rank learns it from the flag
                ok = 0
        obj = [(ok, bytes(uid)) if self.rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        ok, raw = obj[0]
        if not ok:
            raise RuntimeError("rank 0 could not create the RCCL unique id")
        # every rank must reach mmad_comm_create (RCCL's init blocks until all
        # ranks have called it): agree first that all are ready
        ready = fail_stage != "create"
        if not _agree(ready, group, "cuda" if dist.get_backend(group) == "nccl" else "cpu"):
            raise RuntimeError("a rank could not prepare the RCCL communicator"
                               + ("" if ready else " (injected failure on this rank)"))
        uid = (ctypes.c_char * n).from_buffer_copy(raw)
        h = ctypes.c_void_p()
        _native.check(self._lib.mmad_comm_create(ctypes.byref(h), uid, self.world, self.rank),
                      "mmad_comm_create")
        self.handle = h

    def self_test(self, n=4096):
        """Every collective the step uses, through the library's communicator,
        on fresh stream-ordered buffers, checked on the host: sum all-reduce
        (rank r contributes r + 1), in-place reduce-scatter (fp32, bf16) and
        all-gather (fp32, bf16).  A communicator that builds but cannot
        exchange fails here, before any train step depends on it.  Every rank
        issues EVERY collective whatever an earlier check found (a rank that
        stopped at its first failure would leave its peers blocked in the next
        collective); the failures are raised only after the last one."""
        from . import _native
        from ._native import ptr, stream_ptr
        errors = []

        def issue(rc, what):
            # a failed enqueue is recorded, not raised: the peers still issue theirs
            if rc != 0:
                errors.append(f"{what}: {_native.last_error()}")
                return False
            return True

        want = self.world * (self.world + 1) / 2.0
        buf = torch.full((n,), float(self.rank + 1), device="cuda", dtype=torch.float32)
        if issue(self._lib.mmad_allreduce_bucket(self.handle, ptr(buf), n, stream_ptr()),
                 "mmad_allreduce_bucket") and not bool(torch.all(buf == want)):
            errors.append(f"all-reduce: got {float(buf[0])}, want {want}")
        m = 4096 * self.world
        buf = torch.full((m,), float(self.rank + 1), device="cuda", dtype=torch.float32)
        if issue(self._lib.mmad_reduce_scatter_bucket(self.handle, ptr(buf), m, stream_ptr()),
                 "mmad_reduce_scatter_bucket"):
            shard = buf[self.rank * 4096:(self.rank + 1) * 4096]
            if not bool(torch.all(shard == want)):
                errors.append(f"reduce-scatter: got {float(shard[0])}, want {want}")
        buf = torch.full((m,), float(self.rank + 1), device="cuda", dtype=torch.bfloat16)
        if issue(self._lib.mmad_reduce_scatter_bucket_bf16(self.handle, ptr(buf), m, stream_ptr()),
                 "mmad_reduce_scatter_bucket_bf16"):
            shard = buf[self.rank * 4096:(self.rank + 1) * 4096].float()
            if not bool(torch.all(shard == want)):
                errors.append(f"reduce-scatter (bf16): got {float(shard[0])}, want {want}")
        owners = torch.arange(self.world, device="cuda").repeat_interleave(4096).float() + 1.0
        for dt, code in ((torch.float32, _native.F32), (torch.bfloat16, _native.BF16)):
            g = torch.zeros(m, device="cuda", dtype=dt)
            g[self.rank * 4096:(self.rank + 1) * 4096] = float(self.rank + 1)
            if issue(self._lib.mmad_all_gather_bucket(self.handle, ptr(g), m, code, stream_ptr()),
                     f"mmad_all_gather_bucket({dt})") and not bool(torch.all(g.float() == owners)):
                errors.append(f"all-gather ({dt}) failed")
        torch.cuda.synchronize()
        if errors:
            raise RuntimeError("native RCCL self-test: " + "; ".join(errors))

    def close(self):
        if self.handle is not None and self.handle.value:
            self._lib.mmad_comm_destroy(self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _agree(flag, group, device):
    """MIN of a 0/1 flag over the ranks (every rank calls it)."""
    t = torch.tensor([1.0 if flag else 0.0], device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return float(t.item()) == 1.0


class DataParallel:
    """Gradient exchange for the data-parallel step.  The native RCCL path is
    chosen by three collective agreements (each a MIN over the ranks, so the
    ranks always take the same path and never wait in a collective another
    rank skipped): every rank wants it; every rank built its communicator;
    every rank's checked self-test all-reduce passed.  Otherwise all ranks use
    torch.distributed.  ``_fail`` (tests): inject a failure on this rank at
    'uid' / 'create' / 'selftest'."""

    def __init__(self, group=None, native=None, _fail=None, overlap=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.comm = None
        # torch exchange form (see `overlap` below): read here, not at import,
        # so a launcher that sets MMAD_DP_OVERLAP after importing the package
        # gets it (as MMAD_DP_GRAD_BF16 is read in attach_data_parallel)
        self.overlap = (os.environ.get("MMAD_DP_OVERLAP", "0") == "1") if overlap is None else bool(overlap)
        if native is None:
            native = (self.world > 1 and torch.cuda.is_available()
                      and dist.get_backend(group) == "nccl"
                      and os.environ.get("MMAD_NATIVE_COMM", "1") != "0")
        if self.world <= 1:
            return
        dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
        if not _agree(native, group, dev):
            return
        comm, err = None, None
        try:
            comm = NativeComm(group, fail_stage=_fail if _fail in ("uid", "create") else None)
        except Exception as e:  # noqa: BLE001 -- reported below, then fallback together
            err = e
            comm = None
        built = _agree(comm is not None, group, dev)
        passed = False
        if built:
            try:
                if _fail == "selftest":
                    raise RuntimeError("injected self-test failure")
                comm.self_test()
                passed = True
            except Exception as e:  # noqa: BLE001
                err = e
        if built and _agree(passed, group, dev):
            self.comm = comm
            return
        if comm is not None:
            comm.close()
        if dist.get_rank(group) == 0:
            print(f"[mmad] native RCCL exchange unavailable ({err}); using torch.distributed",
                  flush=True)

    def close(self):
        if self.comm is not None:
            self.comm.close()
            self.comm = None

    @property
    def native(self):
        return self.comm is not None

    # torch exchange: overlapped per bucket (True), or the serial form -- one
    # flat all-reduce after the backward, then the flat Adam (False, default;
    # same bits at 2 ranks).  Default off: over gloo (two ranks sharing one GPU,
    # the only multi-rank run available here) the overlapped form is 19 %
    # faster at D=2048 / 1024 windows per rank (13.4 vs 16.6 ms/step) but
    # 4.2 s/step at the C4 shape (VIB, 4096 windows) against 18 ms serial
    # (profiles/r07g_torch_exchange_gloo.txt): the fallback keeps the form
    # that measured well everywhere; env MMAD_DP_OVERLAP=1 (read when the
    # DataParallel is built) or attach_data_parallel(overlap=True) opts in
    overlap = False

    def all_reduce_grads(self, flat_grads):
        if self.world > 1:
            dist.all_reduce(flat_grads, op=dist.ReduceOp.SUM, group=self.group)

    @property
    def overlapped(self):
        return bool(self.overlap)

    def exchange_and_adam(self, nat, loss, lr, betas, eps):
        """The torch exchange of one data-parallel step, after nat.train_step
        was enqueued on the current stream: sum all-reduce of every gradient
        and of the loss, then Adam (one step count for every range).
        Overlapped: bucket b's all-reduce is issued on stream b, which first
        waits for the bucket's dW GEMMs and for the bwd-data GEMM of its lowest
        layer (the last reader of those weights: mmad_ae_wait_dw); Adam of the
        bucket follows on the same stream once its collective is done; the
        small bucket [bias | gamma | beta] and the loss are reduced after the
        backward; the current stream joins every bucket stream.  Adam is
        elementwise and a 2-rank sum is order-free, so at 2 ranks this is the
        serial form's result bit for bit (tests/test_gpu_dp.py)."""
        # the step count advances only once every collective and Adam call of
        # this step has been issued: a collective that raises (e.g. a gloo
        # timeout) leaves it, and the mirrored optimizer 'step', unchanged
        step = nat.adam_step_count + 1
        if not self.overlapped:
            self.all_reduce_grads(nat.grads)
            self.all_reduce_loss(loss)
            nat.adam(lr=lr, betas=betas, eps=eps, step=step)
            nat.adam_step_count = step
            return
        cur = torch.cuda.current_stream()
        plan = getattr(nat, "_dw_plan", None)
        if plan is None:
            plan = nat._dw_plan = nat.dw_plan()
        streams = getattr(nat, "_dw_streams", None)
        if streams is None or len(streams) < len(plan):
            streams = nat._dw_streams = [torch.cuda.Stream(device=nat.device) for _ in plan]
        pending = []
        for (off, n, lo), s in zip(plan, streams):
            nat.wait_dw(lo, s)
            with torch.cuda.stream(s):
                work = dist.all_reduce(nat.grads[off:off + n], op=dist.ReduceOp.SUM, group=self.group,
                                       async_op=True)
            pending.append((work, s, off, n))
        small = nat.grads[nat.n_weight:]
        w_small = dist.all_reduce(small, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        w_loss = dist.all_reduce(loss, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        for work, s, off, n in pending:
            with torch.cuda.stream(s):
                work.wait()
                nat.adam_range(off, n, lr=lr, betas=betas, eps=eps, step=step)
        w_small.wait()
        w_loss.wait()
        nat.adam_range(nat.n_weight, nat.n_params - nat.n_weight, lr=lr, betas=betas, eps=eps, step=step)
        for _, s, _, _ in pending:
            cur.wait_stream(s)
        nat.adam_step_count = step
        nat._mark_synced()

    def all_reduce_loss(self, loss):
        if self.world > 1:
            dist.all_reduce(loss, op=dist.ReduceOp.SUM, group=self.group)

    def all_reduce_sum(self, t):
        """In-place sum over ranks (validation losses: the reference's
        sum-MSE of the whole batch is the sum of the shard losses)."""
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def epoch_end(self, model):
        """Every rank, at every epoch end (before validation, which may deep-
        copy the state_dict): all-gather the sharded master weights / Adam
        moments of the native exchange, average the BN running statistics."""
        if self.native:
            model._native.sync_master()
        self.average_running_stats(model)
        from .auto_encoder import _check_status_all
        _check_status_all(model, force=True)

    def average_running_stats(self, model):
        """BatchNorm running mean / var averaged over the ranks (SURVEY
        §8(e): statistics are per shard while training, averaged for eval;
        called at every epoch end before validation)."""
        if self.world > 1:
            run = model._native.running
            dist.all_reduce(run, op=dist.ReduceOp.SUM, group=self.group)
            run.div_(self.world)

    def shard(self, x):
        """This rank's contiguous row shard of x (shard_rows)."""
        lo, hi = shard_rows(x.shape[0], dist.get_rank(self.group), self.world)
        return x[lo:hi]

    def gather(self, local, n):
        return gather_rows(local, n, self.group) if self.world > 1 else local

    def broadcast_params(self, model, src=0):
        if self.world > 1:
            dist.broadcast(model._native.params, src=src, group=self.group)


def attach_data_parallel(model, group=None, native=None, grad_bf16=None, overlap=None):
    """Replicate rank-0 weights and make AutoEncoder.step all-reduce grads
    (natively over RCCL, overlapped with the backward, when the process group
    is 'nccl'; through torch.distributed otherwise).  grad_bf16 (native path;
    default: env MMAD_DP_GRAD_BF16=1, else off): reduce-scatter the weight
    gradients in bf16 (mmad_ae_set_grad_bf16, half the exchange bytes; not the
    reference's fp32 sum).  overlap (torch exchange; default: env
    MMAD_DP_OVERLAP=1, else off): the per-bucket overlapped all-reduce + Adam."""
    dp = DataParallel(group, native=native, overlap=overlap)
    dp.broadcast_params(model)
    if dp.world > 1:
        model._native.sync_shadow(force=True)
    if dp.native:
        model._native.set_comm(dp.comm)
        if grad_bf16 is None:
            grad_bf16 = os.environ.get("MMAD_DP_GRAD_BF16", "0") == "1"
        if grad_bf16:
            model._native.set_grad_bf16(True)
    model.dist = dp if dp.world > 1 else None
    return model
