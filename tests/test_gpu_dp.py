"""Data-parallel train step through the HIP path: 2 ranks sharing cuda:0 over
gloo (RCCL refuses two ranks on one device; the exchange code is identical).
After one step both ranks must hold identical parameters equal to a
single-process step whose gradient is the sum of the two shard gradients."""
import os
import socket
import types

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg():
    return types.SimpleNamespace(input_size=192, btl_size=16, n_layers=5, gpu_id=0, dtype="f32")


def _model():
    from icra2021_multimodal_ad_amd.model_builder import get_model
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict
    m = get_model(_cfg())
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in
                       init_state_dict(192, 16, 5, seed=51).items()})
    return m


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import torch.distributed as dist
    from icra2021_multimodal_ad_amd import dist as mdist
    from icra2021_multimodal_ad_amd.data import synth_windows
    mdist.init_from_env(backend="gloo")
    torch.cuda.set_device(0)
    m = _model()
    mdist.attach_data_parallel(m)
    x = torch.from_numpy(synth_windows(96, 192, seed=60 + rank)).cuda()
    loss = m.train_step_async(x, torch.optim.Adam(m.parameters(), lr=1e-3))
    torch.cuda.synchronize()
    out[rank] = (m._native.params.cpu().numpy(), float(loss))
    dist.barrier()
    dist.destroy_process_group()


def _xworker(rank, world, port, out, overlap, dtype, mib, dim, batch):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import torch.distributed as dist
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd import dist as mdist
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict
    from icra2021_multimodal_ad_amd.data import synth_windows
    from icra2021_multimodal_ad_amd.model_builder import get_model
    mdist.init_from_env(backend="gloo")
    torch.cuda.set_device(0)
    cfg = _cfg()
    cfg.dtype = dtype
    cfg.input_size = dim
    cfg.btl_size = 16 if dim == 192 else 100
    torch.manual_seed(0)
    with _native.tune(dp_bucket_mib=mib):
        m = get_model(cfg)
    if dim == 192:
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in
                           init_state_dict(192, 16, 5, seed=51).items()})
    mdist.attach_data_parallel(m)
    m.dist.overlap = overlap
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    losses = []
    for s in range(3):
        x = torch.from_numpy(synth_windows(batch, dim, seed=60 + 10 * s + rank)).cuda()
        losses.append(float(m.train_step_async(x, opt)))
    torch.cuda.synchronize()
    nat = m._native
    out[rank] = (nat.params.cpu().numpy(), nat.exp_avg.cpu().numpy(), nat.exp_avg_sq.cpu().numpy(),
                 nat.shadow.float().cpu().numpy() if nat.shadow is not None else None, losses,
                 len(nat.dw_plan()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype,mib,dim,batch", [("f32", 0, 192, 96), ("bf16", 0, 192, 96),
                                                 ("bf16", 8, 192, 96), ("bf16", 8, 2048, 1024)])
def test_torch_exchange_overlapped_equals_serial(dtype, mib, dim, batch):
    """The torch exchange (the path without the native communicator):
    per-bucket all-reduce + Adam on bucket streams gated by the executor's dW
    events (DataParallel.overlap, opt-in) gives the serial form's bits
    -- one flat all-reduce after the backward, then the flat Adam -- over 3
    steps at 2 ranks (a 2-operand sum is order-free, Adam elementwise):
    parameters, Adam moments and the bf16 shadow (losses to 1e-6: tile-
    dependent partial order).  mib = 0: one
    bucket per layer (10 buckets); 8: the default plan (one bucket at D=192,
    five at D=2048 -- the size at which executor events without a system-scope
    fence let the exchange's copy read stale gradients, round 4)."""
    world = 2
    res = {}
    for overlap in (False, True):
        mgr = mp.get_context("spawn").Manager()
        out = mgr.dict()
        mp.start_processes(_xworker, args=(world, _free_port(), out, overlap, dtype, mib, dim, batch),
                           nprocs=world,
                           join=True, start_method="spawn")
        res[overlap] = dict(out)
    for rank in range(world):
        a, b = res[False][rank], res[True][rank]
        for i, name in enumerate(("params", "exp_avg", "exp_avg_sq", "shadow")):
            if a[i] is not None:
                assert np.array_equal(a[i], b[i]), (rank, name)
        # the loss sums one partial per MSE output tile: the per-process
        # autotuner's tile pick may reorder it (1 ulp), the gradients never
        np.testing.assert_allclose(a[4], b[4], rtol=1e-6, atol=0)
    assert np.array_equal(res[True][0][0], res[True][1][0])
    assert res[True][0][5] == (10 if mib == 0 else (1 if dim == 192 else 5))


def test_dp_two_ranks_equals_summed_gradient_step():
    world = 2
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    from icra2021_multimodal_ad_amd.data import synth_windows
    m = _model()
    nat = m._native
    losses, gsum = 0.0, None
    for rank in range(world):
        x = torch.from_numpy(synth_windows(96, 192, seed=60 + rank)).cuda()
        # restore BN running stats between shards is unnecessary: grads do not read them
        losses += float(nat.train_step(x))
        gsum = nat.grads.clone() if gsum is None else gsum + nat.grads
    nat.grads.copy_(gsum)
    nat.adam(lr=1e-3)
    ref = nat.params.cpu().numpy()
    p0, l0 = out[0]
    p1, l1 = out[1]
    assert np.array_equal(p0, p1)
    assert abs(l0 - losses) <= 1e-5 * losses and l0 == l1
    np.testing.assert_allclose(p0, ref, rtol=0, atol=1e-6)


def test_native_comm_single_rank_step_matches_fused():
    """The native RCCL data-parallel step (per-layer all-reduce on the comm
    stream + flat Adam per bucket) with one rank equals the single-process
    fused step (all-reduce of one rank is the identity).  Multi-rank RCCL needs
    one GPU per rank; the exchange semantics are pinned on CPU by
    tests/test_dist_gloo.py."""
    import ctypes
    import types as _t
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd.data import synth_windows
    lib = _native.load()
    n = lib.mmad_comm_unique_id_bytes()
    uid = (ctypes.c_char * n)()
    assert lib.mmad_comm_get_unique_id(uid) == 0, lib.mmad_last_error_string()
    h = ctypes.c_void_p()
    assert lib.mmad_comm_create(ctypes.byref(h), uid, 1, 0) == 0, lib.mmad_last_error_string()
    comm = _t.SimpleNamespace(handle=h)
    try:
        buf = torch.arange(1000, dtype=torch.float32, device="cuda")
        ref = buf.clone()
        assert lib.mmad_allreduce_bucket(h, ctypes.c_void_p(buf.data_ptr()), 1000, None) == 0
        torch.cuda.synchronize()
        assert torch.equal(buf, ref)
        ma, mb = _model(), _model()
        ma._native.set_comm(comm)
        for s in range(3):
            x = torch.from_numpy(synth_windows(200, 192, seed=70 + s)).cuda()
            la = float(ma._native.train_step_fused(x))
            lb = float(mb._native.train_step_fused(x))
            assert abs(la - lb) <= 1e-6 * abs(lb)
        torch.cuda.synchronize()
        d = (ma._native.params - mb._native.params).abs().max().item()
        assert d <= 1e-6, d
        assert torch.equal(ma._native.running, mb._native.running)
        ma._native.set_comm(None)
    finally:
        lib.mmad_comm_destroy(h)


@pytest.mark.parametrize("dtype,mib,fork", [("f32", 8, 0), ("bf16", 8, 0), ("bf16", 0, 0), ("f32", 1000, 0),
                                            ("f32", 8, 1), ("bf16", 1000, 1), ("bf16", 8, 100000)])
def test_native_exchange_schedule_loopback(dtype, mib, fork):
    """Exchange schedule of the native DP step on one GPU: a loopback
    communicator whose all-reduce doubles each bucket (= 2 identical shards)
    after a delay.  Must equal: plain fwd+bwd, grads *= 2, loss *= 2, flat Adam
    -- i.e. every bucket is reduced after its producer finished and before its
    Adam, and the small bucket + loss are reduced too -- whatever the bucket
    plan (knob dp_bucket_mib: 0 = one bucket per layer, 1000 = all weights in
    one bucket closed by layer 0), and whether each side-stream dW GEMM starts
    at its own dz or with its bucket's lowest layer (knob dp_fork_rows: 1 =
    per layer at every batch, 100000 = per bucket)."""
    import ctypes
    import types as _t
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd.data import synth_windows
    from icra2021_multimodal_ad_amd.model_builder import get_model
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict
    lib = _native.load()
    h = ctypes.c_void_p()
    assert lib.mmad_comm_create_loopback(ctypes.byref(h), 2.0) == 0
    comm = _t.SimpleNamespace(handle=h)

    def mk():
        cfg = _t.SimpleNamespace(input_size=700, btl_size=40, n_layers=5, gpu_id=0, dtype=dtype)
        m = get_model(cfg)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in
                           init_state_dict(700, 40, 5, seed=81).items()})
        return m
    try:
        with _native.tune(dp_bucket_mib=mib, dp_fork_rows=fork):
            ma = mk()
        mb = mk()
        ma._native.set_comm(comm)
        for s in range(3):
            x = torch.from_numpy(synth_windows(384, 700, seed=90 + s)).cuda()
            la = float(ma._native.train_step_fused(x))
            lb = mb._native.train_step(x)
            mb._native.grads.mul_(2.0)
            mb._native.adam()
            assert abs(la - 2.0 * float(lb)) <= 1e-5 * abs(la)
        torch.cuda.synchronize()
        d = (ma._native.params - mb._native.params).abs().max().item()
        assert d <= 1e-6, d
        ma._native.set_comm(None)
    finally:
        lib.mmad_comm_destroy(h)


@pytest.mark.parametrize("dtype,fork", [("bf16", 1024), ("f32", 1024), ("bf16", 0)])
def test_native_exchange_vib_mixed_rows_loopback(dtype, fork):
    """The native DP step on a VIB-AE with k = 2 samples: the decoder runs
    k * B = 1024 rows, the encoder B = 512, so at dp_fork_rows = 1024 the
    decoder layers' dW GEMMs fork one by one while the encoder layers' wait
    for their bucket's lowest layer, inside one bucket (dp_bucket_mib = 1000:
    every weight in the bucket layer 0 closes).  With a loopback all-reduce
    that doubles each bucket it must equal fwd+bwd, grads x 2, flat Adam,
    on the same injected samples."""
    import ctypes
    import types as _t
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd.data import synth_windows
    from icra2021_multimodal_ad_amd.model_builder import get_model
    lib = _native.load()
    h = ctypes.c_void_p()
    assert lib.mmad_comm_create_loopback(ctypes.byref(h), 2.0) == 0
    comm = _t.SimpleNamespace(handle=h)

    def mk():
        cfg = _t.SimpleNamespace(input_size=700, btl_size=40, n_layers=5, gpu_id=0, dtype=dtype,
                                 models="vib_ae", vib_k=2, beta_kl=1.0)
        torch.manual_seed(17)
        m = get_model(cfg)
        m._native.sync_shadow(force=True)
        return m
    try:
        with _native.tune(dp_bucket_mib=1000, dp_fork_rows=fork):
            ma = mk()
        mb = mk()
        assert torch.equal(ma._native.params, mb._native.params)
        ma._native.set_comm(comm)
        g = torch.Generator(device="cuda").manual_seed(3)
        for s in range(2):
            x = torch.from_numpy(synth_windows(512, 700, seed=40 + s)).cuda()
            eps = torch.randn(2, 512, 40, device="cuda", generator=g)
            la = float(ma._native.train_step_fused(x, k=2, eps=eps, beta_kl=1.0))
            lb = mb._native.train_step(x, k=2, eps=eps, beta_kl=1.0)
            mb._native.grads.mul_(2.0)
            mb._native.adam()
            assert abs(la - 2.0 * float(lb)) <= 1e-5 * abs(la), (la, float(lb))
        torch.cuda.synchronize()
        d = (ma._native.params - mb._native.params).abs().max().item()
        assert d <= 1e-6, d
        ma._native.set_comm(None)
    finally:
        lib.mmad_comm_destroy(h)


def _nd_cfg():
    return types.SimpleNamespace(input_size=192, btl_size=16, n_layers=5, gpu_id=0, dtype="f32",
                                 models="ae", batch_size=64, n_epochs=2, n_normal=700, n_novelty=140,
                                 anomaly_strength=0.7, data="hsr_objectdrop", target_class=1,
                                 unimodal_normal=False, novelty_ratio=0.0, start_layer_index=0,
                                 end_layer_index=-1, data_seed=5, sampler_seed=6, verbose=0)


def _nd_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import torch.distributed as dist
    from icra2021_multimodal_ad_amd import dist as mdist
    from icra2021_multimodal_ad_amd.data_loaders import get_loaders
    from icra2021_multimodal_ad_amd.novelty_detection import NoveltyDetecter
    mdist.init_from_env(backend="gloo")
    torch.cuda.set_device(0)
    m = _model()
    mdist.attach_data_parallel(m)
    cfg = _nd_cfg()
    det = NoveltyDetecter(cfg)
    dset, tr, va, te = get_loaders(cfg, rank=rank, world=world)
    th, vh, _, m = det.train(m, tr, va)
    res = det.test(m, dset, tr, va, te)
    out[rank] = dict(params=m._native.params.cpu().numpy(), running=m._native.running.cpu().numpy(),
                     vh=list(vh), best=det.best_epoch, res=[list(r) for r in res[:3]],
                     scores={k: (v.copy(), t.copy()) for k, (v, t) in det.last_scores.items()},
                     sd={k: v.cpu().numpy() for k, v in m.state_dict().items()})
    dist.barrier()
    dist.destroy_process_group()


def test_dp_novelty_detecter_two_ranks():
    """NoveltyDetecter.train / test under data parallelism (2 ranks sharing
    cuda:0 over gloo): each rank trains on its rows of every global batch,
    validation losses are summed over the ranks, BN running statistics
    averaged at every epoch end, scoring sharded by rows and all-gathered.
    Both ranks must end with the same parameters, running statistics,
    best-on-valid epoch and metrics, and the gathered per-window BASE / SAP /
    NAP scores must equal a single process scoring the final model."""
    world = 2
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    mp.start_processes(_nd_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    a, b = out[0], out[1]
    assert np.array_equal(a["params"], b["params"])
    assert np.array_equal(a["running"], b["running"])
    assert a["best"] == b["best"] and a["vh"] == b["vh"] and a["res"] == b["res"]
    from icra2021_multimodal_ad_amd.data_loaders import get_loaders
    from icra2021_multimodal_ad_amd.novelty_detection import NoveltyDetecter
    m = _model()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in a["sd"].items()})
    cfg = _nd_cfg()
    det = NoveltyDetecter(cfg)
    dset, tr, va, te = get_loaders(cfg)
    for _ in range(cfg.n_epochs):       # the train sampler's state after training (same train_x order)
        list(iter(tr.sampler))
    det.test(m, dset, tr, va, te)
    for k, (v, t) in det.last_scores.items():
        np.testing.assert_allclose(a["scores"][k][0], v, rtol=1e-5, atol=1e-7, err_msg=k)
        np.testing.assert_allclose(a["scores"][k][1], t, rtol=1e-5, atol=1e-7, err_msg=k)


def test_native_comm_self_test_passes_and_catches_a_broken_exchange():
    """dist.NativeComm.self_test (run before the native exchange is used, the
    ranks fall back to torch.distributed together if it fails): a one-rank
    RCCL communicator sums correctly; a loopback communicator that doubles
    its buffer (a wrong exchange) is rejected -- after issuing every
    collective of the test (the failure of the first check is reported
    together with the later ones: a rank that stopped at its first failure
    would leave its peers blocked in the next collective)."""
    import ctypes
    import types as _t
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd.dist import NativeComm
    lib = _native.load()
    torch.cuda.set_device(0)
    n = lib.mmad_comm_unique_id_bytes()
    uid = (ctypes.c_char * n)()
    assert lib.mmad_comm_get_unique_id(uid) == 0, lib.mmad_last_error_string()
    h = ctypes.c_void_p()
    assert lib.mmad_comm_create(ctypes.byref(h), uid, 1, 0) == 0, lib.mmad_last_error_string()
    good = _t.SimpleNamespace(_lib=lib, handle=h, rank=0, world=1)
    NativeComm.self_test(good)
    lib.mmad_comm_destroy(h)
    hb = ctypes.c_void_p()
    assert lib.mmad_comm_create_loopback(ctypes.byref(hb), 2.0) == 0
    bad = _t.SimpleNamespace(_lib=lib, handle=hb, rank=0, world=1)
    with pytest.raises(RuntimeError, match="self-test") as ei:
        NativeComm.self_test(bad)
    assert "all-reduce" in str(ei.value) and "reduce-scatter" in str(ei.value), str(ei.value)
    lib.mmad_comm_destroy(hb)


def _dp_plan(layers, mib):
    """(offset, n) of every weight exchange bucket (mirror of mmad_ae.hip
    dp_plan: consecutive layers in backward order until >= mib MiB of fp32)."""
    out, acc = [], 0
    for l in range(len(layers) - 1, -1, -1):
        acc += layers[l]["Np"] * layers[l]["Kp"]
        if acc * 4 >= mib * (1 << 20) or l == 0:
            out.append((layers[l]["w_off"], acc))
            acc = 0
    return out


@pytest.mark.parametrize("dtype,rank,mib,gbf,fork", [("bf16", 0, 8, False, 0), ("bf16", 1, 8, False, 0),
                                                     ("f32", 1, 8, False, 0), ("bf16", 1, 0, False, 0),
                                                     ("f32", 0, 2, False, 0), ("bf16", 1, 0, True, 0),
                                                     ("bf16", 0, 8, True, 0), ("f32", 1, 8, True, 0),
                                                     ("bf16", 1, 8, False, 1), ("f32", 0, 0, True, 1)])
def test_sharded_exchange_shard_arithmetic_loopback(dtype, rank, mib, gbf, fork):
    """The sharded DP step (knob dp_shard: reduce-scatter, Adam on this rank's
    1/N of each weight bucket, all-gather of the updated weights) on one GPU,
    through a loopback communicator posing as rank `rank` of 2 (its
    reduce-scatter doubles this rank's slice = 2 identical shards summed into
    the slice RCCL's in-place reduce-scatter writes, its all-gather leaves the
    other rank's shard alone).  This rank's shard of
    every weight bucket -- p, m, v and the bf16 shadow -- equals "grads x 2,
    then Adam" bit for bit; the other shard keeps its pre-step p / m / v;
    the small bucket is all-reduced and fully updated; the handle reports
    stale master weights and refuses to detach until synced.  The shards
    follow the bucket plan (knob dp_bucket_mib: consecutive layers share a
    bucket, split once over the ranks).  gbf: the optional bf16 gradient
    exchange (mmad_ae_set_grad_bf16) -- this rank's shard then equals "bf16(g)
    x 2 widened to fp32, then Adam" bit for bit (the loopback's bf16 sum of
    two identical shards is exact, as RCCL's 2-rank bf16 sum of bf16 inputs
    rounds once).  fork: knob dp_fork_rows (1 = each side-stream dW GEMM at
    its own dz)."""
    import ctypes
    import types as _t
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd.data import synth_windows
    from icra2021_multimodal_ad_amd.model_builder import get_model
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict
    lib = _native.load()
    h = ctypes.c_void_p()
    assert lib.mmad_comm_create_loopback_ranks(ctypes.byref(h), 2.0, 2, rank) == 0
    comm = _t.SimpleNamespace(handle=h)

    def mk():
        cfg = _t.SimpleNamespace(input_size=700, btl_size=40, n_layers=5, gpu_id=0, dtype=dtype)
        m = get_model(cfg)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in
                           init_state_dict(700, 40, 5, seed=83).items()})
        m._native.sync_shadow(force=True)
        return m
    try:
        with _native.tune(dp_bucket_mib=mib, dp_fork_rows=fork):
            ma = mk()
        mb = mk()
        a, b = ma._native, mb._native
        a.set_comm(comm)
        if gbf:
            a.set_grad_bf16(True)
        x = torch.from_numpy(synth_windows(384, 700, seed=95)).cuda()
        p0, m0, v0 = a.params.clone(), a.exp_avg.clone(), a.exp_avg_sq.clone()
        la = float(a.train_step_fused(x))
        lb = b.train_step(x)
        if gbf:
            b.grads[:b.n_weight] = b.grads[:b.n_weight].bfloat16().float()
        b.grads.mul_(2.0)
        b.adam()
        torch.cuda.synchronize()
        assert abs(la - 2.0 * float(lb)) <= 1e-5 * abs(la)
        assert lib.mmad_ae_dp_master_stale(a._h) == 1
        plan = _dp_plan(a.layers, mib)
        assert (len(plan) == len(a.layers)) == (mib == 0)
        for boff, n in plan:
            lo = boff + rank * (n // 2)
            own = slice(lo, lo + n // 2)
            other = slice(boff + (1 - rank) * (n // 2), boff + (2 - rank) * (n // 2))
            for name, ref0 in (("params", p0), ("exp_avg", m0), ("exp_avg_sq", v0)):
                got, want = getattr(a, name), getattr(b, name)
                assert torch.equal(got[own], want[own]), (name, boff)
                assert torch.equal(got[other], ref0[other]), (name, "other shard changed", boff)
            if dtype == "bf16":
                assert torch.equal(a.shadow[own], b.shadow[own])
        nw = a.n_weight
        for name in ("params", "exp_avg", "exp_avg_sq"):      # the small bucket: all-reduced
            assert torch.equal(getattr(a, name)[nw:], getattr(b, name)[nw:]), name
        assert lib.mmad_ae_set_comm(a._h, None) != 0          # stale: detach refused
        with pytest.raises(RuntimeError, match="sharded"):
            ma.state_dict()
        a.sync_master()                                        # loopback all-gather: a no-op
        assert not a.master_stale
        a.set_comm(None)
    finally:
        lib.mmad_comm_destroy(h)


def _c4_model(dtype):
    """BASELINE configs[3]'s per-GPU model: VIB-AE, D=2048, btl 100, 5+5 layers
    (bench.py CONFIGS['c4']), seeded init, shadow synced."""
    import types as _t
    from icra2021_multimodal_ad_amd.model_builder import get_model
    cfg = _t.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype=dtype,
                             models="vib_ae", vib_k=1, beta_kl=1.0)
    torch.manual_seed(29)
    m = get_model(cfg)
    m._native.sync_shadow(force=True)
    return m


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
@pytest.mark.parametrize("gbf", [False, True])
@pytest.mark.parametrize("rank", [0, 3, 7])
def test_c4_sharded_exchange_rank_of_8_loopback(dtype, gbf, rank):
    """The C4 exchange at its own shape (BASELINE configs[3]: VIB-AE, D=2048,
    4096 windows per GPU, 8 ranks), default knobs (dp_bucket_mib 8 ->
    buckets {9}, {8}, {7..3}, {2,1}, {0}; dp_fork_rows default), on one GPU
    through a loopback communicator posing as rank `rank` of 8: its
    reduce-scatter multiplies this rank's 1/8 slice by 8 (= 8 identical
    shards summed into the slice RCCL's in-place reduce-scatter writes), its
    all-gather leaves the other 7 slices alone.  After one step, for every
    weight bucket: this rank's slice of p / m / v (and the bf16 shadow) equals
    "grads x 8, then Adam" of a single-process step on the same batch and
    injected VIB noise, bit for bit; the other 7/8 keep their pre-step values;
    the small bucket (bias / gamma / beta + loss) is all-reduced and fully
    updated.  gbf: the bf16 gradient exchange (x 8 is exact in bf16, so the
    slice equals "bf16(g) x 8 widened, then Adam").  Every bucket of the
    padded layout is a multiple of 128 x 128 values, so n / 8 is an integer
    multiple of 4 and every weight bucket takes the sharded form (the
    all-reduce fallback for other rank counts: the test below)."""
    import ctypes
    import types as _t
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd.data import synth_windows
    lib = _native.load()
    world = 8
    h = ctypes.c_void_p()
    assert lib.mmad_comm_create_loopback_ranks(ctypes.byref(h), float(world), world, rank) == 0
    comm = _t.SimpleNamespace(handle=h)
    try:
        ma, mb = _c4_model(dtype), _c4_model(dtype)
        a, b = ma._native, mb._native
        assert torch.equal(a.params, b.params)
        a.set_comm(comm)
        if gbf:
            a.set_grad_bf16(True)
        x = torch.from_numpy(synth_windows(4096, 2048, seed=400 + rank)).cuda()
        eps = torch.randn(1, 4096, 100, device="cuda",
                          generator=torch.Generator(device="cuda").manual_seed(rank))
        p0, m0, v0 = a.params.clone(), a.exp_avg.clone(), a.exp_avg_sq.clone()
        s0 = a.shadow.clone() if dtype == "bf16" else None
        la = float(a.train_step_fused(x, k=1, eps=eps, beta_kl=1.0))
        lb = b.train_step(x, k=1, eps=eps, beta_kl=1.0)
        if gbf:
            b.grads[:b.n_weight] = b.grads[:b.n_weight].bfloat16().float()
        b.grads.mul_(float(world))
        b.adam()
        torch.cuda.synchronize()
        a.check_status()
        assert abs(la - world * float(lb)) <= 1e-5 * abs(la), (la, float(lb))
        assert lib.mmad_ae_dp_master_stale(a._h) == 1
        plan = _dp_plan(a.layers, 8)
        assert [n for _, n in plan] == [n for _, n, _ in a.dw_plan()]
        assert [lo for _, _, lo in a.dw_plan()] == [9, 8, 3, 1, 0]
        covered = 0
        for boff, n in plan:
            assert n % world == 0 and (n // world) % 4 == 0, (boff, n)
            cnt = n // world
            own = slice(boff + rank * cnt, boff + (rank + 1) * cnt)
            for name, ref0 in (("params", p0), ("exp_avg", m0), ("exp_avg_sq", v0)):
                got, want = getattr(a, name), getattr(b, name)
                assert torch.equal(got[own], want[own]), (name, boff)
                assert not torch.equal(got[own], ref0[own]), (name, "own shard not updated", boff)
                for r in range(world):
                    if r != rank:
                        oth = slice(boff + r * cnt, boff + (r + 1) * cnt)
                        assert torch.equal(got[oth], ref0[oth]), (name, "other shard changed", boff, r)
            if dtype == "bf16":
                assert torch.equal(a.shadow[own], b.shadow[own])
                assert torch.equal(a.shadow[boff:boff + rank * cnt], s0[boff:boff + rank * cnt])
                assert torch.equal(a.shadow[boff + (rank + 1) * cnt:boff + n], s0[boff + (rank + 1) * cnt:boff + n])
            covered += n
        nw = a.n_weight
        assert covered == nw
        for name in ("params", "exp_avg", "exp_avg_sq"):      # the small bucket: all-reduced
            assert torch.equal(getattr(a, name)[nw:], getattr(b, name)[nw:]), name
        assert torch.equal(a.running, b.running)
        a.sync_master()                                        # loopback all-gather: a no-op
        a.set_comm(None)
    finally:
        lib.mmad_comm_destroy(h)


@pytest.mark.parametrize("dtype,world,rank", [("f32", 6, 2), ("bf16", 3, 1), ("bf16", 7, 4)])
def test_c4_exchange_indivisible_world_falls_back_to_all_reduce(dtype, world, rank):
    """A rank count that does not divide a bucket takes the all-reduce form
    for that bucket: the whole bucket summed, then Adam on all of it and the
    shadow.  At the C4 model (buckets of 3407872, 2129920, 2490368, 3964928,
    3670016 values) 3 and 6 ranks divide none of them; 7 divides only layer
    0's bucket, which is sharded while the other four are all-reduced.  The
    result is "grads x world, then Adam" on every all-reduced bucket and on
    this rank's slice of a sharded one, bit for bit; the master weights are
    stale only when some bucket was sharded."""
    import ctypes
    import types as _t
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd.data import synth_windows
    lib = _native.load()
    h = ctypes.c_void_p()
    assert lib.mmad_comm_create_loopback_ranks(ctypes.byref(h), float(world), world, rank) == 0
    comm = _t.SimpleNamespace(handle=h)
    try:
        ma, mb = _c4_model(dtype), _c4_model(dtype)
        a, b = ma._native, mb._native
        a.set_comm(comm)
        x = torch.from_numpy(synth_windows(4096, 2048, seed=77)).cuda()
        eps = torch.randn(1, 4096, 100, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5))
        la = float(a.train_step_fused(x, k=1, eps=eps, beta_kl=1.0))
        lb = b.train_step(x, k=1, eps=eps, beta_kl=1.0)
        b.grads.mul_(float(world))
        b.adam()
        torch.cuda.synchronize()
        assert abs(la - world * float(lb)) <= 1e-5 * abs(la)
        n_sharded = 0
        for boff, n in _dp_plan(a.layers, 8):
            if n % world == 0 and (n // world) % 4 == 0:
                n_sharded += 1
                cnt = n // world
                rng = slice(boff + rank * cnt, boff + (rank + 1) * cnt)
            else:
                rng = slice(boff, boff + n)
            for name in ("params", "exp_avg", "exp_avg_sq"):
                assert torch.equal(getattr(a, name)[rng], getattr(b, name)[rng]), (name, boff)
            if dtype == "bf16":
                assert torch.equal(a.shadow[rng], b.shadow[rng]), boff
        assert n_sharded == (1 if world == 7 else 0)
        nw = a.n_weight
        for name in ("params", "exp_avg", "exp_avg_sq"):
            assert torch.equal(getattr(a, name)[nw:], getattr(b, name)[nw:]), name
        assert lib.mmad_ae_dp_master_stale(a._h) == (1 if n_sharded else 0)
        a.sync_master()
        a.set_comm(None)
    finally:
        lib.mmad_comm_destroy(h)


def test_rank_local_guard_follows_the_attached_communicator():
    """A step whose executor still holds a communicator enters collectives
    even when model.dist has been cleared (bench.py's rank-0 probe does
    exactly that): inside dist.rank_local() it must raise, not run the
    exchange on one rank; detached, the same call runs."""
    import ctypes
    import types as _t
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd import dist as mdist
    from icra2021_multimodal_ad_amd.data import synth_windows
    from icra2021_multimodal_ad_amd.model_builder import get_model
    lib = _native.load()
    h = ctypes.c_void_p()
    assert lib.mmad_comm_create_loopback(ctypes.byref(h), 1.0) == 0
    try:
        m = get_model(_t.SimpleNamespace(input_size=256, btl_size=20, n_layers=5, gpu_id=0, dtype="bf16"))
        x = torch.from_numpy(synth_windows(256, 256, seed=3)).cuda()
        m._native.set_comm(_t.SimpleNamespace(handle=h))
        assert m.dist is None
        with mdist.rank_local():
            with pytest.raises(RuntimeError, match="rank-local"):
                m.train_step_async(x)
        m._native.sync_master()
        m._native.set_comm(None)
        with mdist.rank_local():
            m.train_step_async(x)                  # no exchange attached: allowed
        torch.cuda.synchronize()
    finally:
        lib.mmad_comm_destroy(h)
