"""Data-parallel protocol on CPU: world_size=2 over gloo (127.0.0.1).

On the GPU with the 'nccl' group the default exchange is the native RCCL one
(dist.NativeComm attached to the executor): per bucket of consecutive layers a
reduce-scatter of the fp32 weight gradients, Adam on this rank's 1/N slice,
an all-gather of the bf16 shadow (ZeRO-1), plus one all-reduce of the small
bucket (bias / gamma / beta + loss); parameters are broadcast from rank 0 at
attach time.  The torch fallback checked here (gloo) sums the flat gradient
with one all-reduce -- both are the sum of the per-shard gradients.  Checked here: (1) the all-reduced gradient of
two shards equals the gradient of the concatenated batch (sum-reduced loss),
computed with the CPU oracle per shard; (2) after attach, both ranks hold
rank-0's parameters."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from icra2021_multimodal_ad_amd import dist as mdist
    r, w, _ = mdist.init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    from oracle import ae_oracle as O
    from oracle.model_io import model_from_state_dict, grads_to_flat
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict
    from icra2021_multimodal_ad_amd.data import synth_windows
    sd = init_state_dict(64, 100, 5, seed=9)
    x = synth_windows(32, 64, seed=100 + rank)                   # this rank's shard
    # BN is per shard (DDP semantics): each rank differentiates its own shard
    _, _, g = O.ae_train_grads(x, model_from_state_dict(sd))
    flat = torch.cat([torch.from_numpy(v.ravel()) for v in grads_to_flat(g).values()])
    dp = mdist.DataParallel()
    dp.all_reduce_grads(flat)
    loss = torch.tensor([float(rank + 1)])
    dp.all_reduce_loss(loss)
    params = torch.full((16,), float(rank))
    if dp.world > 1:
        dist.broadcast(params, src=0)
    out[rank] = (flat.numpy().copy(), float(loss.item()), params.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gradient_allreduce():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    from oracle import ae_oracle as O
    from oracle.model_io import model_from_state_dict, grads_to_flat
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict
    from icra2021_multimodal_ad_amd.data import synth_windows
    sd = init_state_dict(64, 100, 5, seed=9)
    shard_sum = None
    for rank in range(world):
        _, _, g = O.ae_train_grads(synth_windows(32, 64, seed=100 + rank), model_from_state_dict(sd))
        f = np.concatenate([v.ravel() for v in grads_to_flat(g).values()])
        shard_sum = f if shard_sum is None else shard_sum + f
    for rank in range(world):
        flat, loss, params = out[rank]
        np.testing.assert_allclose(flat, shard_sum, rtol=1e-5, atol=1e-5)
        assert loss == 3.0
        assert np.all(params == 0.0)


def _shard_worker(rank, world, port, out):
    """Row sharding + all-gather of per-window scores, BatchLoader rank
    shards, running-statistics averaging: the pieces of the data-parallel
    NoveltyDetecter (dist.py, data_loaders.BatchLoader) on CPU tensors."""
    import types
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from icra2021_multimodal_ad_amd import dist as mdist
    from icra2021_multimodal_ad_amd.data_loaders import get_loaders
    mdist.init_from_env(backend="gloo")
    dp = mdist.DataParallel(native=False)
    res = {}
    for n in (7, 8, 1001):
        x = torch.arange(n * 3, dtype=torch.float32).view(n, 3)
        res[f"gather{n}"] = dp.gather(dp.shard(x) * 2.0, n).numpy()
    # running statistics: rank r holds r + 1 everywhere -> mean over ranks
    stub = types.SimpleNamespace(_native=types.SimpleNamespace(running=torch.full((6,), float(rank + 1))))
    dp.average_running_stats(stub)
    res["running"] = stub._native.running.numpy()
    cfg = types.SimpleNamespace(data="hsr_objectdrop", target_class=1, unimodal_normal=False,
                                novelty_ratio=0.0, batch_size=64, input_size=16, n_normal=500,
                                n_novelty=100, data_seed=3, gpu_id=-1)
    _, tr, va, _ = get_loaders(cfg, device="cpu", rank=rank, world=world)
    res["train"] = [xb.numpy() for xb, _ in tr]
    res["valid"] = [xb.numpy() for xb, _ in va]
    out[rank] = res
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_gather_and_loaders():
    import types
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_shard_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for n in (7, 8, 1001):
        ref = np.arange(n * 3, dtype=np.float32).reshape(n, 3) * 2.0
        for r in range(world):
            np.testing.assert_array_equal(out[r][f"gather{n}"], ref)
    for r in range(world):
        np.testing.assert_array_equal(out[r]["running"], np.full(6, 1.5, np.float32))
    # the ranks' batches together are the single-process batches of 2 x 64
    # windows, in order (same sampler permutation on every rank)
    from icra2021_multimodal_ad_amd.data_loaders import get_loaders
    cfg = types.SimpleNamespace(data="hsr_objectdrop", target_class=1, unimodal_normal=False,
                                novelty_ratio=0.0, batch_size=128, input_size=16, n_normal=500,
                                n_novelty=100, data_seed=3, gpu_id=-1)
    _, tr, va, _ = get_loaders(cfg, device="cpu")
    for name, loader in (("train", tr), ("valid", va)):
        single = [xb.numpy() for xb, _ in loader]
        assert len(single) == len(out[0][name]) == len(out[1][name])
        for i, xb in enumerate(single):
            np.testing.assert_array_equal(np.concatenate([out[0][name][i], out[1][name][i]]), xb)


def _fallback_worker(rank, world, port, fail, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from icra2021_multimodal_ad_amd import dist as mdist
    mdist.init_from_env(backend="gloo")
    stage, bad_rank = fail
    dp = mdist.DataParallel(native=True, _fail=stage if rank == bad_rank else None)
    t = torch.tensor([float(rank + 1)])
    dp.all_reduce_sum(t)                       # the torch path works on every rank
    out[rank] = (dp.native, float(t.item()))
    dist.barrier()
    dist.destroy_process_group()


def test_native_comm_failure_on_one_rank_falls_back_together():
    """a rank whose native communicator cannot be built (rank 0's
    unique-id query, or any rank before RCCL init) must not leave its peers
    blocked in a collective: the staged agreement makes every rank fall back to
    torch.distributed together (no hang: the test joins within its timeout)."""
    for fail in (("uid", 0), ("create", 1), ("create", 0)):
        port = _free_port()
        mgr = mp.Manager()
        out = mgr.dict()
        ctx = mp.get_context("spawn")
        ps = [ctx.Process(target=_fallback_worker, args=(r, 2, port, fail, out)) for r in range(2)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(120)
        alive = [p.is_alive() for p in ps]
        for p in ps:
            if p.is_alive():
                p.kill()
        assert not any(alive), f"hang with failure {fail}"
        assert all(p.exitcode == 0 for p in ps), (fail, [p.exitcode for p in ps])
        assert out[0] == (False, 3.0) and out[1] == (False, 3.0), (fail, dict(out))


def test_rank_local_guard():
    """dist.rank_local marks code only some ranks run; a collective step
    entered inside it raises instead of hanging (AutoEncoder.train_step_async
    calls assert_collective_context whenever an exchange is attached)."""
    import pytest
    from icra2021_multimodal_ad_amd import dist as mdist
    mdist.assert_collective_context("outside")          # no-op
    with mdist.rank_local():
        with pytest.raises(RuntimeError, match="rank-local"):
            mdist.assert_collective_context("a DP step")
        with mdist.rank_local():
            pass
        with pytest.raises(RuntimeError):
            mdist.assert_collective_context("still inside")
    mdist.assert_collective_context("outside again")
    import inspect
    from icra2021_multimodal_ad_amd.auto_encoder import AutoEncoder
    src = inspect.getsource(AutoEncoder.train_step_async)
    # the guard follows the executor's communicator, not only model.dist
    # (tests/test_gpu_dp.py::test_rank_local_guard_follows_the_attached_communicator)
    assert "assert_collective_context" in src and "nat, \"_comm\"" in src


def test_exchange_failure_leaves_adam_step_count(monkeypatch):
    """A collective that raises inside DataParallel.exchange_and_adam (e.g. a
    gloo timeout) must not advance the Adam step count: a caller that catches
    the error and continues would otherwise run bias correction one step off.
    The count advances once the collectives and Adam calls are issued."""
    import types

    import pytest
    from icra2021_multimodal_ad_amd import dist as mdist
    monkeypatch.setenv("MMAD_DP_OVERLAP", "1")
    dp = mdist.DataParallel()                 # no process group: world 1
    assert dp.overlap is True                 # env read when built, not at import
    assert mdist.DataParallel(overlap=False).overlap is False
    dp.overlap = False
    calls = []
    nat = types.SimpleNamespace(adam_step_count=7, grads=torch.zeros(4),
                                adam=lambda **kw: calls.append(kw["step"]))

    def boom(_):
        raise RuntimeError("collective timed out")
    monkeypatch.setattr(dp, "all_reduce_grads", boom)
    with pytest.raises(RuntimeError, match="timed out"):
        dp.exchange_and_adam(nat, torch.zeros(()), 1e-3, (0.9, 0.999), 1e-8)
    assert nat.adam_step_count == 7 and calls == []
    monkeypatch.setattr(dp, "all_reduce_grads", lambda g: None)
    dp.exchange_and_adam(nat, torch.zeros(()), 1e-3, (0.9, 0.999), 1e-8)
    assert nat.adam_step_count == 8 and calls == [8]
