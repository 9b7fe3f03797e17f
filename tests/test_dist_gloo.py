"""Data-parallel protocol on CPU: world_size=2 over gloo (127.0.0.1).

The GPU exchange is the same code path with the 'nccl' (RCCL) backend: one sum
all-reduce of the flat fp32 gradient buffer per step, parameters broadcast
from rank 0 at attach time.  Checked here: (1) the all-reduced gradient of
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
