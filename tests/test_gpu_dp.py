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
