"""Torch-exchange DP step (2 ranks sharing cuda:0 over gloo) at a chosen
size, with a traceback dump of every thread if a rank stalls: the harness
for debugging / timing the overlapped exchange (dist.DataParallel.overlap).
Usage: python tools/dp_torch_probe.py <overlap 0|1|2> <model ae|vib_ae> <batch> <steps>
(2: the overlapped form with every bucket stream waiting for the whole
backward instead of its dW events -- isolates the event gating)"""
import faulthandler
import os
import socket
import sys
import time
import types

import torch
import torch.multiprocessing as mp

sys.path.insert(0, ".")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, overlap, model_name, batch, steps):
    faulthandler.dump_traceback_later(60, exit=True)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import torch.distributed as dist
    from icra2021_multimodal_ad_amd import dist as mdist
    from icra2021_multimodal_ad_amd.data import synth_windows_device
    from icra2021_multimodal_ad_amd.model_builder import get_model
    mdist.init_from_env(backend="gloo")
    torch.cuda.set_device(0)
    cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16",
                                models=model_name, vib_k=1, beta_kl=1.0)
    torch.manual_seed(0)
    m = get_model(cfg)
    mdist.attach_data_parallel(m)
    m.dist.overlap = bool(overlap)
    if overlap == 2:
        m._native.dw_events(True)
        m._native._dw_events = True
        m._native.wait_dw = lambda layer, stream: stream.wait_stream(torch.cuda.current_stream())
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    pool = [synth_windows_device(batch, 2048, torch.device("cuda", 0), seed=1000 * rank + i) for i in range(4)]
    for i in range(2):
        m.train_step_async(pool[i % 4], opt)
        print(f"rank {rank} warm step {i} done", flush=True)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = m.train_step_async(pool[i % 4], opt)
    torch.cuda.synchronize()
    dist.barrier()
    el = (time.perf_counter() - t0) / steps * 1e3
    print(f"rank {rank} overlap={overlap} {model_name} B={batch}: {el:.3f} ms/step loss {float(loss):.4f} "
          f"buckets {len(m._native.dw_plan())}", flush=True)
    faulthandler.cancel_dump_traceback_later()
    dist.destroy_process_group()


if __name__ == "__main__":
    overlap, model_name, batch, steps = int(sys.argv[1]), sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    mp.start_processes(worker, args=(2, _port(), overlap, model_name, batch, steps), nprocs=2, join=True,
                       start_method="spawn")
