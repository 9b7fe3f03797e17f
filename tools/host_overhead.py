"""Host-side cost of one train step (enqueue only) vs its GPU time, per mode:
python wrapper (AutoEncoder.train_step_async), raw ctypes call of the eager
executor step, raw ctypes call of the graph-replayed step.
Usage: python tools/host_overhead.py [--dim 2048] [--batch 1024] [--steps 100]"""
import argparse
import ctypes
import os
import sys
import time
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from icra2021_multimodal_ad_amd import _native  # noqa: E402
from icra2021_multimodal_ad_amd._native import ptr, stream_ptr  # noqa: E402
from icra2021_multimodal_ad_amd.model_builder import get_model  # noqa: E402
from icra2021_multimodal_ad_amd.data import synth_windows_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--model", default="ae")
    a = ap.parse_args()
    cfg = types.SimpleNamespace(input_size=a.dim, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16",
                                models=a.model, vib_k=1, beta_kl=1.0)
    m = get_model(cfg)
    nat = m._native
    x = synth_windows_device(a.batch, a.dim, torch.device("cuda", 0), seed=1)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    lib = _native.load()
    for _ in range(5):
        m.train_step_async(x, opt)
    torch.cuda.synchronize()

    def timeit(fn, label):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        tt = time.perf_counter() - t0
        print(f"{label:34s} host {th / a.steps * 1e6:8.1f} us/step   wall {tt / a.steps * 1e6:8.1f} us/step",
              flush=True)

    for graph in (False, True):
        nat.use_graph = graph
        timeit(lambda: m.train_step_async(x, opt), f"python wrapper graph={graph}")
    ws, nb = nat.workspace(a.batch, 1)
    loss = torch.empty(1, device="cuda")
    s = stream_ptr()
    step = [nat.adam_step_count]

    def raw(fn):
        def f():
            step[0] += 1
            rc = getattr(lib, fn)(nat._h, ptr(x), x.stride(0), a.batch, 1, None, 1, 0, 1.0, 1e-3, 0.9,
                                  0.999, 1e-8, step[0], ptr(loss), ws, nb, s)
            assert rc == 0, lib.mmad_last_error_string()
        return f
    timeit(raw("mmad_ae_train_step"), "raw ctypes eager")
    timeit(raw("mmad_ae_train_step_graph"), "raw ctypes graph")
    print("graphs:", lib.mmad_ae_train_graph_count(nat._h))


if __name__ == "__main__":
    main()
