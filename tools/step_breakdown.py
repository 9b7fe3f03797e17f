"""Where a train step's time goes, without a profiler in the way: host enqueue
time per call and wall time per call (GPU-bound when wall > host) for the
fused step, the train-mode forward alone and forward+backward without Adam,
at one workload.  Knob variants are separate processes (env set before the
library loads).
Usage: python tools/step_breakdown.py [--dim 2048] [--batch 1024] [--model ae] [--steps 200]"""
import argparse
import os
import sys
import time
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from icra2021_multimodal_ad_amd.model_builder import get_model  # noqa: E402
from icra2021_multimodal_ad_amd.data import synth_windows_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--model", default="ae")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    cfg = types.SimpleNamespace(input_size=a.dim, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16",
                                models=a.model, vib_k=1, beta_kl=1.0)
    m = get_model(cfg)
    nat = m._native
    x = synth_windows_device(a.batch, a.dim, torch.device("cuda", 0), seed=1)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    for _ in range(5):
        m.train_step_async(x, opt)
    torch.cuda.synchronize()
    loss = torch.empty(1, device="cuda")

    def timeit(fn, label):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        tt = time.perf_counter() - t0
        print(f"{a.tag:10s} {label:24s} host {th / a.steps * 1e6:8.1f} us   wall {tt / a.steps * 1e6:8.1f} us",
              flush=True)

    timeit(lambda: m.train_step_async(x, opt), "step (fused Adam)")
    timeit(lambda: nat.forward(x, train_bn=True, want_xhat=False, want_loss=True), "forward (train BN)")
    timeit(lambda: nat.forward(x, train_bn=False, want_xhat=False, want_loss=True), "forward (eval)")
    timeit(lambda: nat.train_step(x, loss_out=loss), "fwd+bwd (no Adam)")
    nat.check_status()


if __name__ == "__main__":
    main()
