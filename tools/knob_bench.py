"""c2-shaped fused train step with tune-table knobs held for the WHOLE run
(GEMM knobs are read per dispatch, so they must stay set while stepping, unlike
the schedule knobs tools/sched_sweep.py applies at model creation).  Prints
ms/step and the tile each forward / bwd-data GEMM shape was tuned to.
Usage: python tools/knob_bench.py [batch=1024] [steps=300] [knob=value ...]"""
import sys
import time
import types

sys.path.insert(0, ".")
import torch

from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd.data import synth_windows_device
from icra2021_multimodal_ad_amd.model_builder import get_model

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
knobs = {k: int(v) for k, v in (a.split("=") for a in sys.argv[3:])}
dev = torch.device("cuda", 0)
for k, v in knobs.items():
    _native.tune_set(k, v)
m = get_model(types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16"))
m._native.sync_shadow(force=True)
pool = [synth_windows_device(B, 2048, dev, seed=100 + i) for i in range(8)]
for i in range(20):
    m._native.train_step_fused(pool[i % 8])
torch.cuda.synchronize()
best = None
for r in range(3):
    t0 = time.perf_counter()
    for i in range(steps):
        m._native.train_step_fused(pool[i % 8])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    best = ms if best is None else min(best, ms)
print(f"{knobs}: {best:.4f} ms/step (best of 3 x {steps} steps)", flush=True)
