"""Step time of the fused train step with one GEMM class forced to each tile
config: knob 5 = Adam-fused dW GEMMs (default 3), 6 = bwd-data GEMMs, 7 =
forward GEMMs (-1 = autotuned in isolation), 8 = Adam-fused dW GEMMs on the
main stream (-1 = knob 5).
Usage: python tools/tile_adam_sweep.py [knobs=5,6,7] [dim=2048] [batch=1024] [steps=300]"""
import sys
import time
import types

sys.path.insert(0, ".")
import torch

from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd.model_builder import get_model
from icra2021_multimodal_ad_amd.data import synth_windows_device

knobs = [int(k) for k in (sys.argv[1] if len(sys.argv) > 1 else "5,6,7").split(",")]
dim = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 300
DEFAULT = {5: 3, 6: -1, 7: -1, 8: -1}
dev = torch.device("cuda", 0)
lib = _native.load()
pool = [synth_windows_device(B, dim, dev, seed=100 + i) for i in range(8)]
torch.manual_seed(0)
m = get_model(types.SimpleNamespace(input_size=dim, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16"))


def timed():
    for i in range(10):
        m.train_step_async(pool[i % 8])
    torch.cuda.synchronize()
    best = None
    for rep in range(3):
        t0 = time.perf_counter()
        for i in range(steps):
            m.train_step_async(pool[i % 8])
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps * 1e3
        best = el if best is None else min(best, el)
    return best


print(f"defaults: {timed():.4f} ms/step", flush=True)
for k in knobs:
    for v in (-1, 0, 1, 2, 3, 4, 5):
        lib.mmad_tune_set(k, v)
        print(f"knob {k} = {v}: {timed():.4f} ms/step", flush=True)
    lib.mmad_tune_set(k, DEFAULT[k])
print(f"defaults: {timed():.4f} ms/step", flush=True)
