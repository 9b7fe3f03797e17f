"""Step time of the fused train step under executor schedule knobs, one
process, interleaved rounds.  Each configuration is a set of tune knobs
(icra2021_multimodal_ad_amd._native.KNOB / SCHEDULE names) applied while its
model is created (the schedule knobs are read then).
Usage: python tools/sched_sweep.py [dim=2048] [batch=1024] [steps=300] ['k=v,k=v;k=v;...']
(default grid: dw_main x shadow_pair x side_prio)"""
import sys
import time
import types

sys.path.insert(0, ".")
import torch

from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd.model_builder import get_model
from icra2021_multimodal_ad_amd.data import synth_windows_device

dim = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 300
dev = torch.device("cuda", 0)
pool = [synth_windows_device(B, dim, dev, seed=100 + i) for i in range(8)]


def parse(c):
    out = {}
    for kv in filter(None, c.split(",")):
        k, v = kv.split("=")
        out[k] = (v == "1") if k in _native.SCHEDULE else int(v)
    return out


if len(sys.argv) > 4:
    configs = [parse(c) for c in sys.argv[4].split(";")]
else:
    configs = [dict(shadow_pair=pair, dw_main=dm, side_prio=prio) for prio in (0, 1)
               for pair in (False, True) for dm in (1, 2, 3)]
models = []
for knobs in configs:
    torch.manual_seed(0)
    with _native.tune(**knobs):
        m = get_model(types.SimpleNamespace(input_size=dim, btl_size=100, n_layers=5, gpu_id=0,
                                            dtype="bf16"))
    for i in range(20):
        m.train_step_async(pool[i % 8])
    models.append(m)
torch.cuda.synchronize()
best = [None] * len(models)
for rep in range(3):
    for j, m in enumerate(models):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            loss = m.train_step_async(pool[i % 8])
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps * 1e3
        best[j] = el if best[j] is None else min(best[j], el)
for knobs, b in zip(configs, best):
    print(f"{knobs}: {b:.4f} ms/step", flush=True)
