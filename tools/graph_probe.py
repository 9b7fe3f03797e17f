"""The c2 train step, eager or as one captured hipGraph per step, for a
rocprofv3 kernel trace.  Usage: python tools/graph_probe.py eager|graph [steps=30] [knob=value ...]
(extra tune-table knobs, e.g. bn_mode=0 side_prio=1, applied while the model is built)"""
import sys
import time
import types

sys.path.insert(0, ".")
import torch
from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd.model_builder import get_model
from icra2021_multimodal_ad_amd.data import synth_windows_device

mode = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
dev = torch.device("cuda", 0)
extra = {k: int(v) for k, v in (a.split("=") for a in sys.argv[3:])}
with _native.tune(train_graph=mode == "graph", **extra):
    m = get_model(types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16"))
m._native.sync_shadow(force=True)
opt = torch.optim.Adam(m.parameters(), lr=1e-3)
pool = [synth_windows_device(1024, 2048, dev, seed=i) for i in range(8)]
for i in range(10):
    m.train_step_async(pool[i % 8], opt)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(steps):
    m.train_step_async(pool[i % 8], opt)
th = time.perf_counter() - t0
torch.cuda.synchronize()
tw = time.perf_counter() - t0
print(f"{mode} {extra}: host {th / steps * 1e6:.1f} us/step, wall {tw / steps * 1e6:.1f} us/step, "
      f"graphs {m._native._lib.mmad_ae_train_graph_count(m._native._h)}", flush=True)
