"""Where the host time of one eager c3 training step goes (cProfile over
train_step_async, the GPU kept busy): the bench's host_enqueue_ms_per_step
against the raw enqueue onto idle streams.
Usage: python tools/host_profile_c3.py [steps=200]"""
import cProfile
import pstats
import sys
import time
import types

sys.path.insert(0, ".")
import torch  # noqa: E402
from icra2021_multimodal_ad_amd.model_builder import get_model  # noqa: E402
from icra2021_multimodal_ad_amd.data import synth_windows_device  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16",
                            models="vib_ae", vib_k=1, beta_kl=1.0)
torch.manual_seed(0)
model = get_model(cfg)
model._native.sync_shadow(force=True)
opt = torch.optim.Adam(model.parameters(), lr=1e-3)
dev = torch.device("cuda", 0)
pool = [synth_windows_device(4096, 2048, dev, seed=i) for i in range(8)]
for i in range(20):
    model.train_step_async(pool[i % 8], opt)
torch.cuda.synchronize()
raw = 0.0
for i in range(50):
    torch.cuda.synchronize()
    t = time.perf_counter()
    model.train_step_async(pool[i % 8], opt)
    raw += time.perf_counter() - t
torch.cuda.synchronize()
print(f"raw enqueue onto idle streams {raw / 50 * 1e3:.4f} ms/step")
for n in (20, 100, steps):
    t = time.perf_counter()
    for i in range(n):
        model.train_step_async(pool[i % 8], opt)
    th = time.perf_counter() - t
    torch.cuda.synchronize()
    tw = time.perf_counter() - t
    print(f"{n} back-to-back steps: host {th / n * 1e3:.4f} ms/step, wall {tw / n * 1e3:.4f} ms/step")
pr = cProfile.Profile()
pr.enable()
for i in range(steps):
    model.train_step_async(pool[i % 8], opt)
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(15)
