"""bf16 vs fp32 training trajectories on the bench workload (D=2048, B=1024):
same init, same batches; prints the per-step loss ratio bf16/f32.
Usage: python tools/loss_track.py [steps=60]"""
import sys
import types

sys.path.insert(0, ".")
import torch
from icra2021_multimodal_ad_amd.model_builder import get_model
from icra2021_multimodal_ad_amd.common_utils import init_state_dict
from icra2021_multimodal_ad_amd.data import synth_windows_device

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
dev = torch.device("cuda", 0)
sd = {k: torch.from_numpy(v) for k, v in init_state_dict(2048, 100, 5, seed=0).items()}
pool = [synth_windows_device(1024, 2048, dev, seed=i) for i in range(8)]
out = {}
for dt in ("f32", "bf16"):
    cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype=dt)
    m = get_model(cfg)
    m.load_state_dict(sd)
    m._native.sync_shadow(force=True)
    out[dt] = [float(m.train_step_async(pool[i % 8])) for i in range(steps)]
for i in range(0, steps, max(1, steps // 15)):
    print(f"step {i:3d}  f32 {out['f32'][i]:12.2f}  bf16 {out['bf16'][i]:12.2f}  ratio {out['bf16'][i] / out['f32'][i]:.4f}")
print("final", out["f32"][-1], out["bf16"][-1])
