"""Bit-identity A/B across two builds of libmmad.so: a few fused train steps
at a chosen shape from fixed weights / data, then a SHA-256 of parameters,
Adam moments, BN running statistics and the losses.
Usage: python tools/step_hash.py <model ae|vib_ae> <batch> <dtype> [steps=3]"""
import hashlib
import sys
import types

sys.path.insert(0, ".")
import torch
from icra2021_multimodal_ad_amd.data import synth_windows
from icra2021_multimodal_ad_amd.model_builder import get_model

model_name, batch, dtype = sys.argv[1], int(sys.argv[2]), sys.argv[3]
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype=dtype,
                            models=model_name, vib_k=1, beta_kl=1.0)
torch.manual_seed(5)
m = get_model(cfg)
m._native.sync_shadow(force=True)
nat = m._native
eps = torch.randn(1, batch, 100, device="cuda") if model_name == "vib_ae" else None
h = hashlib.sha256()
for s in range(steps):
    x = torch.from_numpy(synth_windows(batch, 2048, seed=300 + s)).cuda()
    loss = nat.train_step_fused(x, eps=eps, beta_kl=1.0 if eps is not None else 0.0, k=1)
    h.update(loss.cpu().numpy().tobytes())
torch.cuda.synchronize()
nat.check_status()
for name in ("params", "exp_avg", "exp_avg_sq", "running"):
    h.update(getattr(nat, name).cpu().numpy().tobytes())
print(f"{model_name} B={batch} {dtype}: {h.hexdigest()}", flush=True)
