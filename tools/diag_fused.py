"""Diagnostic: fused (per-layer Adam in dW epilogue) vs unfused step, after one step."""
import sys, types
sys.path.insert(0, ".")
import numpy as np, torch
from icra2021_multimodal_ad_amd.model_builder import get_model
from icra2021_multimodal_ad_amd.common_utils import init_state_dict
from icra2021_multimodal_ad_amd.data import synth_windows

def mk(dtype):
    cfg = types.SimpleNamespace(input_size=192, btl_size=16, n_layers=5, gpu_id=0, dtype=dtype)
    m = get_model(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in init_state_dict(192, 16, 5, seed=31).items()})
    return m
for dtype in ["f32", "bf16"]:
    ma, mb = mk(dtype), mk(dtype)
    for s in range(3):
        x = torch.from_numpy(synth_windows(200, 192, seed=40 + s)).cuda()
        pa0 = ma._native.params.clone()
        la = ma._native.train_step_fused(x)
        lb = mb._native.train_step(x)
        torch.cuda.synchronize()
        ga, gb = ma._native.grads.clone(), mb._native.grads.clone()
        mb._native.adam()
        torch.cuda.synchronize()
        nat = ma._native
        for l, L in enumerate(nat.layers):
            for name, off, n in (("W", L["w_off"], L["Np"] * L["Kp"]), ("small", L["b_off"], (3 if L["bn"] else 1) * L["Np"])):
                dg = (ga[off:off+n] - gb[off:off+n]).abs().max().item()
                dp = (ma._native.params[off:off+n] - mb._native.params[off:off+n]).abs().max().item()
                if dg > 0 or dp > 1e-7:
                    i = int((ma._native.params[off:off+n] - mb._native.params[off:off+n]).abs().argmax())
                    print(dtype, "step", s, "layer", l, name, "grad diff", dg, "param diff", dp, "at", i,
                          "ga", ga[off+i].item(), "gb", gb[off+i].item())
        print(dtype, "step", s, "loss", float(la), float(lb), "running eq", torch.equal(ma._native.running, mb._native.running))
