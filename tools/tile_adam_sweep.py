"""Step time of the fused train step with one GEMM class forced to each tile
config: knob 5 = Adam-fused dW GEMMs (default -2: shape rule), 6 = bwd-data
GEMMs, 7 = forward GEMMs (-1 = autotuned in isolation), 8 = Adam-fused dW
GEMMs on the main stream (-1 = knob 5).  Next to each step time: the in-step
duration of the largest layer's dW GEMM (executor probe, HIP events on its
stream) and its algorithmic HBM rate (bench.dw_adam_bytes).
Usage: python tools/tile_adam_sweep.py [knobs=5,6,7] [dim=2048] [batch=1024] [steps=300]
                                       [values=-1+0+1+2+3+4+5]  (lists: "," or "+")"""
import ctypes
import statistics
import sys
import time
import types

sys.path.insert(0, ".")
import torch

from bench import dw_adam_bytes, pick_dominant_layer
from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd.model_builder import get_model
from icra2021_multimodal_ad_amd.data import synth_windows_device

knobs = [int(k) for k in (sys.argv[1] if len(sys.argv) > 1 else "5,6,7").split(",")]
dim = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 300
values = [int(v) for v in (sys.argv[5] if len(sys.argv) > 5 else "-1,0,1,2,3,4,5").replace("+", ",").split(",")]
DEFAULT = {5: -2, 6: -1, 7: -1, 8: 0}
dev = torch.device("cuda", 0)
lib = _native.load()
pool = [synth_windows_device(B, dim, dev, seed=100 + i) for i in range(8)]
torch.manual_seed(0)
m = get_model(types.SimpleNamespace(input_size=dim, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16"))
nat = m._native
layer = pick_dominant_layer(nat, B)
L = nat.layers[layer]
nbytes = dw_adam_bytes(L["N"], L["K"], B)


def probe(n=40):
    _native.check(lib.mmad_ae_probe(nat._h, 1, layer, n), "probe")
    for i in range(n):
        m.train_step_async(pool[i % 8])
    torch.cuda.synchronize()
    buf = (ctypes.c_float * n)()
    k = lib.mmad_ae_probe_read(nat._h, buf, n)
    _native.check(lib.mmad_ae_probe(nat._h, 1, -1, 0), "probe off")
    return statistics.median(buf[:k]) * 1e3 if k > 0 else float("nan")


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
    us = probe()
    nat.check_status()
    return f"{best:.4f} ms/step; dW layer {layer} {us:.2f} us = {nbytes / us / 1e3:.0f} GB/s"


print(f"defaults: {timed()}", flush=True)
for k in knobs:
    for v in values:
        lib.mmad_tune_set(k, v)
        print(f"knob {k} = {v}: {timed()}", flush=True)
    lib.mmad_tune_set(k, DEFAULT[k])
print(f"defaults: {timed()}", flush=True)
