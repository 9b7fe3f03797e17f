"""Cost of the data-parallel step schedule on ONE GPU: the fused single-process
step vs the native-exchange step with a loopback communicator (all-reduce =
identity scale 1.0 after a short delay), D=2048, bf16.  The difference
is what the DP schedule costs before any real xGMI traffic.
Usage: python tools/dp_overhead.py [steps=50] [batch=1024] [model=ae]"""
import ctypes
import sys
import time
import types

sys.path.insert(0, ".")
import torch
from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd.model_builder import get_model
from icra2021_multimodal_ad_amd.data import synth_windows_device

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
model = sys.argv[3] if len(sys.argv) > 3 else "ae"
dev = torch.device("cuda", 0)
lib = _native.load()


def run(comm):
    cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16",
                                models=model, vib_k=1, beta_kl=1.0)
    torch.manual_seed(0)
    m = get_model(cfg)
    m._native.sync_shadow(force=True)
    if comm is not None:
        m._native.set_comm(comm)
    pool = [synth_windows_device(batch, 2048, dev, seed=i) for i in range(8)]
    for i in range(10):
        m._native.train_step_fused(pool[i % 8])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        m._native.train_step_fused(pool[i % 8])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    if comm is not None:
        m._native.set_comm(None)
    return dt


h = ctypes.c_void_p()
assert lib.mmad_comm_create_loopback(ctypes.byref(h), 1.0) == 0
t_fused = run(None)
t_dp = run(types.SimpleNamespace(handle=h))
lib.mmad_comm_destroy(h)
print(f"{model} B={batch}: fused step {t_fused * 1e3:.4f} ms, DP schedule (loopback exchange) {t_dp * 1e3:.4f} ms")
