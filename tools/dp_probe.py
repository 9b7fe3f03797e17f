"""One DP-schedule variant alone, for a rocprofv3 kernel trace: the fused
step driven through a loopback communicator posing as rank r of n, with the
tune knob dp_shard = s (n=0: no exchange attached, the fused single-process step).  Usage: python tools/dp_probe.py n r s [steps=20] [batch=1024] [mib=8] [fork=default] [noraw]
(mib: knob dp_bucket_mib, the minimum exchange bucket; fork: knob dp_fork_rows)"""
import ctypes
import sys
import time
import types

sys.path.insert(0, ".")
import torch
from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd.model_builder import get_model
from icra2021_multimodal_ad_amd.data import synth_windows_device

n, r, shard = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
batch = int(sys.argv[5]) if len(sys.argv) > 5 else 1024
mib = int(sys.argv[6]) if len(sys.argv) > 6 else 8
fork = int(sys.argv[7]) if len(sys.argv) > 7 else None   # None: the library default
raw_loop = not (len(sys.argv) > 8 and sys.argv[8] == "noraw")   # noraw: traces end on the timed loop
dev = torch.device("cuda", 0)
lib = _native.load()
h = ctypes.c_void_p()
assert lib.mmad_comm_create_loopback_ranks(ctypes.byref(h), 1.0, max(n, 1), r) == 0
cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16")
with _native.tune(dp_shard=shard, dp_bucket_mib=mib, **({} if fork is None else dict(dp_fork_rows=fork))):
    m = get_model(cfg)
m._native.sync_shadow(force=True)
if n > 0:
    m._native.set_comm(types.SimpleNamespace(handle=h))
pool = [synth_windows_device(batch, 2048, dev, seed=i) for i in range(8)]
for i in range(10):
    m._native.train_step_fused(pool[i % 8])
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(steps):
    m._native.train_step_fused(pool[i % 8])
th = time.perf_counter() - t0
torch.cuda.synchronize()
tw = time.perf_counter() - t0
# raw host cost of enqueueing one step onto idle streams (sync before each)
raw = 0.0
for i in range(steps if raw_loop else 0):
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    m._native.train_step_fused(pool[i % 8])
    raw += time.perf_counter() - t1
torch.cuda.synchronize()
print(f"n={n} r={r} shard={shard} mib={mib} fork={fork} batch={batch}: {tw / steps * 1e3:.4f} ms/step "
      f"(host enqueue in the loop {th / steps * 1e3:.4f}, raw enqueue onto idle streams "
      f"{raw / steps * 1e3:.4f} ms/step)", flush=True)
if n > 0:
    m._native.sync_master()
    m._native.set_comm(None)
lib.mmad_comm_destroy(h)
