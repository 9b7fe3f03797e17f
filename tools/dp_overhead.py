"""Cost of the data-parallel step schedule on ONE GPU, each variant in its own
process (several models in one process share the 4 hardware queues and
serialise each other's streams): the fused single-process step vs the
native-exchange step through a loopback communicator (exchange = scale 1.0
after a short spin), D=2048, bf16: the all-reduce schedule (knob
dp_shard=0), the sharded schedule as one rank of 1 (reduce-scatter = the
loopback all-reduce, Adam on the whole bucket) and as rank 0 of 8 (Adam on
1/8 of each bucket: this rank's share of an 8-GPU step without the
all-gather's traffic).  The loopback's spin (~10 us per bucket on the comm
stream) stands in for the transfer, so the numbers bound the schedule's own
cost from above.
Usage: python tools/dp_overhead.py [steps=50] [batch=1024]"""
import subprocess
import sys

steps = sys.argv[1] if len(sys.argv) > 1 else "50"
batch = sys.argv[2] if len(sys.argv) > 2 else "1024"
fused = subprocess.run([sys.executable, "-c", f"""
import sys, time, types
sys.path.insert(0, '.')
import torch
from icra2021_multimodal_ad_amd.model_builder import get_model
from icra2021_multimodal_ad_amd.data import synth_windows_device
m = get_model(types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype='bf16'))
m._native.sync_shadow(force=True)
pool = [synth_windows_device({batch}, 2048, torch.device('cuda', 0), seed=i) for i in range(8)]
for i in range(10): m._native.train_step_fused(pool[i % 8])
torch.cuda.synchronize(); t0 = time.perf_counter()
for i in range({steps}): m._native.train_step_fused(pool[i % 8])
torch.cuda.synchronize()
print(f'fused single-process step: {{(time.perf_counter() - t0) / {steps} * 1e3:.4f}} ms/step')
"""], capture_output=True, text=True, check=True).stdout.strip()
print(f"B={batch} {fused}", flush=True)
for n, r, s, what in (("1", "0", "0", "DP all-reduce schedule"), ("1", "0", "1", "DP sharded, 1 rank"),
                      ("8", "0", "1", "DP sharded, rank 0 of 8")):
    out = subprocess.run([sys.executable, "tools/dp_probe.py", n, r, s, steps, batch], capture_output=True,
                         text=True, check=True).stdout.strip().splitlines()[-1]
    print(f"B={batch} {what}: {out.split(': ')[-1]}", flush=True)
