"""Step time of the fused train step under executor scheduling options, one
process: MMAD_DW_MAIN (how many of the last dW GEMMs run on the main stream)
x MMAD_SHADOW_PAIR (ping-pong bf16 shadows) x MMAD_SIDE_PRIO (side stream
lowest / highest priority) x MMAD_EV_EVERY (event coalescing).  All are read when a model is created, so each
configuration builds a fresh model.
Usage: python tools/sched_sweep.py [dim=2048] [batch=1024] [steps=300]"""
import os
import sys
import time
import types

sys.path.insert(0, ".")
import torch

from icra2021_multimodal_ad_amd.model_builder import get_model
from icra2021_multimodal_ad_amd.data import synth_windows_device

dim = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 300
dev = torch.device("cuda", 0)
pool = [synth_windows_device(B, dim, dev, seed=100 + i) for i in range(8)]
# configs: "pair,dw_main,side_prio,ev_every;..." (MMAD_SWEEP) or the default grid
if os.environ.get("MMAD_SWEEP"):
    configs = [tuple(c.split(",")) for c in os.environ["MMAD_SWEEP"].split(";")]
else:
    configs = [(pair, dm, prio, "1") for prio in ("0", "1") for pair in ("0", "1")
               for dm in ("0", "1", "2", "3")]
for pair, dm, prio, every in configs:
    if True:
        os.environ["MMAD_SHADOW_PAIR"] = pair
        os.environ["MMAD_DW_MAIN"] = dm
        os.environ["MMAD_SIDE_PRIO"] = prio
        os.environ["MMAD_EV_EVERY"] = every
        torch.manual_seed(0)
        m = get_model(types.SimpleNamespace(input_size=dim, btl_size=100, n_layers=5, gpu_id=0,
                                            dtype="bf16"))
        for i in range(20):
            m.train_step_async(pool[i % 8])
        torch.cuda.synchronize()
        best = None
        for rep in range(3):
            t0 = time.perf_counter()
            for i in range(steps):
                loss = m.train_step_async(pool[i % 8])
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) / steps * 1e3
            best = el if best is None else min(best, el)
        print(f"pair={pair} dw_main={dm} side_prio={prio} ev_every={every}: {best:.4f} ms/step  loss={float(loss):.2f}", flush=True)
        del m
