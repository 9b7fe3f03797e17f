"""Stand-alone time of the train-mode BatchNorm + activation backward
(mmad_bn_act_bwd: the column-sum reduce kernel + bn_bwd_apply_k) at the C3
shapes (4096 windows, bf16), against its algorithmic bytes: the in-step
bn_bwd_apply_k (profiles/r06b_prof_c3) runs beside the side stream's dW+Adam.
Usage: python tools/bn_bwd_time.py [rows=4096]"""
import json
import sys

sys.path.insert(0, ".")
import torch
from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
lib = _native.load()
dev = torch.device("cuda", 0)
for Np in (1664, 1280, 896, 512):
    dy = torch.randn(rows, Np, device=dev).bfloat16()
    a = torch.randn(rows, Np, device=dev).bfloat16()
    mean = torch.zeros(Np, device=dev)
    rstd = torch.ones(Np, device=dev)
    gamma = torch.ones(Np, device=dev)
    dz = torch.empty(rows, Np, device=dev, dtype=torch.bfloat16)
    dg = torch.empty(Np, device=dev)
    db = torch.empty(Np, device=dev)
    dbp = torch.empty(rows // 128, Np, device=dev)
    ws = torch.empty(int(lib.mmad_bn_act_bwd_ws(rows, Np)) // 4 + 1, device=dev)

    def fn():
        call("mmad_bn_act_bwd", 1, 1, 0.2, rows, Np, rows, Np, ptr(dy), ptr(a), ptr(mean), ptr(rstd),
             ptr(gamma), ptr(dz), ptr(dg), ptr(db), ptr(dbp), ptr(ws), stream_ptr())
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    alg = rows * Np * 2 * (2 + 2 + 1)   # reduce reads dy, a; apply reads dy, a, writes dz
    print(json.dumps(dict(rows=rows, Np=Np, us=round(us, 2), alg_MB=round(alg / 1e6, 1),
                          TBps=round(alg / us / 1e6, 2))), flush=True)
