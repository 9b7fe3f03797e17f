"""Split-K x tile sweep of the Adam-fused dW GEMMs (mmad_fc_bwd_weight_adam)
of the D=2048 AE / VIB-AE at one batch: for every layer shape, every split
factor S in {1,2,4,8,16} (tuning knob 9) and tiles {3: 64x64, 0: 128x128,
4: 64x128}, the average launch time over back-to-back launches.
Usage: python tools/splitk_dw_sweep.py [batch=1024] [vib=0]"""
import json
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

from icra2021_multimodal_ad_amd import _native  # noqa: E402
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad, BF16  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
vib = len(sys.argv) > 2 and sys.argv[2] == "1"
enc = [2048, 1658, 1268, 879, 489, 200 if vib else 100]
dec = [100, 489, 879, 1268, 1658, 2048]
shapes = list(zip(enc[:-1], enc[1:])) + list(zip(dec[:-1], dec[1:]))
dev = torch.device("cuda", 0)
lib = _native.load()
_native.enable_gemm_workspace(dev)
s = stream_ptr()
Mp = pad(B)


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for li, (K, N) in enumerate(shapes):
    Kp, Np = pad(K), pad(N)
    dz = torch.randn(Mp, Np, device=dev).bfloat16()
    x = torch.randn(Mp, Kp, device=dev).bfloat16()
    p = torch.randn(Np, Kp, device=dev) * 0.02
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    sh = torch.zeros(Np, Kp, device=dev, dtype=torch.bfloat16)
    rows = []
    for tile in (3, 0, 4):
        for S in (1, 2, 4, 8, 16):
            lib.mmad_tune_set(5, tile)
            lib.mmad_tune_set(9, S)
            try:
                t = timeit(lambda: call("mmad_fc_bwd_weight_adam", BF16, Mp, Np, Kp, ptr(dz), ptr(x), ptr(p),
                                        ptr(m), ptr(v), ptr(sh), None, 0.9, 0.999, 1e-8, 1e-3, 1.0, s))
                call("mmad_gemm_status", s)
            except _native.NativeError as e:
                rows.append({"tile": tile, "S": S, "err": str(e)[:80]})
                continue
            rows.append({"tile": tile, "S": S, "us": round(t, 2)})
    lib.mmad_tune_set(9, 0)
    lib.mmad_tune_set(5, -2)
    base = next(r["us"] for r in rows if r.get("tile") == 3 and r.get("S") == 1 and "us" in r)
    best = min((r for r in rows if "us" in r), key=lambda r: r["us"])
    # what the default rule picks (knob 9 = 0) at the default tile
    t_rule = timeit(lambda: call("mmad_fc_bwd_weight_adam", BF16, Mp, Np, Kp, ptr(dz), ptr(x), ptr(p),
                                 ptr(m), ptr(v), ptr(sh), None, 0.9, 0.999, 1e-8, 1e-3, 1.0, s))
    print(json.dumps({"layer": li, "M": B, "dW": [N, K], "t64": (Np // 64) * (Kp // 64),
                      "rule_split": lib.mmad_gemm_splitk_for(Np, Kp, Mp, BF16, 3),
                      "rule_us": round(t_rule, 2), "tile3_S1_us": base, "best": best, "rows": rows}),
          flush=True)
