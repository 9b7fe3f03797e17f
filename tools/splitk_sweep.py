"""Tile x split-K sweep of the bench GEMM shapes (D=2048 AE, bf16) with the
K loop on and off (tuning knob 3 bit 0 skips it: prologue + epilogue only).
Usage: python tools/splitk_sweep.py [batch=1024] [kinds=fwd,bwd_data,bwd_w] [layers=0,1]  (lists: "," or "+")"""
import json
import sys

sys.path.insert(0, ".")
import torch
from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
kinds = (sys.argv[2] if len(sys.argv) > 2 else "fwd,bwd_data,bwd_w").replace("+", ",").split(",")
layers = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "0,1").replace("+", ",").split(",")]
widths = [2048, 1658, 1268, 879, 489, 100, 489, 879, 1268, 1658, 2048]
dev = torch.device("cuda", 0)
lib = _native.load()
_native.enable_gemm_workspace(dev)
s = stream_ptr()
Mp = pad(B)


def timeit(fn, iters=40):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for li in layers:
    K, N = widths[li], widths[li + 1]
    Kp, Np = pad(K), pad(N)
    x = torch.randn(Mp, Kp, device=dev).bfloat16()
    w = (torch.randn(Np, Kp, device=dev) * 0.02).bfloat16()
    b = torch.zeros(Np, device=dev)
    y = torch.empty(Mp, Np, device=dev, dtype=torch.bfloat16)
    st = torch.empty(Mp // 32, 2, Np, device=dev)
    dz = torch.randn(Mp, Np, device=dev).bfloat16()
    dx = torch.empty(Mp, Kp, device=dev, dtype=torch.bfloat16)
    dw = torch.empty(Np, Kp, device=dev)
    fns = {
        "fwd": lambda: call("mmad_fc_fwd", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1, 0.2,
                            None, None, ptr(y), ptr(st), s),
        "bwd_data": lambda: call("mmad_fc_bwd_data", 1, B, N, K, Mp, Np, Kp, ptr(dz), ptr(w), ptr(dx),
                                 None, s),
        "bwd_w": lambda: call("mmad_fc_bwd_weight", 1, Mp, Np, Kp, ptr(dz), ptr(x), ptr(dw), s),
    }
    fl = 2.0 * B * K * N
    for kind in kinds:
        rows = []
        for tile in range(6):
            for sk in (1, 2, 4):
                lib.mmad_tune_set(0, tile)
                lib.mmad_tune_set(4, sk)
                lib.mmad_tune_set(3, 0)
                try:
                    t = timeit(fns[kind])
                    lib.mmad_tune_set(3, 1)
                    t0 = timeit(fns[kind])
                except Exception as e:  # noqa: BLE001 -- tile does not fit this shape
                    rows.append({"tile": tile, "sk": sk, "err": str(e)[:60]})
                    continue
                rows.append({"tile": tile, "sk": sk, "us": round(t, 2), "us_noloop": round(t0, 2),
                             "tflops": round(fl / t / 1e6, 1)})
        lib.mmad_tune_set(3, 0)
        lib.mmad_tune_set(0, -1)
        lib.mmad_tune_set(4, 0)
        best = min((r for r in rows if "us" in r), key=lambda r: r["us"])
        print(json.dumps({"kind": kind, "layer": li, "M": B, "N": N, "K": K, "best": best,
                          "rows": rows}), flush=True)
