"""GEMM tuning sweep: time every fwd / bwd-data / dW GEMM shape of the
D=2048 bench AE at B=1024 (bf16) for each tile config and XCD group height.
Usage: python tools/gemm_bench.py [batch]"""
import sys, json
sys.path.insert(0, ".")
import torch
from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
widths = [2048, 1658, 1268, 879, 489, 100, 489, 879, 1268, 1658, 2048]
dev = torch.device("cuda", 0)
lib = _native.load()
_native.enable_gemm_workspace(dev)
s = stream_ptr()
Mp = pad(B)

def timeit(fn, iters=30):
    for _ in range(3): fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us

res = []
for li in range(10):
    K, N = widths[li], widths[li + 1]
    Kp, Np = pad(K), pad(N)
    x = torch.randn(Mp, Kp, device=dev).bfloat16()
    w = torch.randn(Np, Kp, device=dev).bfloat16() * 0.02
    b = torch.zeros(Np, device=dev)
    y = torch.empty(Mp, Np, device=dev, dtype=torch.bfloat16)
    st = torch.empty(Mp // 32, 2, Np, device=dev)
    dz = torch.randn(Mp, Np, device=dev).bfloat16()
    dx = torch.empty(Mp, Kp, device=dev, dtype=torch.bfloat16)
    dw = torch.empty(Np, Kp, device=dev)
    shapes = {
        "fwd": (lambda: call("mmad_fc_fwd", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1, 0.2,
                             None, None, ptr(y), ptr(st), s), 2.0 * B * K * N),
        "bwd_data": (lambda: call("mmad_fc_bwd_data", 1, B, N, K, Mp, Np, Kp, ptr(dz), ptr(w), ptr(dx),
                                  None, s), 2.0 * B * K * N),
        "bwd_w": (lambda: call("mmad_fc_bwd_weight", 1, Mp, Np, Kp, ptr(dz), ptr(x), ptr(dw), s),
                  2.0 * B * K * N),
    }
    for kind, (fn, flops) in shapes.items():
        best = None
        for tile in (-1, 0, 1, 2):
            for gm in (-1, 1, 2, 4, 8, 16):
                if tile == -1 and gm != -1:
                    continue
                lib.mmad_tune_set(0, tile); lib.mmad_tune_set(1, gm)
                us = timeit(fn)
                r = dict(layer=li, kind=kind, K=K, N=N, tile=tile, gm=gm, us=round(us, 2),
                         tflops=round(flops / us / 1e6, 1))
                res.append(r)
                if best is None or us < best["us"]:
                    best = r
        auto = [r for r in res if r["layer"] == li and r["kind"] == kind and r["tile"] == -1][0]
        print(f"L{li} {kind:8s} {K:5d}->{N:5d} auto {auto['us']:7.2f}us {auto['tflops']:6.1f}TF | best tile={best['tile']} gm={best['gm']} {best['us']:7.2f}us {best['tflops']:6.1f}TF", flush=True)
lib.mmad_tune_set(0, -1); lib.mmad_tune_set(1, -1)
json.dump(res, open("gpurun_out/gemm_sweep.json", "w"))
