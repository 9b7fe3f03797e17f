"""GEMM tile sweep: time every fwd / bwd-data / dW GEMM shape of the
D=2048 bench AE (bf16) for each forced tile config (knob 0; the XCD group
height stays the planner's).  Lines of JSON on stdout.
Usage: python tools/gemm_bench.py [batch] [tiles, e.g. -1+0+1+2+7+8+9+10] [kinds, e.g. fwd+bwd_data]"""
import json
import sys

sys.path.insert(0, ".")
import torch
from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
TILES = [int(t) for t in sys.argv[2].replace("+", ",").split(",")] if len(sys.argv) > 2 else [-1, 0, 1, 2]
KINDS = sys.argv[3].replace("+", ",").split(",") if len(sys.argv) > 3 else ["fwd", "bwd_data", "bwd_w"]
widths = [2048, 1658, 1268, 879, 489, 100, 489, 879, 1268, 1658, 2048]
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
    return e0.elapsed_time(e1) / iters * 1e3  # us


try:
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
        for kind in KINDS:
            fn, flops = shapes[kind]
            ref = None
            for tile in TILES:
                lib.mmad_tune_set(0, tile)
                out = y if kind == "fwd" else (dx if kind == "bwd_data" else dw)
                fn()
                torch.cuda.synchronize()
                same = None
                if ref is None:
                    ref = out.clone()
                else:
                    same = bool(torch.equal(out, ref))
                us = timeit(fn)
                print(json.dumps(dict(B=B, layer=li, kind=kind, K=K, N=N, tile=tile, us=round(us, 2),
                                      tflops=round(flops / us / 1e6, 1), bits_equal_first=same)), flush=True)
finally:
    lib.mmad_tune_set(0, -1)
