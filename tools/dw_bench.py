"""Microbenchmark of the dW GEMM (+ fused Adam) for one layer shape, per tile
configuration: GEMM only (mmad_fc_bwd_weight), fused dW+Adam
(mmad_fc_bwd_weight_adam), and the flat Adam pass (mmad_adam) over the same
parameters.  Prints one JSON line per variant.
Usage: python tools/dw_bench.py [--batch 1024] [--nout 1658] [--nin 2048] [--iters 20]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from icra2021_multimodal_ad_amd import _native  # noqa: E402
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad, BF16  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--nout", type=int, default=1658)
    ap.add_argument("--nin", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cfgs", default="0,1,2,3,4,5")
    a = ap.parse_args()
    lib = _native.load()
    dev = torch.device("cuda", 0)
    M, N, K = a.batch, a.nout, a.nin
    Mp, Np, Kp = pad(M), pad(N), pad(K)
    g = torch.Generator(device=dev).manual_seed(0)
    dz = torch.zeros(Mp, Np, device=dev, dtype=torch.bfloat16)
    dz[:M, :N] = torch.randn(M, N, device=dev, generator=g).bfloat16()
    x = torch.zeros(Mp, Kp, device=dev, dtype=torch.bfloat16)
    x[:M, :K] = torch.randn(M, K, device=dev, generator=g).bfloat16()
    p = torch.zeros(Np, Kp, device=dev)
    p[:N, :K] = torch.randn(N, K, device=dev, generator=g) * 0.02
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    sh = torch.zeros(Np, Kp, device=dev, dtype=torch.bfloat16)
    dw = torch.empty(Np, Kp, device=dev)
    s = stream_ptr()
    nparam = N * K
    adam_bytes = 26 * nparam + 2 * M * (N + K)
    flops = 2.0 * M * N * K
    for cfg in [int(c) for c in a.cfgs.split(",")]:
        lib.mmad_tune_set(0, cfg)
        lib.mmad_tune_set(5, cfg)
        try:
            t_g = timed(lambda: call("mmad_fc_bwd_weight", BF16, Mp, Np, Kp, ptr(dz), ptr(x), ptr(dw), s),
                        a.iters)
            t_f = timed(lambda: call("mmad_fc_bwd_weight_adam", BF16, Mp, Np, Kp, ptr(dz), ptr(x), ptr(p),
                                     ptr(m), ptr(v), ptr(sh), None, 0.9, 0.999, 1e-8, 1e-3, 1.0, s),
                        a.iters)
        except _native.NativeError as e:
            print(json.dumps({"cfg": cfg, "error": str(e)}))
            continue
        finally:
            lib.mmad_tune_set(0, -1)
            lib.mmad_tune_set(5, -2)
        print(json.dumps({"shape": [M, N, K], "cfg": cfg, "gemm_us": round(t_g, 2),
                          "gemm_tflops": round(flops / t_g / 1e6, 1), "fused_us": round(t_f, 2),
                          "fused_gbs": round(adam_bytes / t_f / 1e3, 1)}), flush=True)
    t_a = timed(lambda: call("mmad_adam", Np * Kp, ptr(p), ptr(dw), ptr(m), ptr(v), 0.9, 0.999, 1e-8,
                             1e-3, 1.0, ptr(sh), Np * Kp, s), a.iters)
    print(json.dumps({"flat_adam_us": round(t_a, 2), "flat_adam_gbs": round(30 * Np * Kp / t_a / 1e3, 1)}))


if __name__ == "__main__":
    main()
