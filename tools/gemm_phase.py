"""Where a GEMM launch's time goes: back-to-back launches of one layer's
forward / bwd-data / dW GEMM with the diagnostic bits of tuning knob 3
(1 = skip the main loop, 2 = skip the epilogue): full, prologue+epilogue,
prologue+loop, prologue only.  Usage: python tools/gemm_phase.py [batch=1024] [layers=0,3,4] [tiles=3,0]"""
import json
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

from icra2021_multimodal_ad_amd import _native  # noqa: E402
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
widths = [2048, 1658, 1268, 879, 489, 100, 489, 879, 1268, 1658, 2048]
layers = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,3,4").split(",")]
tiles = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "3,0").split(",")]
dev = torch.device("cuda", 0)
lib = _native.load()
s = stream_ptr()
Mp = pad(B)


def timeit(fn, iters=50):
    for _ in range(5):
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
        "fwd_nostats": lambda: call("mmad_fc_fwd", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1,
                                    0.2, None, None, ptr(y), None, s),
        "fwd_noact_nostats": lambda: call("mmad_fc_fwd", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), None,
                                          0, 0.0, None, None, ptr(y), None, s),
        "bwd_data": lambda: call("mmad_fc_bwd_data", 1, B, N, K, Mp, Np, Kp, ptr(dz), ptr(w), ptr(dx),
                                 None, s),
        "bwd_w": lambda: call("mmad_fc_bwd_weight", 1, Mp, Np, Kp, ptr(dz), ptr(x), ptr(dw), s),
    }
    kinds = sys.argv[4].split(",") if len(sys.argv) > 4 else list(fns)
    for kind in kinds:
        fn = fns[kind]
        for tile in tiles:
            lib.mmad_tune_set(0, tile)
            row = {"layer": li, "kind": kind, "M": B, "N": N, "K": K, "tile": tile}
            variants = (("full", 0), ("no_loop", 1), ("no_epilogue", 2), ("prologue_only", 3))
            if kind == "fwd":
                variants += (("no_part_store", 8),)
            for name, bits in variants:
                lib.mmad_tune_set(3, bits)
                row[name] = round(timeit(fn), 2)
            lib.mmad_tune_set(3, 0)
            print(json.dumps(row), flush=True)
    lib.mmad_tune_set(0, -1)
