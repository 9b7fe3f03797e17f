"""Calibration: time the library GEMM (torch.mm -> hipBLASLt) on every GEMM
shape of the bench AE next to this build's fused GEMM kernels.
Usage: python tools/blas_cmp.py [batch=1024]"""
import sys
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


tot = {"mine": 0.0, "blas": 0.0}
for li in range(10):
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
    xs, ws, dzs = x[:B, :K], w[:N, :K], dz[:B, :N]
    kinds = {
        "fwd": (lambda: call("mmad_fc_fwd", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1, 0.2,
                             None, None, ptr(y), ptr(st), s),
                lambda: torch.mm(xs, ws.t())),
        "bwd_data": (lambda: call("mmad_fc_bwd_data", 1, B, N, K, Mp, Np, Kp, ptr(dz), ptr(w), ptr(dx),
                                  None, s),
                     lambda: torch.mm(dzs, ws)),
        "bwd_w": (lambda: call("mmad_fc_bwd_weight", 1, Mp, Np, Kp, ptr(dz), ptr(x), ptr(dw), s),
                  lambda: torch.mm(dzs.t(), xs)),
    }
    fl = 2.0 * B * K * N
    for kind, (mine, blas) in kinds.items():
        tm, tb = timeit(mine), timeit(blas)
        tot["mine"] += tm
        tot["blas"] += tb
        print(f"L{li} {kind:8s} {K:5d}->{N:5d} mine {tm:7.2f}us {fl / tm / 1e6:6.1f}TF | "
              f"hipblaslt {tb:7.2f}us {fl / tb / 1e6:6.1f}TF", flush=True)
print("total us", {k: round(v, 1) for k, v in tot.items()})
