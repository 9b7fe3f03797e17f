"""Average duration of one GEMM shape (HIP events over back-to-back launches)
with a forced tile configuration; prints us and TFLOP/s.
Usage: python tools/gemm_time.py kind layer batch tile [iters=50]"""
import sys
sys.path.insert(0, ".")
import torch
from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad

kind, li, B, tile = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 50
widths = [2048, 1658, 1268, 879, 489, 100, 489, 879, 1268, 1658, 2048]
K, N = widths[li], widths[li + 1]
Kp, Np, Mp = pad(K), pad(N), pad(B)
dev = torch.device("cuda", 0)
lib = _native.load()
lib.mmad_tune_set(0, tile)
x = torch.randn(Mp, Kp, device=dev).bfloat16()
w = (torch.randn(Np, Kp, device=dev) * 0.02).bfloat16()
b = torch.zeros(Np, device=dev)
y = torch.empty(Mp, Np, device=dev, dtype=torch.bfloat16)
st = torch.empty(Mp // 32, 2, Np, device=dev)
dz = torch.randn(Mp, Np, device=dev).bfloat16()
dx = torch.empty(Mp, Kp, device=dev, dtype=torch.bfloat16)
dw = torch.empty(Np, Kp, device=dev)
s = stream_ptr()


def launch():
    if kind == "fwd":
        call("mmad_fc_fwd", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1, 0.2, None, None, ptr(y), ptr(st), s)
    elif kind == "bwd_data":
        call("mmad_fc_bwd_data", 1, B, N, K, Mp, Np, Kp, ptr(dz), ptr(w), ptr(dx), None, s)
    else:
        call("mmad_fc_bwd_weight", 1, Mp, Np, Kp, ptr(dz), ptr(x), ptr(dw), s)


for _ in range(5):
    launch()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    launch()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / iters
print(f"{kind} layer {li} B={B} M={Mp} N={Np} K={Kp} tile={tile}: {us:.2f} us, "
      f"{2.0 * B * N * K / us / 1e6:.1f} TFLOP/s", flush=True)
