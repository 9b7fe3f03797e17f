"""Decompose one GEMM launch: time it per tile config and split factor, whole
kernel vs main loop only (knob 3 = 2: epilogue skipped after the split-K
combine) vs prologue + combine + epilogue only (knob 3 = 1: no K loop).
Usage: python tools/gemm_probe.py [kind=fwd|bwd_data|bwd_w] [layer=0] [batch=1024]"""
import sys
sys.path.insert(0, ".")
import torch
from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad

kind = sys.argv[1] if len(sys.argv) > 1 else "fwd"
li = int(sys.argv[2]) if len(sys.argv) > 2 else 0
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
widths = [2048, 1658, 1268, 879, 489, 100, 489, 879, 1268, 1658, 2048]
K, N = widths[li], widths[li + 1]
Kp, Np, Mp = pad(K), pad(N), pad(B)
dev = torch.device("cuda", 0)
lib = _native.load()
_native.enable_gemm_workspace(dev)
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
        call("mmad_fc_fwd", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1, 0.2, None, None, ptr(y),
             ptr(st), s)
    elif kind == "bwd_data":
        call("mmad_fc_bwd_data", 1, B, N, K, Mp, Np, Kp, ptr(dz), ptr(w), ptr(dx), None, s)
    else:
        call("mmad_fc_bwd_weight", 1, Mp, Np, Kp, ptr(dz), ptr(x), ptr(dw), s)


def timeit(iters=30):
    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        launch()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


fl = 2.0 * B * K * N
print(f"{kind} L{li} {B}x{K}->{N}")
for split in (1, 2, 4):
    for tile in (0, 1, 2, 3, 4, 5):
        lib.mmad_tune_set(0, tile)
        lib.mmad_tune_set(4, split)
        row = []
        for dbg in (0, 2, 1):
            lib.mmad_tune_set(3, dbg)
            row.append(timeit())
        lib.mmad_tune_set(3, 0)
        print(f"  split {split} tile {tile}: full {row[0]:7.2f}us ({fl / row[0] / 1e6:6.1f}TF)  "
              f"loop-only {row[1]:7.2f}us  no-loop {row[2]:7.2f}us", flush=True)
lib.mmad_tune_set(0, -1)
lib.mmad_tune_set(4, 0)
