"""The last decoder layer's MSE-fused GEMM at the c3 shape (4096 windows,
1658 -> 2048, bf16) against the plain forward GEMM of the same shape: whole
launch, and with the diagnostic bit that skips the epilogue (knob 3 = 2), per
tile.  Tells what the MSE epilogue (fp32 target read, dz store, loss / bias
partials) costs beyond the forward epilogue.
Usage: python tools/mse_probe.py [batch=4096] [tiles=2,1,0,9]"""
import json
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

from icra2021_multimodal_ad_amd import _native  # noqa: E402
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
tiles = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "2,1,0,9").split(",")]
K, N = 1658, 2048
Mp, Np, Kp = pad(B), pad(N), pad(K)
dev = torch.device("cuda", 0)
lib = _native.load()
s = stream_ptr()
x = torch.zeros(Mp, Kp, device=dev, dtype=torch.bfloat16)
x[:B, :K] = torch.randn(B, K, device=dev).bfloat16()
w = torch.zeros(Np, Kp, device=dev, dtype=torch.bfloat16)
w[:N, :K] = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
b = torch.zeros(Np, device=dev)
tgt = torch.randn(B, N, device=dev)
y = torch.empty(Mp, Np, device=dev, dtype=torch.bfloat16)
part = torch.empty(Mp // 32, 2, Np, device=dev)


def fwd():
    call("mmad_fc_fwd", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1, 0.2, None, None, ptr(y),
         ptr(part), s)


def mse():
    call("mmad_fc_fwd_mse", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), ptr(tgt), N, 2.0, ptr(y),
         ptr(part), s)


def timeit(fn, iters=40):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for t in tiles:
    lib.mmad_tune_set(0, t)
    row = {"tile": t}
    for name, fn in (("fwd", fwd), ("mse", mse)):
        for dbg, tag in ((0, "full"), (2, "no_epilogue"), (1, "no_loop")):
            lib.mmad_tune_set(3, dbg)
            row[f"{name}_{tag}_us"] = round(timeit(fn), 2)
        lib.mmad_tune_set(3, 0)
    print(json.dumps(row), flush=True)
lib.mmad_tune_set(0, -1)
