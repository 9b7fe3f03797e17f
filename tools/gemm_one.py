"""Run one GEMM shape repeatedly (for rocprofv3 PMC passes).
Usage: python tools/gemm_one.py [kind=fwd|bwd_data|bwd_w] [layer=0] [batch=1024] [iters=20] [tile=-1] [gm=-1] [model=ae|vib_ae]"""
import sys
sys.path.insert(0, ".")
import torch
from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad

kind = sys.argv[1] if len(sys.argv) > 1 else "fwd"
li = int(sys.argv[2]) if len(sys.argv) > 2 else 0
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
tile = int(sys.argv[5]) if len(sys.argv) > 5 else -1
gm = int(sys.argv[6]) if len(sys.argv) > 6 else -1
model = sys.argv[7] if len(sys.argv) > 7 else "ae"
from icra2021_multimodal_ad_amd.common_utils import ae_widths
enc, dec = ae_widths(2048, 100, 5, enc_out=200 if model == "vib_ae" else None)   # VIB: mu | log-var
widths = enc + dec[1:]
K, N = widths[li], widths[li + 1]
Kp, Np, Mp = pad(K), pad(N), pad(B)
dev = torch.device("cuda", 0)
lib = _native.load()
_native.enable_gemm_workspace(dev)
lib.mmad_tune_set(0, tile)
lib.mmad_tune_set(1, gm)
x = torch.randn(Mp, Kp, device=dev).bfloat16()
w = (torch.randn(Np, Kp, device=dev) * 0.02).bfloat16()
b = torch.zeros(Np, device=dev)
y = torch.empty(Mp, Np, device=dev, dtype=torch.bfloat16)
st = torch.empty(Mp // 32, 2, Np, device=dev)
dz = torch.randn(Mp, Np, device=dev).bfloat16()
dx = torch.empty(Mp, Kp, device=dev, dtype=torch.bfloat16)
dw = torch.empty(Np, Kp, device=dev)
s = stream_ptr()
for _ in range(iters):
    if kind == "fwd":
        call("mmad_fc_fwd", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1, 0.2, None, None, ptr(y), ptr(st), s)
    elif kind == "bwd_data":
        call("mmad_fc_bwd_data", 1, B, N, K, Mp, Np, Kp, ptr(dz), ptr(w), ptr(dx), None, s)
    else:
        call("mmad_fc_bwd_weight", 1, Mp, Np, Kp, ptr(dz), ptr(x), ptr(dw), s)
torch.cuda.synchronize()
print("done", kind, li, B, "unique MB", (Mp * Kp + Np * Kp) * 2 / 1e6)
