"""Back-to-back launches of ONE Adam-fused dW GEMM (mmad_fc_bwd_weight_adam)
at a bench shape, for rocprofv3 PMC passes.  The Adam state rotates over
enough buffer sets (> the 256 MiB Infinity Cache) that every launch streams
p / m / v from HBM as in the train step.
Usage: python tools/dw_one.py [batch=1024] [nout=1658] [nin=2048] [launches=40] [tile=3]"""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

from icra2021_multimodal_ad_amd import _native  # noqa: E402
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad, BF16  # noqa: E402

B, N, K = (int(a) for a in (sys.argv[1:4] + ["1024", "1658", "2048"][len(sys.argv[1:4]):]))
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 40
tile = int(sys.argv[5]) if len(sys.argv) > 5 else 3
dev = torch.device("cuda", 0)
lib = _native.load()
Mp, Np, Kp = pad(B), pad(N), pad(K)
dz = torch.randn(Mp, Np, device=dev).bfloat16()
x = torch.randn(Mp, Kp, device=dev).bfloat16()
per_set = Np * Kp * 14            # p, m, v fp32 + bf16 shadow
nsets = max(2, int(3 * 256 * 2**20 // per_set) + 1)
sets = [(torch.randn(Np, Kp, device=dev) * 0.02, torch.zeros(Np, Kp, device=dev),
         torch.zeros(Np, Kp, device=dev), torch.zeros(Np, Kp, device=dev, dtype=torch.bfloat16))
        for _ in range(nsets)]
s = stream_ptr()
lib.mmad_tune_set(5, tile)
for i in range(iters):
    p, m, v, sh = sets[i % nsets]
    call("mmad_fc_bwd_weight_adam", BF16, Mp, Np, Kp, ptr(dz), ptr(x), ptr(p), ptr(m), ptr(v), ptr(sh),
         None, 0.9, 0.999, 1e-8, 1e-3, 1.0, s)
torch.cuda.synchronize()
print(f"dw_one B={B} N={N} K={K} tile={tile} launches={iters} sets={nsets}")
