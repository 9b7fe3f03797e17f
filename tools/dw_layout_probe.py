"""What a K-major dW would cost: the dW contraction dW[N][K] = dz^T a over B
rows, timed (1) as this build runs it (mmad_fc_bwd_weight: both operands
MN-major, transposed on the LDS read; fp32 out, no Adam) and (2) as a plain
K-major GEMM of the same FLOPs (mmad_fc_fwd on dz^T [N][B] and a^T [K][B]
copies: bf16 out, no epilogue work), every tile the dispatcher has, interleaved
in one process.  A probe for the transposed-activation design in DESIGN.md
section 9; not used by the product.
Usage: python tools/dw_layout_probe.py [batch=4096] [nout=1658] [nin=2048] [rounds=5]"""
import statistics
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

from icra2021_multimodal_ad_amd import _native  # noqa: E402
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad, BF16  # noqa: E402

B, N, K = (int(a) for a in (sys.argv[1:4] + ["4096", "1658", "2048"][len(sys.argv[1:4]):]))
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
dev = torch.device("cuda", 0)
lib = _native.load()
_native.enable_gemm_workspace(dev)
Mp, Np, Kp = pad(B), pad(N), pad(K)
dz = torch.randn(Mp, Np, device=dev).bfloat16()
a = torch.randn(Mp, Kp, device=dev).bfloat16()
dzt = dz.t().contiguous()          # [Np][Mp]
at = a.t().contiguous()            # [Kp][Mp]
dw = torch.empty(Np, Kp, device=dev)
y = torch.empty(Np, Kp, device=dev, dtype=torch.bfloat16)
s = stream_ptr()
fl = 2.0 * B * N * K


def timeit(fn, iters=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def mn(tile):
    def f():
        lib.mmad_tune_set(0, tile)
        call("mmad_fc_bwd_weight", BF16, Mp, Np, Kp, ptr(dz), ptr(a), ptr(dw), s)
    return f


def km(tile):
    def f():
        lib.mmad_tune_set(0, tile)
        call("mmad_fc_fwd", BF16, N, K, B, Np, Kp, Mp, ptr(dzt), ptr(at), None, 0, 0.0, None, None,
             ptr(y), None, s)
    return f


arms = {f"mn t{t}": mn(t) for t in (0, 3, 5, 1, 2)}
arms.update({f"km t{t}": km(t) for t in (0, 5, 1, 2, 6)})
res = {k: [] for k in arms}
try:
    for _ in range(rounds):
        for k, f in arms.items():
            res[k].append(timeit(f))
finally:
    lib.mmad_tune_set(0, -1)
print(f"dW {N}x{K} over B={B}: " + " | ".join(
    f"{k} {statistics.median(v):7.2f}us {fl / statistics.median(v) / 1e6:6.1f}TF" for k, v in res.items()))
