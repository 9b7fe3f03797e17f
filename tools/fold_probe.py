"""The train-mode BN fold (bn_fold_k: batch statistics -> scale / shift,
W' = W diag(scale) in bf16, sum_k shift[k] W[n][k] partials) at the c3 shapes,
timed three ways: back-to-back launches of the fold alone; fold after the
producer's forward GEMM (the in-step pair: GEMM -> fold, the fold's time from
the pair minus the GEMM alone); and the stats-merge share (the same launches
with the statistics of a 32-row batch, i.e. one partial per column).
Usage: python tools/fold_probe.py [batch=4096]"""
import ctypes
import json
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

from icra2021_multimodal_ad_amd import _native  # noqa: E402
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad  # noqa: E402
from icra2021_multimodal_ad_amd.common_utils import ae_widths  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dev = torch.device("cuda", 0)
lib = _native.load()
fold = lib._Z21mmad_bn_finalize_foldiiiiiPKfS0_S0_PfS1_ffS1_S1_S1_S1_S0_iPvS1_S2_
fold.restype = ctypes.c_int
P = ctypes.c_void_p
fold.argtypes = [ctypes.c_int] * 5 + [P] * 5 + [ctypes.c_float] * 2 + [P] * 5 + [ctypes.c_int, P, P, P]
s = stream_ptr()
enc, dec = ae_widths(2048, 100, 5, enc_out=200)
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


for li in range(3):                       # producer layers 0..2 (their consumers 1..3)
    K, N = enc[li], enc[li + 1]
    Nc = enc[li + 2]
    Kp, Np, Ncp = pad(K), pad(N), pad(Nc)
    x = torch.randn(Mp, Kp, device=dev).bfloat16()
    w = (torch.randn(Np, Kp, device=dev) * 0.02).bfloat16()
    b = torch.zeros(Np, device=dev)
    a = torch.empty(Mp, Np, device=dev, dtype=torch.bfloat16)
    stats = torch.empty(Mp // 32, 2, Np, device=dev)
    g = torch.ones(Np, device=dev)
    be = torch.zeros(Np, device=dev)
    rm, rv = torch.zeros(Np, device=dev), torch.ones(Np, device=dev)
    sm, sr, sc, sh = (torch.empty(Np, device=dev) for _ in range(4))
    W = torch.randn(Ncp, Np, device=dev) * 0.02
    wout = torch.empty(Ncp, Np, device=dev, dtype=torch.bfloat16)
    cpart = torch.empty(Np // 64, Ncp, device=dev)

    def gemm():
        call("mmad_fc_fwd", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1, 0.2, None, None, ptr(a),
             ptr(stats), s)

    def fold_only(m=B):
        rc = fold(1, m, N, pad(m) if m < Mp else Mp, Np, ptr(stats), ptr(g), ptr(be), ptr(rm), ptr(rv), 0.1, 1e-5,
                  ptr(sm), ptr(sr), ptr(sc), ptr(sh), ptr(W), Ncp, ptr(wout), ptr(cpart), s)
        assert rc == 0, _native.last_error()

    def pair():
        gemm()
        fold_only()
    gemm()
    torch.cuda.synchronize()
    t_gemm = timeit(gemm)
    t_fold = timeit(fold_only)
    t_pair = timeit(pair)
    t_fold_1part = timeit(lambda: fold_only(128))
    print(json.dumps({"producer_layer": li, "shape": f"{B}x{K}->{N}, consumer {Nc}", "gemm_us": round(t_gemm, 2),
                      "fold_alone_us": round(t_fold, 2), "pair_us": round(t_pair, 2),
                      "fold_in_pair_us": round(t_pair - t_gemm, 2),
                      "fold_128_rows_us": round(t_fold_1part, 2),
                      "fold_bytes": Ncp * Np * 6 + Mp // 32 * 2 * Np * 4}), flush=True)
