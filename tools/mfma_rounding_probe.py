"""Signed-error statistics of this build's fp32 GEMM (v_mfma_f32_16x16x4_f32,
the exact-fp32 parity path) and bf16 GEMM (v_mfma_f32_16x16x32_bf16, fp32
accumulate) against a float64 reference of the same contraction, beside
torch-CPU fp32 (BLAS) as the control: a rounding mode other than
round-to-nearest-even inside the MFMA accumulation would show as a mean
signed error many standard errors from zero (|y| biased toward zero for
truncation).  Probe for DESIGN.md section 5 (the loss-EMA offset).
Usage: python tools/mfma_rounding_probe.py [M=4096] [N=1024] [K=1728]"""
import sys

sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from icra2021_multimodal_ad_amd import _native  # noqa: E402
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad, F32, BF16  # noqa: E402

M, N, K = (int(a) for a in (sys.argv[1:4] + ["4096", "1024", "1728"][len(sys.argv[1:4]):]))
dev = torch.device("cuda", 0)
_native.load()
_native.enable_gemm_workspace(dev)
Mp, Np, Kp = pad(M), pad(N), pad(K)
g = torch.Generator().manual_seed(3)
out = {}
for dt_name, dt, tdt in (("f32", F32, torch.float32), ("bf16", BF16, torch.bfloat16)):
    x = torch.zeros(Mp, Kp)
    w = torch.zeros(Np, Kp)
    x[:M, :K] = torch.randn(M, K, generator=g)
    w[:N, :K] = torch.randn(N, K, generator=g) * 0.05
    xq, wq = x.to(tdt), w.to(tdt)                        # the operands the GPU sees
    ref = (xq.double()[:M, :K] @ wq.double()[:N, :K].T)  # exact products, fp64 sums
    y = torch.empty(Mp, Np, device=dev, dtype=torch.float32 if dt == F32 else torch.bfloat16)
    xd, wd = xq.to(dev), wq.to(dev)                      # kept alive until the sync below
    if dt == F32:
        call("mmad_fc_fwd", dt, M, N, K, Mp, Np, Kp, ptr(xd), ptr(wd), None, 0, 0.0, None,
             None, ptr(y), None, stream_ptr())
        gpu = y.float().cpu().double()[:M, :N]
    else:
        # the bf16 output rounds the fp32 accumulator once (RNE): a biased
        # accumulation shows as more outputs rounded the biased way
        yb = torch.empty(Mp, Np, device=dev, dtype=torch.bfloat16)
        rows = torch.empty(Np // 128, Mp, device=dev)
        diff = torch.zeros(M, N, device=dev)
        zref = torch.zeros(Mp, Np, device=dev, dtype=torch.bfloat16)
        call("mmad_fc_fwd_score", dt, M, N, K, Mp, Np, Kp, ptr(xd), ptr(wd), None, 0, 0.0,
             None, None, ptr(yb), ptr(zref), ptr(rows), ptr(diff), N, stream_ptr())
        torch.cuda.synchronize()
        gpu = yb.float().cpu().double()[:M, :N]           # bf16-rounded output (RNE in the epilogue)
        ref = ref.to(torch.bfloat16).double()             # the exact sum rounded the same way
    torch.cuda.synchronize()
    cpu = (xq.float()[:M, :K] @ wq.float()[:N, :K].T).double()
    for name, val in (("gpu", gpu), ("torch_cpu_fp32", cpu)):
        e = (val - ref)
        se = (e * torch.sign(ref)).numpy().ravel()          # positive = |y| too large
        nz = se[se != 0]
        out[(dt_name, name)] = (float(se.mean()), float(se.std() / np.sqrt(se.size)),
                                int((nz > 0).sum()), int((nz < 0).sum()), float(np.abs(e.numpy()).max()))
for k, (m, sem, pos, neg, mx) in out.items():
    print(f"{k[0]:4s} {k[1]:15s} mean signed |y| error {m:+.3e} (s.e. {sem:.1e}, {m / sem if sem else 0:+.1f} s.e.); "
          f"|y| too large {pos}, too small {neg}; max abs err {mx:.2e}")
