"""The BN-backward apply kernel (bn_bwd_apply_k: dz = act'(a) * gamma rstd / M
(M dy - sum dy - xhat sum dy xhat) from the bwd-data epilogue's fp64 column
partials) at the c3 shapes, alone: back-to-back launches with the 4096-row
batch's 64 partials per column and with 2 (the merge's share), against the
bytes it must move (dy, a in; dz out; bf16).
Usage: python tools/apply_probe.py [batch=4096]"""
import ctypes
import json
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

from icra2021_multimodal_ad_amd import _native  # noqa: E402
from icra2021_multimodal_ad_amd._native import ptr, stream_ptr, pad  # noqa: E402
from icra2021_multimodal_ad_amd.common_utils import ae_widths  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dev = torch.device("cuda", 0)
lib = _native.load()
fn = lib._Z21mmad_bn_act_bwd_applyiifiiiiPKvS0_PKfS2_S2_PKdiPvPfS6_S6_S5_
fn.restype = ctypes.c_int
P = ctypes.c_void_p
fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_float] + [ctypes.c_int] * 4 + [P] * 6 + [ctypes.c_int] + [P] * 5
s = stream_ptr()
enc, dec = ae_widths(2048, 100, 5, enc_out=200)
Mp = pad(B)


def timeit(f, iters=50):
    for _ in range(5):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for N in (enc[1], dec[4], enc[3]):          # 1678, 1658, 939 columns
    Np = pad(N)
    dy = torch.randn(Mp, Np, device=dev).bfloat16()
    a = torch.randn(Mp, Np, device=dev).bfloat16()
    mean, rstd, gamma = torch.zeros(Np, device=dev), torch.ones(Np, device=dev), torch.ones(Np, device=dev)
    part = torch.randn(Mp // 64, 2, Np, device=dev, dtype=torch.float64)
    dz = torch.empty(Mp, Np, device=dev, dtype=torch.bfloat16)
    dg, db = torch.empty(Np, device=dev), torch.empty(Np, device=dev)
    dbp = torch.empty(Mp // 128, Np, device=dev)

    def run(nparts):
        rc = fn(1, 1, 0.2, B, N, Mp, Np, ptr(dy), ptr(a), ptr(mean), ptr(rstd), ptr(gamma), ptr(part), nparts,
                ptr(dz), ptr(dg), ptr(db), ptr(dbp), s)
        assert rc == 0, _native.last_error()
    row = {"cols": N, "rows": B, "bytes": Mp * Np * 6}
    for rb in (1, 2, 4):
        lib.mmad_tune_set(13, rb)          # row slabs per block (the partials merged once per block)
        t64 = timeit(lambda: run(Mp // 64))
        t2 = timeit(lambda: run(2))
        row[f"rb{rb}_us"] = round(t64, 2)
        row[f"rb{rb}_2parts_us"] = round(t2, 2)
        row[f"rb{rb}_tb_s"] = round(row["bytes"] / (t64 * 1e-6) / 1e12, 2)
    lib.mmad_tune_set(13, 2)
    print(json.dumps(row), flush=True)
