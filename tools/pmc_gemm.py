"""Summarise the rocprofv3 passes of ONE roofline GEMM into
profiles/<tag>_pmc_<kind>.json, the file bench.py / bench_score.py read for
`traffic` and (encoder GEMM) the MFMA-busy fraction.

Passes (each its own rocprofv3 run, tools/gpu_pmc.sh):
  <tag>_pmc_fetch  FETCH_SIZE            (gfx950: x2 for 16-B/lane streaming reads)
  <tag>_pmc_write  WRITE_SIZE
  <tag>_pmc_hit    TCC_HIT_sum TCC_MISS_sum
  <tag>_pmc_mfma   SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
  <tag>_trace      --kernel-trace (durations of the same launches, no counters)

MFMA accounting (MI355X_MICROARCH.md, rocprofv3 / constants rows):
SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles, 16 per v_mfma_f32_16x16x32_bf16
(the check `mfma_busy_over_issued` compares it with the MFMAs the padded
problem issues); the busy fraction is busy / (1024 SIMDs x cycles), with
cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs; reads high on
dispatches shorter than ~0.3 ms) and, independently, the kernel-trace
duration x 2.4 GHz (the max clock: a lower bound on the fraction).

Usage: python tools/pmc_gemm.py <kind> <tag> <batch> <model> [extra-json]
  kind = traffic (encoder layer-1 forward) | dw (layer-0 dW + Adam) | score"""
import collections
import json
import os
import sqlite3
import statistics
import sys

sys.path.insert(0, ".")
from bench import src_sha16  # noqa: E402
from icra2021_multimodal_ad_amd.common_utils import ae_widths  # noqa: E402
from icra2021_multimodal_ad_amd._native import pad  # noqa: E402

kind, tag, B, model = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
extra = json.loads(sys.argv[5]) if len(sys.argv) > 5 else {}
enc, dec = ae_widths(2048, 100, 5, enc_out=200 if model == "vib_ae" else None)
if kind == "score":
    K, N = dec[-2], dec[-1]
else:
    K, N = enc[0], enc[1]
Kp, Np, Mp = pad(K), pad(N), pad(B)


def medians(pass_name):
    path = f"gpurun_out/{tag}_pmc_{pass_name}/run_results.db"
    if not os.path.exists(path):
        return {}
    c = sqlite3.connect(path)
    names = dict(c.execute("select dispatch_id, name from kernels").fetchall())
    vals = collections.defaultdict(list)
    for d, n, v in c.execute("select dispatch_id, counter_name, sum(counter_value) from pmc_events "
                             "group by dispatch_id, counter_name order by dispatch_id"):
        if "mmad_gemm" in names.get(d, ""):
            vals[n].append(v)
    # skip the autotune / warm launches
    return {n: statistics.median(v[3:] if len(v) > 6 else v) for n, v in vals.items()}


med = {}
for p in ("fetch", "write", "hit", "mfma"):
    med.update(medians(p))
dur_us = None
tpath = f"gpurun_out/{tag}_trace/run_results.db"
if os.path.exists(tpath):
    c = sqlite3.connect(tpath)
    ds = [d for n, d in c.execute("select name, duration from kernels order by start") if "mmad_gemm" in n]
    ds = ds[3:] if len(ds) > 6 else ds
    dur_us = statistics.median(ds) / 1e3 if ds else None

flops = 2.0 * B * K * N
if kind == "traffic":
    what = f"forward, encoder layer 1 ({B}x{K} . {N}x{K}^T, bf16; bias + LeakyReLU + BN-stat epilogue)"
    alg = 2 * (B * K + N * K + B * N) + (B // 32) * 2 * N * 4
    wl = {"dim": K, "batch": B, "dtype": "bf16"}
    cmd = f"python3 tools/gemm_one.py fwd 0 {B} 40 -1 -1 {model}"
elif kind == "dw":
    what = f"bwd-weight + fused Adam (dW[{N}x{K}] over {B} windows, bf16)"
    alg = 26 * N * K + 2 * B * (N + K)
    wl = {"dim": K, "batch": B, "dtype": "bf16", "model": model, "layer": 0}
    cmd = f"python3 tools/dw_one.py {B} {N} {K} 40 -2 (Adam state rotated over > 256 MiB: cold, as in the step)"
else:
    what = f"score, last decoder layer ({B}x{K} . {N}x{K}^T, bf16; y stored, sum (y - ref)^2 row partials)"
    alg = 2 * (B * Kp + Np * Kp) + 2 * B * Np + 2 * B * Np + (Np // 128) * B * 4
    wl = {"dim": 2048, "batch": B, "dtype": "bf16", "kind": "score"}
    cmd = f"python3 tools/score_one.py {B} 20"
d = {"kernel": f"mmad_gemm {what}", "workload": wl,
     "src_sha16": src_sha16(kind),
     "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | TCC_HIT_sum TCC_MISS_sum | "
                "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE | --kernel-trace (separate passes, "
                f"tools/gpu_pmc.sh) -- {cmd}",
     "algorithmic_bytes_per_launch": alg, "flops_per_launch": flops}
d.update({k: med.get(k) for k in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum",
                                  "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE")})
d["correction"] = ("gfx950: FETCH_SIZE (KB) reports half the bytes of 16-B/lane streaming reads -> x2; "
                   "WRITE_SIZE exact for 16-B stores (MI355X_MICROARCH.md HBM section)")
if med.get("FETCH_SIZE") is not None and med.get("WRITE_SIZE") is not None:
    d["traffic_bytes_per_launch"] = int((2 * med["FETCH_SIZE"] + med["WRITE_SIZE"]) * 1024)
    d["traffic_over_algorithmic"] = round(d["traffic_bytes_per_launch"] / alg, 3)
if med.get("TCC_HIT_sum") is not None:
    d["l2_hit_rate"] = round(med["TCC_HIT_sum"] / (med["TCC_HIT_sum"] + med["TCC_MISS_sum"]), 4)
if dur_us is not None:
    d["kernel_trace_median_us"] = round(dur_us, 2)
    d["achieved_tflops_trace"] = round(flops / (dur_us * 1e-6) / 1e12, 1)
busy = med.get("SQ_VALU_MFMA_BUSY_CYCLES")
if busy:
    # SIMD cycles of the padded problem's MFMAs: Mp*Np*Kp / (16*16*32) of them, 16 each
    issued = Mp * Np * Kp / (16 * 16 * 32) * 16
    d["mfma_issued_cycles"] = issued
    d["mfma_busy_over_issued"] = round(busy / issued, 4)
    gr = med.get("GRBM_GUI_ACTIVE")
    if gr:
        d["mfma_busy_frac_grbm"] = round(busy / (1024 * gr / 8), 4)
        if dur_us:
            d["effective_clock_ghz_grbm"] = round(gr / 8 / (dur_us * 1e3), 3)
    if dur_us:
        d["mfma_busy_frac_at_2p4ghz"] = round(busy / (1024 * 2.4e3 * dur_us), 4)
d.update(extra)
json.dump(d, open(f"profiles/{tag}_pmc_{kind}.json", "w"), indent=1)
print(json.dumps(d))
