"""Per-launch HBM traffic of the c5 roofline kernel (tools/score_one.py) from
three rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE, TCC hit/miss), gfx950
FETCH_SIZE x2 correction; writes profiles/<tag>_pmc_score.json, which
bench_score.py reads for the c5 roofline's `traffic`.
Usage: python tools/pmc_score.py <tag> [batch=65536]"""
import collections
import json
import sqlite3
import statistics
import sys

tag = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
K, N = 1658, 2048            # last decoder layer of the D=2048 AE (btl 100, 5 layers)
Kp, Np = 1664, 2048
med = {}
for p in ("fetch", "write", "hit"):
    c = sqlite3.connect(f"gpurun_out/{tag}_pmc_{p}/run_results.db")
    names = dict(c.execute("select dispatch_id, name from kernels").fetchall())
    vals = collections.defaultdict(list)
    for d, n, v in c.execute("select dispatch_id, counter_name, sum(counter_value) from pmc_events "
                             "group by dispatch_id, counter_name"):
        if "mmad_gemm_kernel" in names.get(d, ""):
            vals[n].append(v)
    for n, v in vals.items():
        med[n] = statistics.median(v)
f, w = med["FETCH_SIZE"], med["WRITE_SIZE"]
hit, miss = med["TCC_HIT_sum"], med["TCC_MISS_sum"]
alg = 2 * (B * Kp + Np * Kp) + 2 * B * Np + 2 * B * Np + (Np // 128) * B * 4   # x, W; y out, ref in; row partials
d = {"kernel": f"mmad_gemm_kernel score, last decoder layer ({B}x{K} . {N}x{K}^T, bf16; y stored, "
               "sum (y - ref)^2 row partials), autotuned tile",
     "workload": {"dim": 2048, "batch": B, "dtype": "bf16", "kind": "score"},
     "command": "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE | --pmc TCC_HIT_sum TCC_MISS_sum "
                f"(separate passes) -- python3 tools/score_one.py {B} 20",
     "FETCH_SIZE_KB_median": f, "WRITE_SIZE_KB_median": w, "TCC_HIT_sum": hit, "TCC_MISS_sum": miss,
     "l2_hit_rate": round(hit / (hit + miss), 4),
     "correction": "gfx950: FETCH_SIZE reports half the bytes of 16-B/lane streaming reads "
                   "(MI355X_MICROARCH.md HBM section) -> x2; WRITE_SIZE exact for 16-B stores",
     "traffic_bytes_per_launch": int((2 * f + w) * 1024),
     "algorithmic_bytes_per_launch": alg}
d["traffic_over_algorithmic"] = round(d["traffic_bytes_per_launch"] / alg, 3)
json.dump(d, open(f"profiles/{tag}_pmc_score.json", "w"), indent=1)
print(d["traffic_bytes_per_launch"], d["traffic_over_algorithmic"], d["l2_hit_rate"])
