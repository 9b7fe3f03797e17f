"""Per-launch HBM traffic of the roofline GEMM from the three rocprofv3 PMC
passes of tools/gpu_profile_round.sh (FETCH_SIZE, WRITE_SIZE, TCC hit/miss),
with the gfx950 FETCH_SIZE x2 correction; writes profiles/<tag>_pmc_traffic.json.
Usage: python tools/pmc_traffic.py <tag> [batch=1024] [model=ae|vib_ae]"""
import collections
import json
import sqlite3
import statistics
import sys

tag = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
model = sys.argv[3] if len(sys.argv) > 3 else "ae"
sys.path.insert(0, ".")
from icra2021_multimodal_ad_amd.common_utils import ae_widths  # noqa: E402
N = ae_widths(2048, 100, 5, enc_out=200 if model == "vib_ae" else None)[0][1]
K = 2048
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
d = {"kernel": f"mmad_gemm_kernel fwd, encoder layer 1 ({B}x{K} . {N}x{K}^T, bf16), autotuned tile",
     "workload": {"dim": K, "batch": B, "dtype": "bf16"},
     "command": "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE | --pmc TCC_HIT_sum TCC_MISS_sum "
                "(separate passes, tools/gpu_profile_round.sh) -- python3 tools/gemm_one.py fwd 0 {B} 40 -1 -1 {model}".format(B=B, model=model),
     "FETCH_SIZE_KB_median": f, "WRITE_SIZE_KB_median": w, "TCC_HIT_sum": hit, "TCC_MISS_sum": miss,
     "l2_hit_rate": round(hit / (hit + miss), 4),
     "correction": "gfx950: FETCH_SIZE reports half the bytes of 16-B/lane streaming reads "
                   "(MI355X_MICROARCH.md HBM section) -> x2; WRITE_SIZE exact for 16-B stores",
     "traffic_bytes_per_launch": int((2 * f + w) * 1024),
     "algorithmic_bytes_per_launch": 2 * (B * K + N * K + B * N) + (B // 32) * 2 * N * 4,   # + BN partials
     "note": "memory-side bytes include Infinity-Cache hits: each XCD's L2 fetches its own copy "
             "of the A/B panels its tiles read"}
d["traffic_over_algorithmic"] = round(d["traffic_bytes_per_launch"] / d["algorithmic_bytes_per_launch"], 3)
json.dump(d, open(f"profiles/{tag}_pmc_traffic.json", "w"), indent=1)
print(d["traffic_bytes_per_launch"], d["l2_hit_rate"])
