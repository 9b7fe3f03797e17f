"""Per-launch HBM traffic of the roofline GEMM from the three rocprofv3 PMC
passes of tools/gpu_profile_round.sh (FETCH_SIZE, WRITE_SIZE, TCC hit/miss),
with the gfx950 FETCH_SIZE x2 correction; writes profiles/<tag>_pmc_traffic.json.
Usage: python tools/pmc_traffic.py <tag>"""
import collections
import json
import sqlite3
import statistics
import sys

tag = sys.argv[1]
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
d = {"kernel": "mmad_gemm_kernel fwd, encoder layer 1 (1024x2048 . 1658x2048^T, bf16), autotuned tile",
     "workload": {"dim": 2048, "batch": 1024, "dtype": "bf16"},
     "command": "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE | --pmc TCC_HIT_sum TCC_MISS_sum "
                "(separate passes, tools/gpu_profile_round.sh) -- python3 tools/gemm_one.py fwd 0 1024 40",
     "FETCH_SIZE_KB_median": f, "WRITE_SIZE_KB_median": w, "TCC_HIT_sum": hit, "TCC_MISS_sum": miss,
     "l2_hit_rate": round(hit / (hit + miss), 4),
     "correction": "gfx950: FETCH_SIZE reports half the bytes of 16-B/lane streaming reads "
                   "(MI355X_MICROARCH.md HBM section) -> x2; WRITE_SIZE exact for 16-B stores",
     "traffic_bytes_per_launch": int((2 * f + w) * 1024),
     "algorithmic_bytes_per_launch": 14853120,
     "note": "memory-side bytes include Infinity-Cache hits: each XCD fetches its own copy of its "
             "A/B panels (8 L2s), ~2.8x the compulsory bytes"}
json.dump(d, open(f"profiles/{tag}_pmc_traffic.json", "w"), indent=1)
print(d["traffic_bytes_per_launch"], d["l2_hit_rate"])
