"""Per-launch HBM traffic of the Adam-fused dW GEMM from separate rocprofv3
PMC passes over tools/dw_one.py (FETCH_SIZE, WRITE_SIZE, TCC hit/miss,
MFMA busy), gfx950 FETCH_SIZE x2 correction (MI355X_MICROARCH.md, HBM);
writes profiles/<tag>_pmc_dw.json (read by bench.py for roofline.traffic).
Usage: python tools/pmc_dw.py <tag> <batch> <nout> <nin> <layer> <model>"""
import collections
import json
import sqlite3
import statistics
import sys

tag, B, N, K, layer, model = sys.argv[1], *map(int, sys.argv[2:6]), sys.argv[6]
tile = sys.argv[7] if len(sys.argv) > 7 else "64x64"   # label of the tile dw_one.py ran
med = {}
dur = []
for p in ("fetch", "write", "hit", "mfma"):
    c = sqlite3.connect(f"gpurun_out/{tag}_pmc_{p}/run_results.db")
    names = dict(c.execute("select dispatch_id, name from kernels").fetchall())
    vals = collections.defaultdict(list)
    for d, n, v in c.execute("select dispatch_id, counter_name, sum(counter_value) from pmc_events "
                             "group by dispatch_id, counter_name"):
        if "mmad_gemm_kernel" in names.get(d, ""):
            vals[n].append(v)
    for n, v in vals.items():
        med[n] = statistics.median(v[3:] if len(v) > 6 else v)   # skip the autotune / warm launches

alg = 26 * N * K + 2 * B * (N + K)
d = {"kernel": f"mmad_gemm_kernel bwd-weight + fused Adam (dW[{N}x{K}] over {B} windows, bf16, tile {tile})",
     "workload": {"dim": 2048, "batch": B, "dtype": "bf16", "model": model, "layer": layer},
     "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | TCC_HIT_sum TCC_MISS_sum | "
                "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE (separate passes) -- python3 tools/dw_one.py "
                f"{B} {N} {K} 40 3 (Adam state rotated over > 256 MiB: cold, as in the step)",
     "FETCH_SIZE_KB_median": med.get("FETCH_SIZE"), "WRITE_SIZE_KB_median": med.get("WRITE_SIZE"),
     "TCC_HIT_sum": med.get("TCC_HIT_sum"), "TCC_MISS_sum": med.get("TCC_MISS_sum"),
     "SQ_VALU_MFMA_BUSY_CYCLES": med.get("SQ_VALU_MFMA_BUSY_CYCLES"),
     "GRBM_GUI_ACTIVE": med.get("GRBM_GUI_ACTIVE"),
     "correction": "gfx950: FETCH_SIZE reports half the bytes of 16-B/lane streaming reads -> x2; "
                   "WRITE_SIZE exact for 16-B stores",
     "algorithmic_bytes_per_launch": alg}
if med.get("FETCH_SIZE") is not None and med.get("WRITE_SIZE") is not None:
    d["traffic_bytes_per_launch"] = int((2 * med["FETCH_SIZE"] + med["WRITE_SIZE"]) * 1024)
    d["traffic_over_algorithmic"] = round(d["traffic_bytes_per_launch"] / alg, 3)
if med.get("TCC_HIT_sum") is not None:
    d["l2_hit_rate"] = round(med["TCC_HIT_sum"] / (med["TCC_HIT_sum"] + med["TCC_MISS_sum"]), 4)
json.dump(d, open(f"profiles/{tag}_pmc_dw.json", "w"), indent=1)
print(json.dumps(d))
