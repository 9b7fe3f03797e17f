"""Median per-dispatch PMC counter value per (kernel, grid) from rocprofv3
SQLite outputs, for the non-GEMM kernels of a step (BN fold / apply, pack, ...).
FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 units).
Usage: python tools/pmc_by_kernel.py <dir-or-db>..."""
import collections
import glob
import os
import re
import sqlite3
import statistics
import sys


def short(n):
    m = re.search(r"(bn_\w+_k|pack_input_k|vib_\w+_k|reduce_jobs_k|matrix_colsum_k|adam\w*_k)", n)
    return m.group(1) if m else n[:40]


for arg in sys.argv[1:]:
    dbs = [arg] if arg.endswith(".db") else glob.glob(os.path.join(arg, "**", "*.db"), recursive=True)
    for db in dbs:
        c = sqlite3.connect(db)
        kcols = [r[1] for r in c.execute("pragma table_info(kernels)")]
        gcol = "grid_size" if "grid_size" in kcols else ("grid_size_x" if "grid_size_x" in kcols else None)
        q = f"select dispatch_id, name{', ' + gcol if gcol else ''} from kernels"
        meta = {r[0]: (r[1], r[2] if gcol else 0) for r in c.execute(q)}
        vals = collections.defaultdict(list)
        for d, n, v in c.execute("select dispatch_id, counter_name, sum(counter_value) from pmc_events "
                                 "group by dispatch_id, counter_name"):
            name, grid = meta.get(d, ("?", 0))
            if "mmad_gemm_kernel" in name:
                continue
            vals[(short(name), grid, n)].append(v)
        print(db)
        for k in sorted(vals):
            print(f"  {k[0]:22s} grid={k[1]:8d} {k[2]:12s} n={len(vals[k]):3d} median={statistics.median(vals[k]):12.1f}")
