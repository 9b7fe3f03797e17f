"""Median per-dispatch value of every PMC counter of the mmad_gemm kernels in
one or more rocprofv3 SQLite outputs.  Usage: python tools/pmc_dump.py <db>..."""
import collections
import sqlite3
import statistics
import sys

for db in sys.argv[1:]:
    c = sqlite3.connect(db)
    names = dict(c.execute("select dispatch_id, name from kernels").fetchall())
    vals = collections.defaultdict(list)
    for d, n, v in c.execute("select dispatch_id, counter_name, sum(counter_value) from pmc_events "
                             "group by dispatch_id, counter_name"):
        if "mmad_gemm_kernel" in names.get(d, ""):
            vals[n].append(v)
    print(db)
    for n in sorted(vals):
        print(f"  {n:28s} n={len(vals[n]):3d} median={statistics.median(vals[n]):14.1f}")
