"""Median per-dispatch PMC counters per kernel (GEMMs included: this build's
mmad_gemm_kernel<...> by tile configuration, and the library's kernels) from
rocprofv3 SQLite outputs, plus the ratios that read the main loop:
  mfma_frac  = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 4 SIMDs ... ) is
               NOT used (SQ units differ); instead, per wave:
  wait_any / wave_cycles, wait_inst / wave_cycles, active / wave_cycles,
  lds_conflict / lds_idx_active.
Usage: python tools/pmc_kernels.py <dir-or-db>..."""
import collections
import glob
import os
import re
import sqlite3
import statistics
import sys


def short(n):
    m = re.search(r"mmad_gemm_kernelI\w+?Li(\d)ELi(\d)E", n)
    if m:
        return f"mmad_gemm cfg{m.group(1)} epi{m.group(2)}"
    return re.sub(r"\(.*", "", n)[:60]


for arg in sys.argv[1:]:
    dbs = [arg] if arg.endswith(".db") else glob.glob(os.path.join(arg, "**", "*.db"), recursive=True)
    for db in dbs:
        c = sqlite3.connect(db)
        meta = dict(c.execute("select dispatch_id, name from kernels"))
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        for d, n, v in c.execute("select dispatch_id, counter_name, sum(counter_value) from pmc_events "
                                 "group by dispatch_id, counter_name"):
            vals[short(meta.get(d, "?"))][n].append(v)
        print(db)
        for k, cs in vals.items():
            med = {n: statistics.median(v) for n, v in cs.items()}
            cnt = len(next(iter(cs.values())))
            print(f"  {k}  (n={cnt})")
            for n in sorted(med):
                print(f"      {n:28s} {med[n]:16.1f}")
            wc = med.get("SQ_WAVE_CYCLES")
            if wc:
                for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                    if n in med:
                        print(f"      {n + ' / WAVE_CYCLES':40s} {med[n] / wc:8.3f}")
            if med.get("SQ_LDS_IDX_ACTIVE"):
                print(f"      {'LDS_BANK_CONFLICT / LDS_IDX_ACTIVE':40s} "
                      f"{med.get('SQ_LDS_BANK_CONFLICT', 0) / med['SQ_LDS_IDX_ACTIVE']:8.3f}")
