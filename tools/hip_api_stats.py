"""Host-side HIP API cost from a rocprofv3 --hip-trace SQLite output: calls,
total and average duration per API name (the host enqueue breakdown).
Usage: python tools/hip_api_stats.py <dir-or-db> [--steps N]"""
import glob
import os
import sqlite3
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 1
    dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    c = sqlite3.connect(dbs[0])
    cols = [r[1] for r in c.execute("pragma table_info(regions)")]
    name = "name" if "name" in cols else cols[5]
    import collections
    durs = collections.defaultdict(list)
    for n, st, en in c.execute(f"select {name}, start, end from regions"):
        durs[n].append(en - st)
    rows = sorted(durs.items(), key=lambda kv: -sum(kv[1]))
    print(f"{'api':44s} {'calls':>7s} {'total_ms':>9s} {'avg_us':>8s} {'med_us':>7s} {'p90_us':>7s}")
    for n, d in rows[:30]:
        d = sorted(d)
        print(f"{str(n)[:44]:44s} {len(d):7d} {sum(d) / 1e6:9.2f} {sum(d) / len(d) / 1e3:8.2f} "
              f"{d[len(d) // 2] / 1e3:7.2f} {d[int(len(d) * 0.9)] / 1e3:7.2f}")
    # steady state: the last `steps` calls' spacing of hipLaunchKernel
    print(f"total {sum(sum(v) for v in durs.values()) / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
