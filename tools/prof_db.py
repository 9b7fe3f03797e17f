"""Summarise a rocprofv3 SQLite output (ROCm 7.2 default format).

Usage: python tools/prof_db.py <run_results.db> [--by-grid] [--csv out.csv] [--filter substr]
Prints per-kernel (optionally per grid size) call count, average / total
duration, in order of first dispatch."""
import argparse
import collections
import csv
import re
import sqlite3


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name) if not name.startswith("void at::") else name[:60]
    m = re.match(r"_Z\d+(\w+?)I(.*)E(v|S)", name)
    return name[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--by-grid", action="store_true")
    ap.add_argument("--csv")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, grid_x, workgroup_x, duration, start from kernels order by start")
    agg = collections.OrderedDict()
    for name, gx, wx, dur, st in rows:
        if a.filter and a.filter not in name:
            continue
        key = (short(name), gx // max(wx, 1)) if a.by_grid else (short(name), 0)
        e = agg.setdefault(key, [0, 0])
        e[0] += 1
        e[1] += dur
    tot = sum(v[1] for v in agg.values()) or 1
    out = []
    for (n, g), (cnt, d) in agg.items():
        out.append(dict(name=n, blocks=g, calls=cnt, avg_us=round(d / cnt / 1e3, 3),
                        total_us=round(d / 1e3, 1), pct=round(100.0 * d / tot, 2)))
    for r in sorted(out, key=lambda r: -r["total_us"]) if not a.by_grid else out:
        print(f"{r['name'][:90]:90s} blk={r['blocks']:6d} n={r['calls']:5d} avg={r['avg_us']:9.2f}us "
              f"tot={r['total_us']:10.1f}us {r['pct']:6.2f}%")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)


if __name__ == "__main__":
    main()
