"""Per-step kernel timeline from a rocprofv3 SQLite trace of bench.py.

Steps are delimited by the input-packing kernel (one per train step).  Prints,
for the median step among the last N, every kernel with its stream, start
offset and duration, and per-kernel-class totals averaged over those steps.
Usage: python tools/prof_step.py <run_results.db> [--last 20] [--csv out.csv]"""
import argparse
import collections
import csv
import re
import sqlite3
import statistics


def short(name):
    m = re.search(r"mmad_gemm_kernel<?I?(.*?)(E?EvPKT|>\()", name)
    if "mmad_gemm_kernel" in name:
        # template args: T, TO, AK, BK_, CFG, EPI, TR
        if name.startswith("_Z"):
            a = re.findall(r"Lb([01])E|Li(\d+)E", name)
            vals = [x[0] or x[1] for x in a] + ["0"]
            ak, bk, cfg, epi, tr = vals[:5]
        else:
            inner = name[name.index("<") + 1:name.index(">")]
            parts = [p.strip() for p in inner.split(",")]
            if parts[-1] in ("true", "false"):
                ak, bk, cfg, epi, tr = parts[-5:]
            else:
                ak, bk, cfg, epi = parts[-4:]
                tr = "false"
            tr = "1" if tr == "true" else "0"
        epin = {"0": "fwd", "1": "mse", "2": "bwd_data", "3": "bwd_w", "4": "score"}[epi]
        return f"gemm[{epin} cfg{cfg}{' tr' if tr == '1' else ''}]"
    m = re.match(r"_ZN12_GLOBAL__N_1\d+(\w+?)(I|E)", name)
    if m:
        return m.group(1)
    m = re.match(r"\(anonymous namespace\)::(\w+)", name)
    if m:
        return m.group(1)
    return name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--csv")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, stream_id, start, end from kernels order by start"))
    starts = [i for i, r in enumerate(rows) if "pack_input_k" in r[0]]
    steps = [rows[starts[i]:starts[i + 1]] for i in range(len(starts) - 1)]
    steps = steps[-a.last:]
    walls = [s[-1][3] - s[0][2] for s in steps]
    med = sorted(range(len(steps)), key=lambda i: walls[i])[len(steps) // 2]
    st = steps[med]
    t0 = st[0][2]
    print(f"{len(steps)} steps, wall (first start -> last end) median {statistics.median(walls) / 1e3:.1f} us")
    for name, sid, s, e in st:
        print(f"  +{(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:7.2f} us  stream {sid}  {short(name)}")
    # the step boundary: pack-to-pack period and the previous step's last kernels
    periods = [steps[i + 1][0][2] - steps[i][0][2] for i in range(len(steps) - 1)]
    if periods:
        print(f"pack-to-pack period median {statistics.median(periods) / 1e3:.1f} us")
    if med > 0:
        print("previous step's last kernels (offsets from this step's pack):")
        for name, sid, s, e in sorted(steps[med - 1], key=lambda r: r[3])[-4:]:
            print(f"  {(s - t0) / 1e3:+9.1f} .. {(e - t0) / 1e3:+9.1f} us  stream {sid}  {short(name)}")
    agg = collections.OrderedDict()
    for stp in steps:
        for name, sid, s, e in stp:
            k = short(name)
            v = agg.setdefault(k, [0, 0.0])
            v[0] += 1
            v[1] += (e - s) / 1e3
    n = len(steps)
    print("per-step totals (avg over steps):")
    out = []
    for k, (cnt, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:36s} calls/step {cnt / n:5.1f}  us/step {tot / n:8.1f}")
        out.append(dict(kernel=k, calls_per_step=round(cnt / n, 2), us_per_step=round(tot / n, 2),
                        avg_us=round(tot / cnt, 2)))
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)


if __name__ == "__main__":
    main()
