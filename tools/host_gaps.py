"""Host enqueue timeline of one steady-state step from a rocprofv3
--hip-trace --kernel-trace SQLite output: every HIP API call of the step's
host thread in order, its duration and the host time spent BEFORE it since
the previous call ended (executor / Python code), with the kernel a launch
enqueued.  Usage: python tools/host_gaps.py <dir> [--step-kernel pack_input_k]"""
import glob
import os
import sqlite3
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[sys.argv.index("--step-kernel") + 1] if "--step-kernel" in sys.argv else "pack_input_k"
    db = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    kcols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    rcols = [r[1] for r in c.execute("pragma table_info(regions)")]
    rows = c.execute("select name, start, end, tid, id from regions order by start").fetchall()
    # main thread = the one with the most launches
    from collections import Counter
    tid = Counter(r[0] == "hipLaunchKernel" and r[3] for r in rows).most_common(2)
    tid = [t for t, _ in tid if t is not False][0]
    rows = [r for r in rows if r[3] == tid]
    # launches <-> dispatches by order (the runtime's own blit kernels, from
    # memcpy / memset, are not hipLaunchKernel calls)
    disp = [n for (n,) in c.execute("select name from kernels order by dispatch_id")
            if not n.startswith("__amd_rocclr")]
    launches = [r[4] for r in rows if r[0] == "hipLaunchKernel"]
    kname = dict(zip(launches, disp))
    if len(disp) != len(launches):
        print(f"warning: {len(launches)} launches vs {len(disp)} dispatches (mapping by order)")
    # step boundaries: launches of the marker kernel
    idx = [i for i, r in enumerate(rows) if r[0] == "hipLaunchKernel" and marker in str(kname.get(r[4], ""))]
    if len(idx) < 3:
        print("marker launches:", len(idx), "kernel names:", len(kname))
        print("kernels cols:", kcols)
        print("regions cols:", rcols)
        for r in c.execute("select * from regions limit 3"):
            print(r)
        for r in c.execute("select * from kernels limit 2"):
            print(r)
        return
    a, b = idx[-3], idx[-2]
    print(f"step: {len(rows[a:b])} API calls, host {(rows[b][1] - rows[a][1]) / 1e3:.1f} us")
    prev_end = rows[a - 1][2]
    for r in rows[a:b]:
        gap = (r[1] - prev_end) / 1e3
        k = kname.get(r[4], "")
        k = k.replace("(anonymous namespace)::", "")[:70]
        print(f"{gap:7.2f} {(r[2] - r[1]) / 1e3:7.2f}  {r[0][:26]:26s} {k}")
        prev_end = r[2]


if __name__ == "__main__":
    main()
