"""A/B of GEMM tile configurations on the forward / score shapes, interleaved
in one process (cdna_hip_programming.md rule 24), with hipBLASLt (torch.mm)
timed alongside, and a bit-identity check of every tile's output against the
first one's.
Usage: python tools/tile_ab.py <batch> [tiles=6+7] [layers=0+8+9] [rounds=5] [kind=fwd|score]"""
import statistics
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

from icra2021_multimodal_ad_amd import _native  # noqa: E402
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
# a tile may carry a debug-knob value: "7d2" = tile 7 with dbg 2 (loop only)
tiles = (sys.argv[2] if len(sys.argv) > 2 else "6+7").split("+")
layers = [int(t) for t in (sys.argv[3] if len(sys.argv) > 3 else "0+8+9").split("+")]
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
kind = sys.argv[5] if len(sys.argv) > 5 else "fwd"
widths = [2048, 1658, 1268, 879, 489, 100, 489, 879, 1268, 1658, 2048]
pairs = list(zip(widths[:-1], widths[1:]))
if "--vib" in sys.argv:                 # the c3 model: encoder output 2 x 100 (mu | log-var)
    e = [2048, 1678, 1308, 939, 569, 200]
    d = [100, 489, 879, 1268, 1658, 2048]
    pairs = list(zip(e[:-1], e[1:])) + list(zip(d[:-1], d[1:]))
dev = torch.device("cuda", 0)
lib = _native.load()
_native.enable_gemm_workspace(dev)
s = stream_ptr()
Mp = pad(B)
torch.manual_seed(0)


def timeit(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for li in layers:
    K, N = pairs[li]
    Kp, Np = pad(K), pad(N)
    x = torch.empty(Mp, Kp, device=dev).uniform_(-1, 1).bfloat16()
    x[:, K:] = 0
    w = (torch.empty(Np, Kp, device=dev).uniform_(-1, 1) * 0.05).bfloat16()
    w[N:] = 0
    w[:, K:] = 0
    b = torch.randn(Np, device=dev) * 0.1
    y = torch.empty(Mp, Np, device=dev, dtype=torch.bfloat16)
    st = torch.empty(Mp // 32, 2, Np, device=dev)
    ref = torch.randn(Mp, Np, device=dev).bfloat16()
    rowsq = torch.empty(Np // 128, Mp, device=dev)
    dx = torch.empty(Mp, Kp, device=dev, dtype=torch.bfloat16)
    xs, ws = x[:B, :K], w[:N, :K]
    fl = 2.0 * B * K * N
    iters = max(5, int(2e-3 / max(fl / 1.0e15, 1e-7)))    # ~2 ms of work per timing

    def mine():
        if kind == "score":
            call("mmad_fc_fwd_score", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 0, 0.2, None, None,
                 ptr(y), ptr(ref), ptr(rowsq), None, 0, s)
        elif kind == "bwd_data":
            call("mmad_fc_bwd_data", 1, B, N, K, Mp, Np, Kp, ptr(ref), ptr(w), ptr(dx), None, s)
        elif kind == "fwdns":     # no BN-stat partials
            call("mmad_fc_fwd", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1, 0.2, None, None,
                 ptr(y), None, s)
        elif kind == "fwdlin":    # no activation, no BN-stat partials
            call("mmad_fc_fwd", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 0, 0.2, None, None,
                 ptr(y), None, s)
        else:
            call("mmad_fc_fwd", 1, B, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1, 0.2, None, None,
                 ptr(y), ptr(st), s)
    outs = {}
    res = {t: [] for t in tiles}
    res["blas"] = []
    for r in range(rounds):
        for t in tiles:
            tt, _, dbg = t.partition("d")
            per = tt.endswith("p")              # "6p": the persistent grid (knob 12)
            lib.mmad_tune_set(0, int(tt.rstrip("p")))
            lib.mmad_tune_set(3, int(dbg or 0))
            lib.mmad_tune_set(12, 1 if per else 0)
            res[t].append(timeit(mine, iters))
            lib.mmad_tune_set(3, 0)
            lib.mmad_tune_set(12, 0)
            if r == 0:
                torch.cuda.synchronize()
                outs[t] = ((dx if kind == "bwd_data" else y).clone(),
                           rowsq.clone() if kind == "score" else st.clone())
        lib.mmad_tune_set(0, -1)
        if kind == "bwd_data":
            res["blas"].append(timeit(lambda: torch.mm(ref[:B, :N], ws), iters))
        else:
            res["blas"].append(timeit(lambda: torch.mm(xs, ws.t()), iters))
    lib.mmad_tune_set(0, -1)
    line = [f"L{li} {kind} {B}x{K}->{N}:"]
    for t, v in res.items():
        med = statistics.median(v)
        line.append(f"{'tile ' + str(t) if t != 'blas' else 'hipblaslt'} {med:8.2f}us {fl / med / 1e6:7.1f}TF "
                    f"(min {min(v):.2f})")
    t0 = tiles[0]
    same = [f"{t}:{'=' if torch.equal(outs[t][0], outs[t0][0]) and torch.equal(outs[t][1], outs[t0][1]) else 'DIFF'}"
            for t in tiles[1:] if "d" not in t]
    print(" | ".join(line), "| bits vs tile", t0, " ".join(same), flush=True)
