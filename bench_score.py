"""Scoring benchmark (BASELINE config C5: reconstruction_aggregation scoring over
1M synthetic windows, 1 GPU).  Prints ONE JSON line.

Workload: the RaPP scoring path of the reference (reconstruction_aggregation.py
:6-37 get_diffs + utils/metric.py:133 BASE and :145-181 SAP), streamed over N
windows already resident in HBM: ONE native call for the whole pass
(mmad_ae_score_stream), captured once as a hipGraph and replayed with one
launch (--no-graph: eager launches).  Per batch: eval AE forward, then the
encoder over x_hat reusing the encoder activations of x; per-layer
squared-diff row sums in the GEMM epilogues -- the diffs are never
materialised.  BASE and SAP per window are reduced on the device.
--nap adds the NAP score (utils/metric.py:183-238): fit on a train set of diffs,
then per batch the diffs are materialised and scored by one GEMM
(mmad_nap_score).

roofline: the dominant score GEMM (decoder last layer with the score
epilogue, algorithmic flops 2*B*K*N) timed with per-launch HIP event pairs.
cpu_baseline: the oracle's numpy get_diffs + BASE/SAP on a bounded sample on
the host (kind "port")."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BF16_PEAK_TFLOPS = 2500.0
F32_PEAK_TFLOPS = 157.3


def score_flops_per_window(enc, dec):
    ae = sum(a * b for a, b in zip(enc[:-1], enc[1:])) + sum(a * b for a, b in zip(dec[:-1], dec[1:]))
    en = sum(a * b for a, b in zip(enc[:-1], enc[1:]))
    return 2.0 * (ae + en)


def cpu_baseline(d, budget_s=10.0):
    import numpy as np
    from threadpoolctl import threadpool_limits
    from oracle import ae_oracle as O
    from oracle.model_io import model_from_state_dict
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict
    from icra2021_multimodal_ad_amd.data import synth_windows
    from bench import host_cores
    threads, n_aff, quota = host_cores()     # affinity capped by the cgroup quota
    m = model_from_state_dict(init_state_dict(d, 100, 5, seed=0))
    x = synth_windows(4096, d, seed=3)
    n, t0 = 0, time.perf_counter()
    with threadpool_limits(threads):
        while time.perf_counter() - t0 < budget_s and n < 64 * 1024:
            diffs = O.get_diffs(x, m, batch_size=698)
            O.base_score(diffs)
            O.sap_score(diffs)
            n += x.shape[0]
    el = time.perf_counter() - t0
    return {"value": n / el, "unit": "windows/sec", "cores": threads, "kind": "port",
            "sample": f"{n} windows of oracle get_diffs+BASE+SAP (numpy fp32, batch 698) at D={d}, "
                      f"{el:.1f} s, BLAS threads={threads} (affinity {n_aff} CPUs, cgroup quota "
                      f"{quota if quota is not None else 'none'})"}


def _setup(dim, dtype, N, batch):
    """Model after 20 train steps (real BN statistics), eval mode; N windows
    resident in HBM; one warm / tuning scoring batch."""
    import torch
    import types
    from icra2021_multimodal_ad_amd.model_builder import get_model
    from icra2021_multimodal_ad_amd.data import synth_windows_device
    from icra2021_multimodal_ad_amd import reconstruction_aggregation as ra
    dev = torch.device("cuda", 0)
    cfg = types.SimpleNamespace(input_size=dim, btl_size=100, n_layers=5, gpu_id=0, dtype=dtype)
    torch.manual_seed(0)
    model = get_model(cfg)
    for i in range(20):
        model.train_step_async(synth_windows_device(1024, dim, dev, seed=500 + i))
    model.eval()
    nat = model._native
    nat.sync_shadow(force=True)
    x = torch.empty((N, dim), device=dev)
    for s0 in range(0, N, 65536):
        n = min(65536, N - s0)
        x[s0:s0 + n] = synth_windows_device(n, dim, dev, seed=7 + s0)
    layer_sq = torch.empty((nat.n_enc + 1, N), device=dev)
    ra.score_windows(x[:batch], model, batch, out=layer_sq[:, :batch])   # warm / tile tuning
    torch.cuda.synchronize()
    return model, nat, x, layer_sq


def score_gemm_roofline(nat, B, iters=30):
    """The largest score GEMM (last decoder layer, score epilogue vs x) at B
    rows, per-launch HIP event pairs on the launch stream."""
    import torch
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr
    dev = nat.device
    L = nat.layers[-1]
    Mp = _native.pad(B)
    tdt = torch.bfloat16 if nat.dt == _native.BF16 else torch.float32
    xin = torch.randn((Mp, L["Kp"]), device=dev).to(tdt)
    ref = torch.randn((Mp, L["Np"]), device=dev).to(tdt)
    out = torch.empty((Mp, L["Np"]), device=dev, dtype=tdt)
    rowsq = torch.empty((L["Np"] // 128, Mp), device=dev)
    w = nat.shadow[L["w_off"]:] if nat.shadow is not None else nat.params[L["w_off"]:]
    bb = nat.params[L["b_off"]:]
    s = stream_ptr()

    def launch():
        call("mmad_fc_fwd_score", nat.dt, B, L["N"], L["K"], Mp, L["Np"], L["Kp"], ptr(xin), ptr(w),
             ptr(bb), 0, 0.2, None, None, ptr(out), ptr(ref), ptr(rowsq), None, 0, s)
    for _ in range(5):
        launch()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for e0, e1 in ev:
        e0.record()
        launch()
        e1.record()
    torch.cuda.synchronize()
    avg = sum(e0.elapsed_time(e1) for e0, e1 in ev) / 1e3 / len(ev)
    fl = 2.0 * B * L["K"] * L["N"]
    peak = BF16_PEAK_TFLOPS if nat.dt == _native.BF16 else F32_PEAK_TFLOPS
    # HBM bytes per launch from the newest PMC summary of the same kernel and
    # shape taken on THIS build's GEMM sources (tools/gpu_pmc.sh +
    # tools/pmc_gemm.py); one taken on other sources is reported as prior
    from bench import pmc_fields
    want = {"dim": nat.enc_widths[0], "batch": B, "dtype": "bf16" if nat.dt == _native.BF16 else "f32",
            "kind": "score"}
    tf, _ = pmc_fields("score", want)
    res = {"kernel": f"mmad_gemm score (decoder last layer {B}x{L['K']} . "
                     f"{L['N']}x{L['K']}^T + sum (y-x)^2 epilogue)",
           "bound": "mfma", "achieved": round(fl / avg / 1e12, 2), "peak": peak,
           "unit": "TFLOP/s", "frac": round(fl / avg / 1e12 / peak, 4), **tf,
           "avg_us": round(avg * 1e6, 2), "flops_per_launch": fl,
           "timing": f"{iters} launches, a HIP event pair around each"}
    return res


def run_c5(args):
    """bench.py --config c5: BASELINE configs[4].  One step = one whole RaPP
    scoring pass (BASE + SAP per window) over 1,048,576 windows resident in
    HBM, replayed as one captured hipGraph (mmad_ae_score_stream) plus the
    on-device BASE / SAP reductions; W untimed passes, then K timed passes
    between synchronize pairs."""
    import torch
    from icra2021_multimodal_ad_amd import reconstruction_aggregation as ra
    dim = args.dim or 2048
    batch = args.batch or 65536
    N = 1 << 20
    model, nat, x, layer_sq = _setup(dim, args.dtype, N, batch)
    widths = nat.diff_widths()

    def one_pass():
        ra.score_windows(x, model, batch, out=layer_sq, graph=True)
        return ra.base_from_layer_sq(layer_sq, widths), ra.sap_from_layer_sq(layer_sq, widths)
    for _ in range(max(1, args.warmup)):        # the first call captures the graph
        one_pass()
    torch.cuda.synchronize()
    diag = os.environ.get("MMAD_CRASH_DIAG")
    if diag:
        # crash diagnostics (round-5 SIGSEGV under rocprofv3): every Python
        # thread's stack on a fatal signal, and this process's memory map
        # once every library is loaded, so a native frame's address can be
        # resolved to library + offset afterwards
        import faulthandler
        os.makedirs(diag, exist_ok=True)
        faulthandler.enable(file=open(os.path.join(diag, "faulthandler.txt"), "w"), all_threads=True)
        with open("/proc/self/maps") as f, open(os.path.join(diag, "maps.txt"), "w") as g:
            g.write(f.read())
    t0 = time.perf_counter()
    for _ in range(args.steps):
        base, sap = one_pass()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    nat.check_status()
    value = args.steps * N / el
    fpw = score_flops_per_window(nat.enc_widths, nat.dec_widths)
    res = {
        "metric": "sensor-windows/sec (RaPP scoring: BASE+SAP)",
        "value": round(value, 1), "unit": "sensor-windows/sec", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (seeded 4-modal windows resident in HBM, AE after 20 train steps)",
        "config": {"workload": f"c5 (BASELINE configs[4]): RaPP scoring (get_diffs + BASE + SAP), "
                               f"D={dim}, btl=100, n_layers=5, {N} windows per step in batches of "
                               f"{batch}, one hipGraph replay per step", "global_batch": N,
                   "input_dim": dim, "parallelism": "dp1"},
        "model_tflops": round(value * fpw / 1e12, 2),
        "host_enqueue_ms_per_step": round(t_host / args.steps * 1e3, 4),
        "score_checksum": {"base_mean": float(base.mean()), "sap_mean": float(sap.mean())},
        "roofline": score_gemm_roofline(nat, batch),
    }
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(dim, budget_s=min(args.cpu_budget, 12.0))
    if getattr(args, "tune", None):
        res["tune"] = args.tune
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=1 << 20)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--nap", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    args = ap.parse_args()

    import torch
    import types
    from icra2021_multimodal_ad_amd.model_builder import get_model
    from icra2021_multimodal_ad_amd.data import synth_windows_device
    from icra2021_multimodal_ad_amd import reconstruction_aggregation as ra
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr

    dev = torch.device("cuda", 0)
    cfg = types.SimpleNamespace(input_size=args.dim, btl_size=100, n_layers=5, gpu_id=0, dtype=args.dtype)
    torch.manual_seed(0)
    model = get_model(cfg)
    # a few train steps so BN running statistics are real
    for i in range(20):
        model.train_step_async(synth_windows_device(1024, args.dim, dev, seed=500 + i))
    model.eval()
    nat = model._native
    nat.sync_shadow(force=True)
    widths = nat.diff_widths()

    # all windows resident in HBM before timing
    N = args.windows
    x = torch.empty((N, args.dim), device=dev)
    for s in range(0, N, 65536):
        n = min(65536, N - s)
        x[s:s + n] = synth_windows_device(n, args.dim, dev, seed=7 + s)
    layer_sq = torch.empty((nat.n_enc + 1, N), device=dev)
    ra.score_windows(x[: args.batch], model, args.batch, out=layer_sq[:, : args.batch])  # warm/tune
    torch.cuda.synchronize()

    def timed(graph, xs, bs, out, reps):
        best = None
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ra.score_windows(xs, model, bs, out=out, graph=graph)
            b_ = ra.base_from_layer_sq(out, widths)
            s_ = ra.sap_from_layer_sq(out, widths)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            best = el if best is None else min(best, el)
        return best, b_, s_

    # the first graph call runs eagerly and captures the pass; timed: replays
    ra.score_windows(x, model, args.batch, out=layer_sq, graph=not args.no_graph)
    best, base, sap = timed(not args.no_graph, x, args.batch, layer_sq, args.reps)
    eager, _, _ = timed(False, x, args.batch, layer_sq, 1)
    # the reference's own scoring batch (get_diffs default 698) over 64k
    # windows: launch-bound, where the captured graph matters
    ns = min(N, 1 << 16)
    small = {}
    for g_ in (False, True):
        ra.score_windows(x[:ns], model, 698, out=layer_sq[:, :ns], graph=g_)
        small["graph" if g_ else "eager"] = timed(g_, x[:ns], 698, layer_sq[:, :ns], 3)[0]
    value = N / best
    fpw = score_flops_per_window(nat.enc_widths, nat.dec_widths)

    res = {
        "metric": "sensor-windows/sec (RaPP scoring: BASE+SAP)",
        "value": round(value, 1),
        "unit": "sensor-windows/sec",
        "n_gpus": 1,
        "windows": N,
        "higher_is_better": True,
        "dtype": args.dtype,
        "data": "synthetic (seeded 4-modal windows resident in HBM, AE after 20 train steps)",
        "config": {"workload": f"RaPP scoring (get_diffs + BASE + SAP) D={args.dim}, btl=100, "
                               f"n_layers=5, batch {args.batch}", "windows": N},
        "ms_total": round(best * 1e3, 3),
        "launch": "eager" if args.no_graph else "hipGraph replay (one graph for the whole pass)",
        "eager_ms_total": round(eager * 1e3, 3),
        "batch698": {"windows": ns, "eager_windows_per_s": round(ns / small["eager"], 1),
                     "graph_windows_per_s": round(ns / small["graph"], 1)},
        "model_tflops": round(value * fpw / 1e12, 2),
        "score_checksum": {"base_mean": float(base.mean()), "sap_mean": float(sap.mean())},
    }

    # roofline: the largest score GEMM (last decoder layer, score epilogue vs x)
    L = nat.layers[-1]
    B = args.batch
    Mp = _native.pad(B)
    tdt = torch.bfloat16 if nat.dt == _native.BF16 else torch.float32
    xin = torch.randn((Mp, L["Kp"]), device=dev).to(tdt)
    ref = torch.randn((Mp, L["Np"]), device=dev).to(tdt)
    out = torch.empty((Mp, L["Np"]), device=dev, dtype=tdt)
    rowsq = torch.empty((L["Np"] // 128, Mp), device=dev)
    w = nat.shadow[L["w_off"]:] if nat.shadow is not None else nat.params[L["w_off"]:]
    bb = nat.params[L["b_off"]:]
    s = stream_ptr()

    def launch():
        call("mmad_fc_fwd_score", nat.dt, B, L["N"], L["K"], Mp, L["Np"], L["Kp"], ptr(xin), ptr(w),
             ptr(bb), 0, 0.2, None, None, ptr(out), ptr(ref), ptr(rowsq), None, 0, s)
    for _ in range(5):
        launch()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(30)]
    for e0, e1 in ev:
        e0.record()
        launch()
        e1.record()
    torch.cuda.synchronize()
    avg = sum(e0.elapsed_time(e1) for e0, e1 in ev) / 1e3 / len(ev)
    fl = 2.0 * B * L["K"] * L["N"]
    peak = BF16_PEAK_TFLOPS if nat.dt == _native.BF16 else F32_PEAK_TFLOPS
    res["roofline"] = {"kernel": f"mmad_gemm_kernel score (decoder last layer {B}x{L['K']} . "
                                 f"{L['N']}x{L['K']}^T + sum (y-x)^2 epilogue)",
                       "bound": "mfma", "achieved": round(fl / avg / 1e12, 2), "peak": peak,
                       "unit": "TFLOP/s", "frac": round(fl / avg / 1e12 / peak, 4), "traffic": None,
                       "avg_us": round(avg * 1e6, 2), "flops_per_launch": fl}

    if args.nap:
        ntr = 20000
        xtr = synth_windows_device(ntr, args.dim, dev, seed=99)
        tr = []
        for s0 in range(0, ntr, 4096):
            _, d = nat.score(xtr[s0:s0 + 4096], want_diffs=True)
            tr.append(d)
        tr = torch.cat(tr)
        nap = ra.NapScorer(model).fit(train_diffs=tr)
        nn_ = min(N, 1 << 18)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s0 in range(0, nn_, args.batch):
            _, d = nat.score(x[s0:s0 + args.batch], want_diffs=True)
            nap.score(d)
        torch.cuda.synchronize()
        res["nap"] = {"windows": nn_, "windows_per_s": round(nn_ / (time.perf_counter() - t0), 1),
                      "fit_train_windows": ntr, "rank": int(nap.fit_state["v"].shape[1])}

    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args.dim)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
