"""Benchmark: sensor-windows/sec of the AE train step (fwd + sum-MSE + bwd +
Adam) on synthetic 4-modal windows -- BASELINE.json configs[1]: D=2048,
batch=1024 per GPU, bf16 storage / fp32 accumulate, 1..8 MI355X (weak scaling,
per-layer RCCL all-reduce of the gradients overlapped with the backward).

Prints ONE JSON line (rank 0) with the driver's fields plus ``roofline`` (the
encoder's first GEMM, the dominant kernel, timed with a HIP event pair around
back-to-back launches on the stream it runs on; HBM traffic from the newest
profiles/*_pmc_traffic.json) and ``cpu_baseline`` (the oracle's numpy fp32 train step on
host cores, bounded sample).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--dim 2048] [--batch 1024]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
F32_PEAK_TFLOPS = 157.3     # f32 MFMA = vector rate


def ae_flops_per_window(widths_enc, widths_dec):
    macs = sum(a * b for a, b in zip(widths_enc[:-1], widths_enc[1:]))
    macs += sum(a * b for a, b in zip(widths_dec[:-1], widths_dec[1:]))
    return 6.0 * macs, macs   # fwd 2*MAC + bwd-data 2*MAC + bwd-weight 2*MAC


def cpu_baseline(d, batch, budget_s=12.0, threads=16):
    """Oracle (numpy fp32) train step timed on host cores: a bounded sample of
    the same workload (whole steps at the same D and batch)."""
    import numpy as np
    from threadpoolctl import threadpool_limits
    from oracle import ae_oracle as O
    from oracle.model_io import model_from_state_dict
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict
    from icra2021_multimodal_ad_amd.data import synth_windows
    threads = min(threads, os.cpu_count() or 1)
    model = model_from_state_dict(init_state_dict(d, 100, 5, seed=0))
    x = synth_windows(batch, d, seed=1)
    st = {}
    with threadpool_limits(limits=threads):
        O.train_step(x, model, st)            # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            O.train_step(x, model, st)
            n += 1
            el = time.perf_counter() - t0
            if el > budget_s or n >= 50:
                break
    return {"value": n * batch / el, "unit": "sensor-windows/sec", "cores": threads,
            "kind": "port",
            "sample": f"{n} oracle train steps (numpy fp32 fwd+bwd+Adam) at D={d}, batch={batch}, "
                      f"{el:.1f} s, BLAS threads={threads}"}


def gemm_roofline(model, batch, iters=50):
    """Average duration of the encoder's first-layer forward GEMM (the largest
    MFMA kernel of the step) from HIP events on the launch stream."""
    import torch
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr
    nat = model._native
    L = nat.layers[0]
    Mp = _native.pad(batch)
    dt = nat.dt
    tdt = torch.bfloat16 if dt == _native.BF16 else torch.float32
    dev = nat.device
    xin = torch.randn((Mp, L["Kp"]), device=dev).to(tdt)
    out = torch.empty((Mp, L["Np"]), device=dev, dtype=tdt)
    stats = torch.empty((Mp // 32, 2, L["Np"]), device=dev)
    w = nat.shadow[L["w_off"]:] if nat.shadow is not None else nat.params[L["w_off"]:]
    b = nat.params[L["b_off"]:]
    s = stream_ptr()
    _native.enable_gemm_workspace(dev)   # split-K workspace, as the executor's GEMMs have

    def launch():
        call("mmad_fc_fwd", dt, batch, L["N"], L["K"], Mp, L["Np"], L["Kp"], ptr(xin), ptr(w), ptr(b),
             1, 0.2, None, None, ptr(out), ptr(stats), s)
    for _ in range(5):
        launch()
    # one event pair on the launch stream around `iters` back-to-back launches
    # (the queue stays full, so this is the kernel duration plus the GPU's
    # dispatch gap; an event pair per launch adds ~2 us of event overhead and
    # disagrees with rocprofv3's kernel-trace average)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        launch()
    e1.record()
    torch.cuda.synchronize()
    avg_s = e0.elapsed_time(e1) / 1e3 / iters
    flops = 2.0 * batch * L["K"] * L["N"]
    peak = BF16_PEAK_TFLOPS if dt == _native.BF16 else F32_PEAK_TFLOPS
    ach = flops / avg_s / 1e12
    return {"kernel": f"mmad_gemm_kernel fwd (encoder layer 1: {batch}x{L['K']} . {L['N']}x{L['K']}^T,"
                      f" bias+LeakyReLU+BN-stat epilogue)",
            "bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(ach / peak, 4), "traffic": _pmc_traffic(L["K"], batch, dt),
            "avg_us": round(avg_s * 1e6, 2), "flops_per_launch": flops}


def _pmc_traffic(dim, batch, dt):
    """HBM-side bytes per launch of the roofline kernel from the committed
    rocprofv3 PMC passes (newest profiles/*_pmc_traffic.json: FETCH_SIZE x2 +
    WRITE_SIZE, gfx950 correction) when they were taken at this workload."""
    import glob
    from icra2021_multimodal_ad_amd import _native
    for f in sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                           "*_pmc_traffic.json")))[::-1]:
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        w = d.get("workload", {})
        if (w.get("dim"), w.get("batch"), w.get("dtype")) == (dim, batch,
                                                             "bf16" if dt == _native.BF16 else "f32"):
            return d["traffic_bytes_per_launch"]
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=1024, help="windows per GPU per step")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--model", default="ae", choices=["ae", "vib_ae"],
                    help="vib_ae: BASELINE config C3/C4 (VIB head, k=1, beta_kl=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from icra2021_multimodal_ad_amd import dist as mdist
    from icra2021_multimodal_ad_amd.model_builder import get_model
    from icra2021_multimodal_ad_amd.data import synth_windows_device
    import types

    rank, world, local = mdist.init_from_env()
    torch.cuda.set_device(local)
    cfg = types.SimpleNamespace(input_size=args.dim, btl_size=100, n_layers=5, gpu_id=local,
                                dtype=args.dtype, models=args.model, vib_k=1, beta_kl=1.0)
    torch.manual_seed(0)
    model = get_model(cfg)
    mdist.attach_data_parallel(model)
    model._native.sync_shadow(force=True)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    dev = torch.device("cuda", local)
    # a pool of distinct synthetic batches resident in HBM before timing
    pool = [synth_windows_device(args.batch, args.dim, dev, seed=1000 * rank + i) for i in range(8)]

    for i in range(args.warmup):
        model.train_step_async(pool[i % len(pool)], opt)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = model.train_step_async(pool[i % len(pool)], opt)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    loss_v = float(loss.item())

    nat = model._native
    fpw, _ = ae_flops_per_window(nat.enc_widths, nat.dec_widths)
    windows = args.steps * args.batch * world
    value = windows / el
    res = {
        "metric": "sensor-windows/sec (train fwd+bwd)",
        "value": round(value, 1),
        "unit": "sensor-windows/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (seeded 4-modal window generator, random-init weights)",
        "config": {"workload": f"{'VIB-AE' if args.model == 'vib_ae' else 'FC-AE'} train step "
                               f"(fwd+sum-MSE{'+KL' if args.model == 'vib_ae' else ''}+bwd+Adam), "
                               f"D={args.dim}, btl=100, "
                               f"n_layers=5, {args.batch} windows/GPU",
                   "global_batch": args.batch * world, "input_dim": args.dim,
                   "parallelism": f"dp{world}",
                   "exchange": ("native RCCL per-layer buckets overlapped with backward"
                                if model.dist is not None and model.dist.native else
                                ("torch.distributed flat all-reduce" if world > 1 else "none"))},
        "model_tflops": round(value * fpw / 1e12, 2),
        "final_loss": loss_v,
    }
    if rank == 0:
        res["roofline"] = gemm_roofline(model, args.batch)
        if not args.no_cpu_baseline and world == 1:   # host baseline: rank 0 at N=1 only
            res["cpu_baseline"] = cpu_baseline(args.dim, args.batch, budget_s=args.cpu_budget)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        if model.dist is not None and model.dist.native:
            model._native.set_comm(None)
            model.dist.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
