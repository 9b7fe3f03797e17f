"""Producer benchmark: the HSR_Net multimodal fusion (utils/data_loaders.py:
152-229) that turns raw sensor streams into the [N x 1728] windows the
autoencoder trains and scores on.  Prints ONE JSON line.

Workload: N windows (default 65536) of seeded U[0,1] raw modalities already
resident in HBM -- hand RGB [3x32x32], head depth [32x32], F/T scalar, 13
MFCCs (the shapes utils/data_loaders.py:369-396 hands to the net) -- fused by
ONE native call (mmad_hsr_fuse; one 256-thread workgroup per window) into
fp32 rows of 1728.  The reference runs the net one window at a time in a
Python loop with a growing torch.cat (:183-228).

Per window: 877,088 MACs (conv1r 49,152, conv2r 589,824, conv3r 65,536,
conv1d 8,192, conv2d 147,456, conv3d 16,384, conv1l 288, conv2l 256) =
1.754 MFLOP; compulsory HBM bytes 16,440 in + 6,912 out = 23,352 B.
Arithmetic intensity 75 FLOP/B, above the fp32 vector ridge (157.3 TFLOP/s
/ 8 TB/s = 20), so the roofline is the fp32 VALU peak.
cpu_baseline: the oracle (numpy fp32, batched) on a bounded sample."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

F32_PEAK_TFLOPS = 157.3
HBM_PEAK_GBS = 8000.0
MACS = {"conv1r": 16 * 256 * 12, "conv2r": 16 * 256 * 144, "conv3r": 16 * 64 * 64,
        "conv1d": 8 * 256 * 4, "conv2d": 8 * 256 * 72, "conv3d": 8 * 64 * 32,
        "conv1l": 8 * 2 * 18, "conv2l": 16 * 16}
FLOPS_PER_WINDOW = 2.0 * sum(MACS.values())
BYTES_PER_WINDOW = 4 * (3072 + 1024 + 1 + 13) + 4 * 1728


def cpu_baseline(net, budget_s=10.0):
    import numpy as np
    from threadpoolctl import threadpool_limits
    from oracle.hsr_oracle import hsr_forward
    threads = min(16, os.cpu_count() or 1)
    W = {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()}
    rng = np.random.default_rng(5)
    b = 512
    r = rng.random((b, 3, 32, 32), np.float32)
    d = rng.random((b, 1, 32, 32), np.float32)
    t = rng.random((b, 1), np.float32)
    m = rng.random((b, 13), np.float32)
    n, t0 = 0, time.perf_counter()
    with threadpool_limits(threads):
        while time.perf_counter() - t0 < budget_s and n < 64 * 1024:
            hsr_forward(W, r, d, t, m)
            n += b
    el = time.perf_counter() - t0
    return {"value": n / el, "unit": "windows/sec", "cores": threads, "kind": "port",
            "sample": f"{n} windows of the oracle HSR_Net forward (numpy fp32, batches of {b}), "
                      f"{el:.1f} s, BLAS threads={threads}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import types
    from icra2021_multimodal_ad_amd.hsr_net import HSR_Net

    n = args.windows
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = HSR_Net(False, types.SimpleNamespace(slicing_size=n, gpu_id=0)).to(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    r = torch.rand(n, 1, 3, 32, 32, device=dev, generator=g)
    d = torch.rand(n, 1, 1, 32, 32, device=dev, generator=g)
    t = torch.rand(n, 1, device=dev, generator=g)
    m = torch.rand(n, 1, 1, 13, device=dev, generator=g)
    out = torch.empty(n, 1728, device=dev)
    for _ in range(3):
        net(r, d, None, t, m, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        net(r, d, None, t, m, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    value = n / (ms * 1e-3)
    tflops = value * FLOPS_PER_WINDOW / 1e12
    res = {
        "metric": "sensor-windows/sec (HSR_Net multimodal fusion producer)",
        "value": round(value, 1),
        "unit": "sensor-windows/sec",
        "n_gpus": 1,
        "windows": n,
        "higher_is_better": True,
        "dtype": "f32",
        "data": "synthetic (seeded U[0,1] raw modalities resident in HBM, random-init convs)",
        "config": {"workload": "HSR_Net(r, d, None, t, m) fused rows [N x 1728], one native call",
                   "windows": n},
        "ms_per_call": round(ms, 4),
        "checksum": float(out.double().mean()),
        "roofline": {"kernel": "hsr_fuse_k (one workgroup per window)", "bound": "valu-fp32",
                     "achieved": round(tflops, 2), "peak": F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(tflops / F32_PEAK_TFLOPS, 4), "traffic": None,
                     "hbm_gbs": round(value * BYTES_PER_WINDOW / 1e9, 1),
                     "hbm_frac": round(value * BYTES_PER_WINDOW / 1e9 / HBM_PEAK_GBS, 4),
                     "flops_per_window": FLOPS_PER_WINDOW, "bytes_per_window": BYTES_PER_WINDOW},
    }
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(net)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
