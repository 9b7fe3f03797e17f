"""Teacher-forced single steps: the REFERENCE's mid-training state, one more
step by the reference (8 and 1 torch threads) and -- on the GPU -- by the
product from the same state (tests/test_gpu_teacher.py).  Looks for a
per-step bias that a long trajectory comparison cannot separate from chaotic
drift ("What's weak" 1: the product's loss EMAs sit below
the reference ensemble).

Runs only in the build container (needs /root/reference); writes
tests/golden/teacher.npz.  Usage:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_teacher.py

Configuration: tests/golden/gen_nap_wc.py's (D=256, btl 20, 5 layers, batch
500, 12 batches per epoch), seed 0, the reference trained with 8 threads.
Snapshots are taken BEFORE steps SNAP_STEPS (0-based) of that run: every
parameter, the BatchNorm buffers (running mean / var, num_batches_tracked),
torch.optim.Adam's exp_avg / exp_avg_sq / step.  The batch of that step is
not stored: the product regenerates it from the build's seeded loaders (the
same generator and sampler the reference run used; its index is stored).
From each snapshot the reference takes ONE step (AutoEncoder.step,
models/auto_encoder.py:57-77, with optim.Adam(lr=1e-3), novelty_detection.py:90)
with 8 threads (stored in full: loss, every gradient, every parameter and
BatchNorm buffer after the step) and with 1 thread (stored as its deviation
from the 8-thread step, per tensor: the reference's own summation-order band).

What runs from the reference, unmodified: model_builder.get_model,
AutoEncoder.step.  Shim: collections.Iterable (models/abstract_model.py:25).
"""
import collections
import collections.abc
import os
import sys
import types
from copy import deepcopy

sys.dont_write_bytecode = True
collections.Iterable = collections.abc.Iterable
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(1, REF)
sys.path.insert(2, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from napwc_config import config_for  # noqa: E402
from icra2021_multimodal_ad_amd.common_utils import init_state_dict  # noqa: E402
from icra2021_multimodal_ad_amd.data_loaders import get_loaders  # noqa: E402

SEED = 0
SNAP_STEPS = (36, 72, 108)


def build(cfg):
    from model_builder import get_model
    model = get_model(types.SimpleNamespace(input_size=cfg.input_size, btl_size=cfg.btl_size,
                                            n_layers=cfg.n_layers, gpu_id=-1))
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    return model, opt


def stats_vs(a, b, before):
    """per-tensor deviation of step result `a` from `b` (same start `before`)"""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    d = a - b
    out = {"max": np.abs(d).max(), "norm": np.linalg.norm(d)}
    if before is not None:
        db = b - np.asarray(before, np.float64)        # b's update
        den = float((db * db).sum())
        out["step_ratio"] = float((d * db).sum()) / den if den > 0 else 0.0
    else:
        den = float((b * b).sum())
        out["proj"] = float((d * b).sum()) / den if den > 0 else 0.0
    return out


def one_step(cfg, snap, x, nthreads):
    from models.auto_encoder import AutoEncoder
    torch.set_num_threads(nthreads)
    model, opt = build(cfg)
    model.load_state_dict(deepcopy(snap["model"]))
    # Optimizer.load_state_dict keeps the given state tensors (no copy): a
    # step would update the snapshot's exp_avg / exp_avg_sq / step in place
    opt.load_state_dict(deepcopy(snap["opt"]))
    eng = types.SimpleNamespace(model=model, optimizer=opt, config=cfg)
    (loss,) = AutoEncoder.step(eng, (x, torch.zeros(x.shape[0])))
    grads = {n: p.grad.detach().numpy().copy() for n, p in model.named_parameters()}
    sd = {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
    st = opt.state_dict()["state"]
    names = [n for n, _ in model.named_parameters()]
    mv = {n: (st[i]["exp_avg"].numpy().copy(), st[i]["exp_avg_sq"].numpy().copy()) for i, n in enumerate(names)}
    return float(loss), grads, sd, mv


def oracle_step(snap, x, names):
    """The same step by the CPU oracle (oracle/ae_oracle.py: numpy fp32,
    OpenBLAS GEMMs -- a foreign fp32 implementation) from the snapshot."""
    from oracle import ae_oracle as O
    from oracle.model_io import model_from_state_dict, state_dict_from_model, grads_to_flat
    sd = {k: v.numpy().copy() for k, v in snap["model"].items()}
    m = model_from_state_dict(sd)
    st = deepcopy(snap["opt"])["state"]
    state = {"t": int(st[0]["step"])}
    pmap = {"layer.weight": "W", "layer.bias": "b", "bn.weight": "gamma", "bn.bias": "beta"}
    for i, n in enumerate(names):
        side = "enc" if n.startswith("encoder") else "dec"
        li = int(n.split(".")[2])
        key = (side, li, pmap[n.split(".", 3)[3]])
        state[("m",) + key] = st[i]["exp_avg"].numpy().astype(np.float32).copy()
        state[("v",) + key] = st[i]["exp_avg_sq"].numpy().astype(np.float32).copy()
    loss, _, grads = O.ae_train_grads(x.numpy(), m)
    O.adam_step(m, grads, state)
    return float(loss), grads_to_flat(grads), state_dict_from_model(m)


def main():
    from models.auto_encoder import AutoEncoder
    cfg = config_for(SEED)
    torch.set_num_threads(8)
    model, opt = build(cfg)
    sd0 = init_state_dict(cfg.input_size, cfg.btl_size, cfg.n_layers, seed=cfg.model_seed)
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd0.items()})
    _, train_loader, _, _ = get_loaders(cfg, device="cpu")
    eng = types.SimpleNamespace(model=model, optimizer=opt, config=cfg)
    snaps, step = [], 0
    per_epoch = len(train_loader)
    for epoch in range(1, max(SNAP_STEPS) // per_epoch + 3):
        for bi, (x, y) in enumerate(train_loader):
            if step in SNAP_STEPS:
                snaps.append({"step": step, "epoch": epoch, "batch": bi, "x": x.clone(),
                              "model": deepcopy(model.state_dict()), "opt": deepcopy(opt.state_dict())})
            if step >= max(SNAP_STEPS):
                break
            AutoEncoder.step(eng, (x, y))
            step += 1
        if len(snaps) == len(SNAP_STEPS):
            break
    assert len(snaps) == len(SNAP_STEPS), ([s["step"] for s in snaps], step)
    names = [n for n, _ in model.named_parameters()]
    out = {"meta/seed": np.int64(SEED), "meta/snap_steps": np.asarray(SNAP_STEPS, np.int64),
           "meta/per_epoch": np.int64(per_epoch), "meta/param_names": np.asarray(names),
           "meta/torch": np.asarray(torch.__version__)}
    for s in snaps:
        p = f"s{s['step']}/"
        out[p + "epoch"] = np.int64(s["epoch"])
        out[p + "batch"] = np.int64(s["batch"])
        out[p + "x_checksum"] = np.float64(s["x"].double().sum())
        for k, v in s["model"].items():
            out[p + "before/" + k] = v.numpy().copy()
        st = s["opt"]["state"]
        out[p + "adam_step"] = np.int64(int(st[0]["step"]))
        for i, n in enumerate(names):
            out[p + "exp_avg/" + n] = st[i]["exp_avg"].numpy().copy()
            out[p + "exp_avg_sq/" + n] = st[i]["exp_avg_sq"].numpy().copy()
        l8, g8, sd8, mv8 = one_step(cfg, s, s["x"], 8)
        l1, g1, sd1, mv1 = one_step(cfg, s, s["x"], 1)
        lo, go, sdo = oracle_step(s, s["x"], names)
        out[p + "ref8/loss"] = np.float64(l8)
        for n in names:
            out[p + "ref8/grad/" + n] = g8[n]
        for k in sd8:
            out[p + "ref8/after/" + k] = sd8[k]
        # the two bands: the reference's own (1 thread) and a foreign fp32
        # implementation's (the oracle), as per-tensor deviations from ref8
        for tag, (lx, gx, sdx) in (("ref1", (l1, g1, sd1)), ("orc", (lo, go, sdo))):
            out[p + f"{tag}/loss"] = np.float64(lx)
            for n in names:
                for k, v in stats_vs(gx[n], g8[n], None).items():
                    out[p + f"{tag}/grad_{k}/" + n] = np.float64(v)
            for k in sd8:
                if k.endswith("num_batches_tracked"):
                    continue
                for kk, v in stats_vs(sdx[k], sd8[k], s["model"][k].numpy()).items():
                    out[p + f"{tag}/after_{kk}/" + k] = np.float64(v)
        print(f"snapshot step {s['step']}: ref8 loss {l8:.6f} ref1 {l1:.6f} (rel {(l1 - l8) / l8:+.2e}) "
              f"oracle {lo:.6f} (rel {(lo - l8) / l8:+.2e})", flush=True)
    np.savez_compressed(os.path.join(HERE, "teacher.npz"), **out)
    print("wrote", os.path.join(HERE, "teacher.npz"), os.path.getsize(os.path.join(HERE, "teacher.npz")))


if __name__ == "__main__":
    main()
