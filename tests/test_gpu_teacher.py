"""Teacher-forced single steps (tests/golden/teacher.npz, gen_teacher.py): the
product takes ONE fp32 training step from the REFERENCE's own mid-training
state (parameters, BatchNorm buffers, Adam exp_avg / exp_avg_sq / step) on the
same batch, and its deviation from the reference's 8-thread step is held to
the band of two other fp32 programs from the same state: the reference with
1 thread and the CPU oracle (numpy / OpenBLAS).

What this separates: a per-step BIAS (BatchNorm running-variance factor,
Adam bias correction / eps placement / (1 - beta) constants, a reduction
order that favours one sign) would show at every snapshot as a deviation
larger than the band and with a consistent sign (loss lower, update larger);
chaotic drift of a whole trajectory would not.  VERDICT round 4 asked for
this (the product's trained loss EMAs sit below the ensemble's).

Bars (per snapshot, per tensor, on the Euclidean norm of the deviation from
ref8): product <= 3 x max(ref1's, oracle's) + 2^-22 x |ref8| (the floor
covers tensors on which two programs agree bit for bit); the step-size ratio
<d(update), update_ref8> / |update_ref8|^2 within 3 x the band's, and the
loss within 3 x the band.  The signed statistics are printed (pytest -s) and
summarised by test_teacher_no_signed_bias."""
import json
import os
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
FLOOR = 2.0 ** -22


def _cfg():
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from napwc_config import config_for    # plain configuration data (no reference import)
    return config_for(0)


def _batch(cfg, epoch, bi):
    """The training batch (epoch, bi) of the seeded loaders -- the same
    generator and sampler order the reference run used."""
    from icra2021_multimodal_ad_amd.data_loaders import get_loaders
    _, tl, _, _ = get_loaders(cfg, device="cpu")
    for e in range(1, epoch + 1):
        for i, (x, _) in enumerate(tl):
            if e == epoch and i == bi:
                return x
    raise AssertionError("batch not found")


def _product_step(g, p, cfg, x, fused):
    from icra2021_multimodal_ad_amd import _native
    from icra2021_multimodal_ad_amd.model_builder import get_model
    names = [str(n) for n in g["meta/param_names"]]
    with _native.tune(keep_grads=1):
        mcfg = types.SimpleNamespace(input_size=cfg.input_size, btl_size=cfg.btl_size,
                                     n_layers=cfg.n_layers, gpu_id=0, dtype="f32")
        m = get_model(mcfg)
    sd = {k[len(p + "before/"):]: torch.from_numpy(np.asarray(g[k])) for k in g.files
          if k.startswith(p + "before/")}
    m.load_state_dict(sd)
    nat = m._native
    layers = list(m.encoder.layer_list) + list(m.decoder.layer_list)
    for buf, key in ((nat.exp_avg, "exp_avg/"), (nat.exp_avg_sq, "exp_avg_sq/")):
        for l, layer in enumerate(layers):
            side = "encoder" if l < len(m.encoder.layer_list) else "decoder"
            i = l if side == "encoder" else l - len(m.encoder.layer_list)
            pre = p + key + f"{side}.net.{i}."
            w, b, ga, be = nat.param_views(buf, l)
            w.copy_(torch.from_numpy(g[pre + "layer.weight"]))
            b.copy_(torch.from_numpy(g[pre + "layer.bias"]))
            if layer.bn is not None:
                ga.copy_(torch.from_numpy(g[pre + "bn.weight"]))
                be.copy_(torch.from_numpy(g[pre + "bn.bias"]))
    nat.adam_step_count = int(g[p + "adam_step"])
    xd = x.cuda()
    if fused:
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        eng = types.SimpleNamespace(model=m, optimizer=opt, config=mcfg)
        (loss,) = m.step(eng, (xd, torch.zeros(x.shape[0])))
    else:
        m.train()
        loss = float(nat.train_step(xd))
        m._count_bn_step()
        nat.adam(lr=1e-3)
    torch.cuda.synchronize()
    grads = {}
    for l, layer in enumerate(layers):
        side = "encoder" if l < len(m.encoder.layer_list) else "decoder"
        i = l if side == "encoder" else l - len(m.encoder.layer_list)
        w, b, ga, be = nat.param_views(nat.grads, l)
        pre = f"{side}.net.{i}."
        grads[pre + "layer.weight"] = w.cpu().numpy()
        grads[pre + "layer.bias"] = b.cpu().numpy()
        if layer.bn is not None:
            grads[pre + "bn.weight"] = ga.cpu().numpy()
            grads[pre + "bn.bias"] = be.cpu().numpy()
    after = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    return float(loss), grads, after, names


def _dev(a, b, before=None):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    d = a - b
    out = {"norm": float(np.linalg.norm(d)), "ref_norm": float(np.linalg.norm(b))}
    if before is not None:
        db = b - np.asarray(before, np.float64)
        den = float((db * db).sum())
        out["step_ratio"] = float((d * db).sum()) / den if den > 0 else 0.0
        out["upd_norm"] = float(np.sqrt(den))
    return out


def _analyse(g, fused):
    cfg = _cfg()
    rows = []
    for s in g["meta/snap_steps"]:
        p = f"s{int(s)}/"
        x = _batch(cfg, int(g[p + "epoch"]), int(g[p + "batch"]))
        assert abs(float(x.double().sum()) - float(g[p + "x_checksum"])) <= 1e-6 * abs(float(g[p + "x_checksum"])) + 1e-6
        loss, grads, after, names = _product_step(g, p, cfg, x, fused)
        l8 = float(g[p + "ref8/loss"])
        row = {"step": int(s), "loss_dev": (loss - l8) / l8,
               "loss_band": max(abs(float(g[p + "ref1/loss"]) - l8), abs(float(g[p + "orc/loss"]) - l8)) / l8,
               "tensors": []}
        for n in names:
            d = _dev(grads[n], g[p + "ref8/grad/" + n])
            band = max(float(g[p + "ref1/grad_norm/" + n]), float(g[p + "orc/grad_norm/" + n]))
            row["tensors"].append({"t": "grad/" + n, "dev": d["norm"], "band": band, "scale": d["ref_norm"]})
        for k in after:
            if k.endswith("num_batches_tracked"):
                assert int(after[k]) == int(g[p + "ref8/after/" + k]), k
                continue
            d = _dev(after[k], g[p + "ref8/after/" + k], g[p + "before/" + k])
            band = max(float(g[p + "ref1/after_norm/" + k]), float(g[p + "orc/after_norm/" + k]))
            rband = max(abs(float(g[p + "ref1/after_step_ratio/" + k])),
                        abs(float(g[p + "orc/after_step_ratio/" + k])))
            row["tensors"].append({"t": "after/" + k, "dev": d["norm"], "band": band,
                                   "scale": d["ref_norm"], "upd": d["upd_norm"], "ratio": d["step_ratio"],
                                   "ratio_band": rband})
        rows.append(row)
    return rows


@pytest.mark.parametrize("fused", [True, False], ids=["fused_step", "train_step+adam"])
def test_teacher_forced_step_within_reference_band(golden, fused):
    g = golden("teacher")
    rows = _analyse(g, fused)
    out = os.environ.get("MMAD_TEACHER_OUT")
    if out:
        with open(out + ("_fused" if fused else "_unfused") + ".json", "w") as f:
            json.dump(rows, f)
    worst = []
    for r in rows:
        assert abs(r["loss_dev"]) <= 3 * r["loss_band"] + 1e-7, (r["step"], r["loss_dev"], r["loss_band"])
        for t in r["tensors"]:
            lim = 3 * t["band"] + FLOOR * t["scale"]
            worst.append((t["dev"] / lim if lim > 0 else 0.0, r["step"], t["t"]))
            assert t["dev"] <= lim, (r["step"], t)
            # the step-size ratio where the deviation is above the ulp floor
            # (an update of a few ulps makes a one-ulp difference a large ratio)
            if "ratio" in t and t["dev"] > FLOOR * t["scale"]:
                assert abs(t["ratio"]) <= 3 * t["ratio_band"] + 1e-6, (r["step"], t)
    worst.sort(reverse=True)
    print("worst dev / limit:", worst[:5])


def test_teacher_no_signed_bias(golden):
    """Across snapshots and tensors, the product's signed deviations (loss and
    step-size ratio of every parameter update) are not one-sided beyond what
    the reference's own band shows: a systematic bias would put (almost) every
    ratio on one side."""
    g = golden("teacher")
    rows = _analyse(g, True)
    ratios = np.array([t["ratio"] for r in rows for t in r["tensors"] if "ratio" in t and t["upd"] > 0])
    bands = np.array([t["ratio_band"] for r in rows for t in r["tensors"] if "ratio" in t and t["upd"] > 0])
    loss_devs = [r["loss_dev"] for r in rows]
    pos, neg = int((ratios > 0).sum()), int((ratios < 0).sum())
    print(f"loss deviations {loss_devs}; step ratios: {pos} positive, {neg} negative, "
          f"{len(ratios) - pos - neg} exact; mean {ratios.mean():+.3e} (band mean {bands.mean():.3e})")
    # mean signed ratio inside the band's typical size (round 4's Adam, with
    # 1 - beta formed in float, gave -7.7e-6 here: 16 of 156 positive), and
    # the signs of the non-zero ratios not one-sided beyond 3 sigma of a fair coin
    assert abs(ratios.mean()) <= bands.mean() + 1e-7
    assert abs(pos - neg) <= 3.0 * np.sqrt(pos + neg) + 1, (pos, neg)
