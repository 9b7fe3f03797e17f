"""Anomaly-score metrics with the reference's API (utils/metric.py:26-238),
computed on the device by the native kernels (mmad_rank_metrics,
mmad_threshold_metrics in include/mmad.h) instead of sklearn/numpy.

Same names, arguments and return tuples as the reference:
  get_auc_roc(score, label)                      :29-44  (roc_curve + auc)
  get_auc_prc(score, label)                      :97-116 (precision_recall_curve + auc)
  get_f1_score(valid, test, label, q)            :118-130 (q forced to 0.90, :120)
  get_confusion_matrix(score, label, thr)        :83-95  (score >= thr)
  get_recon_loss(valid_diff, test_diff, label)   :132-143  BASE
  get_d_loss(train, valid, test, label, ...)     :145-181  SAP
  get_d_norm_loss(train, valid, test, label, config, ...) :183-238  NAP
Scores are fp32 like the reference's ((d**2).mean(axis=1) of fp32 diffs);
labels are booleans (True = anomaly, novelty_detection.py:31-34).  Inputs may
be numpy arrays or tensors; everything runs on the current CUDA device.
"""
import ctypes

import numpy as np
import torch

from . import _native
from ._native import ptr, stream_ptr

F1_QUANTILE = 0.90   # utils/metric.py:120 overrides the f1_quantiles argument


def _dev():
    _native.require_gpu()
    return torch.device("cuda", torch.cuda.current_device())


def _as_scores(x):
    t = torch.as_tensor(x)
    return t.to(_dev(), torch.float32).reshape(-1).contiguous()


def _as_labels(y):
    t = torch.as_tensor(np.asarray(y) if not torch.is_tensor(y) else y)
    return (t.reshape(-1) != 0).to(_dev(), torch.uint8).contiguous()


_ws = {}


def _workspace(kind, nbytes):
    dev = _dev()
    key = (kind, dev)
    w = _ws.get(key)
    if w is None or w.numel() < nbytes + 256:
        w = torch.empty(int(nbytes) + 256, dtype=torch.uint8, device=dev)
        _ws[key] = w
    base = w.data_ptr()
    return ctypes.c_void_p((base + 255) // 256 * 256), int(w.numel() - ((base + 255) // 256 * 256 - base))


def rank_metrics(score, label):
    """(auroc, aupr, n_pos, n_neg) of fp32 scores vs boolean labels."""
    lib = _native.load()
    s, lab = _as_scores(score), _as_labels(label)
    n = s.numel()
    if n != lab.numel():
        raise ValueError(f"score/label length mismatch: {n} vs {lab.numel()}")
    out = torch.empty(4, dtype=torch.float64, device=s.device)
    ws, nb = _workspace("rank", lib.mmad_rank_metrics_ws_bytes(n))
    _native.call("mmad_rank_metrics", n, ptr(s), ptr(lab), ptr(out), ws, nb, stream_ptr())
    return tuple(float(v) for v in out.cpu())


def threshold_metrics(valid_score, test_score, test_label, q=F1_QUANTILE):
    """(threshold, f1, p, r, precision, recall, tp, fp, fn, tn)."""
    lib = _native.load()
    v, t, lab = _as_scores(valid_score), _as_scores(test_score), _as_labels(test_label)
    if t.numel() != lab.numel():
        raise ValueError("test score/label length mismatch")
    out = torch.empty(10, dtype=torch.float64, device=t.device)
    ws, nb = _workspace("thr", lib.mmad_threshold_metrics_ws_bytes(v.numel()))
    _native.call("mmad_threshold_metrics", v.numel(), ptr(v), t.numel(), ptr(t), ptr(lab), float(q),
                 ptr(out), ws, nb, stream_ptr())
    return tuple(float(x) for x in out.cpu())


def get_norm(x, norm_type=2):
    """utils/metric.py:26-27."""
    return abs(x) ** norm_type


def get_auc_roc(score, test_label, nap=False):
    """utils/metric.py:29-44."""
    return rank_metrics(score, test_label)[0]


def get_auc_prc(score, test_label):
    """utils/metric.py:97-116."""
    return rank_metrics(score, test_label)[1]


def get_f1_score(valid_score, test_score, test_label, f1_quantiles=(.99,)):
    """utils/metric.py:118-130 (returns f1, threshold)."""
    r = threshold_metrics(valid_score, test_score, test_label, F1_QUANTILE)
    return r[1], r[0]


def get_confusion_matrix(score, test_label, threshold):
    """utils/metric.py:83-95 (returns precision, recall at score >= threshold)."""
    r = threshold_metrics(np.asarray([threshold], np.float32), score, test_label, 0.0)
    return r[4], r[5]


def _summary(valid_score, test_score, test_label):
    auroc, aupr, _, _ = rank_metrics(test_score, test_label)
    r = threshold_metrics(valid_score, test_score, test_label, F1_QUANTILE)
    return auroc, aupr, r[1], r[4], r[5]


def _mean_sq(diffs):
    """(d**2).mean(axis=1) of one [N, W] diff matrix or a list concatenated
    along the feature axis, fp32 on the device."""
    if isinstance(diffs, (list, tuple)):
        num = None
        width = 0
        for d in diffs:
            t = torch.as_tensor(d).to(_dev(), torch.float32)
            s = (t * t).sum(dim=1)
            num = s if num is None else num + s
            width += t.shape[1]
        return num / float(width)
    t = torch.as_tensor(diffs).to(_dev(), torch.float32)
    return (t * t).mean(dim=1)


def _clamp(n, start_layer_index, end_layer_index):
    """utils/metric.py:155-162."""
    if end_layer_index is None:
        end_layer_index = n + 1
    if start_layer_index > n - 1:
        start_layer_index = n - 1
    if end_layer_index - start_layer_index < 1:
        end_layer_index = start_layer_index + 1
    return start_layer_index, end_layer_index


def get_recon_loss(valid_diff, test_diff, test_label, f1_quantiles=(.99,)):
    """BASE, utils/metric.py:132-143: (loss, auroc, aupr, f1, precision, recall)."""
    loss = _mean_sq(test_diff)
    auroc, aupr, f1, p, r = _summary(_mean_sq(valid_diff), loss, test_label)
    return loss.cpu().numpy(), auroc, aupr, f1, p, r


def get_d_loss(train_diffs, valid_diffs, test_diffs, test_label, start_layer_index=0,
               end_layer_index=None, gpu_id=-1, norm_type=2, f1_quantiles=(.99,)):
    """SAP, utils/metric.py:145-181."""
    s, e = _clamp(len(test_diffs), start_layer_index, end_layer_index)
    d_loss = _mean_sq(list(test_diffs[s:e]))
    auroc, aupr, f1, p, r = _summary(_mean_sq(list(valid_diffs[s:e])), d_loss, test_label)
    return d_loss.cpu().numpy(), auroc, aupr, f1, p, r


def get_d_norm_loss(train_diffs, valid_diffs, test_diffs, test_label, config, start_layer_index=0,
                    end_layer_index=None, gpu_id=-1, norm_type=2, f1_quantiles=(.99,), model=None):
    """NAP, utils/metric.py:183-238: Rotater/Standardizer fitted on the train
    diffs, then the native NAP run (reconstruction_aggregation.NapScorer).
    ``config.train_diffs`` (if set) receives the concatenated train diffs, as
    the reference saves them at :205 (consumed by test_file/FullTest.py:33)."""
    from .reconstruction_aggregation import NapScorer
    s, e = _clamp(len(test_diffs), start_layer_index, end_layer_index)
    cat = lambda ds: torch.cat([torch.as_tensor(d).to(_dev(), torch.float32) for d in ds[s:e]], dim=1)
    tr = cat(train_diffs)
    path = getattr(config, "train_diffs", None) if config is not None else None
    if path:
        torch.save(tr.cpu(), path)
    nap = NapScorer.standalone(tr.shape[1]).fit(train_diffs=tr)
    valid_score = nap.score(cat(valid_diffs))
    score = nap.score(cat(test_diffs))
    if norm_type != 2:
        raise NotImplementedError("NAP norm_type other than 2 (the reference only uses 2)")
    auroc, aupr, f1, p, r = _summary(valid_score, score, test_label)
    return score.cpu().numpy(), auroc, aupr, f1, p, r
