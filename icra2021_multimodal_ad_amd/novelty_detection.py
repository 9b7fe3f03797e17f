"""NoveltyDetecter: the reference's train-and-test driver
(novelty_detection.py:10-127) without pytorch-ignite, on the native hot path.

train (:88-127): Adam(lr 1e-3) (:90); a trainer Engine running
``AutoEncoder.step`` per mini-batch and an evaluator Engine running
``AutoEncoder.validate`` over the valid loader at every EPOCH_COMPLETED
(:103-108); ``model.attach`` puts ignite-style RunningAverage(alpha 0.98,
reset per epoch) 'recon' metrics on both; the evaluator keeps a deep copy of
the state_dict whenever its EMA beats the lowest so far (:114-122); after
``n_epochs`` the best state is loaded back (:125).

test (:15-85): BASE (:42-47), SAP (:50-60) and NAP (:62-73) scores with
AUROC / AUPR / F1 / precision / recall.  The scores are produced on the
device: BASE and SAP from the fused scoring pass (mmad_ae_score_stream:
per-window squared-diff sums, the diffs never materialised), NAP from the
device diffs (mmad_ae_score) through the native NAP run; the metrics by the
native rank/threshold kernels (metric.py).  Train diffs are scored in batches
of ``config.batch_size`` and valid/test in 698 (:36-38, get_diffs' default).

Data parallel (model.dist set by dist.attach_data_parallel):
the loaders hand each rank its rows of every global batch, validation losses
are summed over the ranks (every rank keeps the same best-on-valid state),
BatchNorm running statistics are averaged over the ranks at every epoch end
before validation, and scoring is sharded by rows with the per-window scores
(and the NAP fit's train diffs) all-gathered, so every rank reports the
single-process metrics.
"""
from copy import deepcopy

import numpy as np
import torch

from . import metric
from .engine_loop import Engine, Events
from .reconstruction_aggregation import (NapScorer, base_from_layer_sq, sap_from_layer_sq,
                                         score_windows)


def _layer_sq(model, x, batch_size):
    return score_windows(x.to(model._native.device).float().contiguous(), model,
                         batch_size=batch_size, graph=False)


def _device_diffs(model, x, batch_size):
    """Concatenated get_diffs output [N, sum widths] on the device."""
    nat = model._native
    x = x.to(nat.device).float()
    parts = [nat.score(x[s:s + batch_size], want_diffs=True)[1] for s in range(0, x.shape[0], batch_size)]
    nat.check_status()
    return torch.cat(parts, dim=0)


def _nap_model(model, cfg):
    """The model whose diffs NAP consumes.  NAP standardises every principal
    component of the train diffs by its variance (utils/normalize.py:36-45,
    utils/metric.py:219-222), down to ~1e-10 of the largest on these models,
    so bf16 activations -- 8 significant bits -- turn the low-variance
    components into quantisation noise: bf16 scoring of one fp32-trained
    model moved NAP AUROC by ~0.1 while BASE / SAP moved < 0.001
    (profiles/r03v_e2e_bf16_training.json).  For a bf16 model NAP therefore
    reads the diffs of an fp32 eval twin built from the same fp32 master
    weights and BN statistics (the reference's own precision); BASE / SAP stay
    on the bf16 path.  ``config.nap_dtype = 'model'`` keeps the model's own."""
    if getattr(model, "mmad_dtype", "f32") == "f32" or getattr(cfg, "nap_dtype", "f32") != "f32":
        return model
    import types
    from .model_builder import get_model
    tcfg = types.SimpleNamespace(**vars(cfg))
    tcfg.dtype = "f32"
    tcfg.gpu_id = model._native.device.index
    twin = get_model(tcfg)
    twin.load_state_dict(model.state_dict())
    twin.eval()
    return twin


class NoveltyDetecter:
    def __init__(self, config):
        self.config = config

    # ------------------------------------------------------------------ test
    def scores(self, model, train_x, valid_x, test_x):
        """(valid, test) score pairs per method: {'base','sap','nap'} ->
        (valid_score [Nv], test_score [Nt]) fp32 device tensors."""
        cfg = self.config
        model.eval()
        nat = model._native
        widths = nat.diff_widths()
        n = len(widths)
        start = getattr(cfg, "start_layer_index", 0)
        end = cfg.n_layers + 1 - getattr(cfg, "end_layer_index", -1)   # novelty_detection.py:57
        dp = model.dist if getattr(model, "dist", None) is not None and model.dist.world > 1 else None

        def rows(fn, x):
            # per-window rows of fn(x): this rank's shard, all-gathered (DP)
            if dp is None:
                return fn(x)
            return dp.gather(fn(dp.shard(x)), x.shape[0])

        out = {}
        with torch.no_grad():
            # [n_layers+1, N] per-layer sums, gathered along the windows
            lv = rows(lambda v: _layer_sq(model, v, 698).t().contiguous(), valid_x).t()
            lt = rows(lambda v: _layer_sq(model, v, 698).t().contiguous(), test_x).t()
            out["base"] = (base_from_layer_sq(lv, widths), base_from_layer_sq(lt, widths))
            out["sap"] = (sap_from_layer_sq(lv, widths, start, end), sap_from_layer_sq(lt, widths, start, end))
            nap = NapScorer(model, start_layer_index=start, end_layer_index=end)
            cuts = np.cumsum([0] + widths)
            sel = slice(int(cuts[nap.sel.start]), int(cuts[min(nap.sel.stop, n)]))
            nm = _nap_model(model, cfg)
            nap_train = rows(lambda v: _device_diffs(nm, v, cfg.batch_size)[:, sel].contiguous(), train_x)
            path = getattr(cfg, "train_diffs", None)
            if path and (dp is None or torch.distributed.get_rank(dp.group) == 0):
                torch.save(nap_train.cpu(), path)           # utils/metric.py:205
            nap = NapScorer.standalone(nap_train.shape[1], device=nat.device).fit(train_diffs=nap_train)
            del nap_train
            out["nap"] = (rows(lambda v: nap.score(_device_diffs(nm, v, 698)[:, sel]), valid_x),
                          rows(lambda v: nap.score(_device_diffs(nm, v, 698)[:, sel]), test_x))
            del nm
        return out

    def test(self, model, dset_manager, train_loader, valid_loader, test_loader, df_test=None):
        """novelty_detection.py:15-85.  Returns ((base_auroc, base_aupr),
        (sap_auroc, sap_aupr), (nap_auroc, nap_aupr), df_test) with df_test a
        list of result rows (the reference appends to a pandas DataFrame)."""
        cfg = self.config
        model.eval()
        with torch.no_grad():
            train_x, _ = dset_manager.get_transformed_data(train_loader)
            valid_x, _ = dset_manager.get_transformed_data(valid_loader)
            test_x, test_y = dset_manager.get_transformed_data(test_loader)
        test_y = np.asarray(test_y)
        if getattr(cfg, "unimodal_normal", False):
            test_y = np.where(np.isin(test_y, [cfg.target_class]), False, True)
        else:
            test_y = np.where(np.isin(test_y, [cfg.target_class]), True, False)
        self.model = model
        self.last_inputs = (train_x, valid_x, test_x, test_y)
        sc = self.scores(model, train_x, valid_x, test_x)
        row = {}
        res = {}
        for name in ("base", "sap", "nap"):
            v, t = sc[name]
            auroc, aupr, _, _ = metric.rank_metrics(t, test_y)
            thr = metric.threshold_metrics(v, t, test_y)
            row.update({f"{name}_auroc": auroc, f"{name}_aupr": aupr, f"{name}_f1score": thr[1],
                        f"{name}_precision": thr[4], f"{name}_recalls": thr[5]})
            res[name] = (auroc, aupr)
        self.last_scores = {k: (v.cpu().numpy(), t.cpu().numpy()) for k, (v, t) in sc.items()}
        self.last_row = row
        self.last_test_label = test_y
        df_test = list(df_test or []) + [row]
        return res["base"], res["sap"], res["nap"], df_test

    # ----------------------------------------------------------------- train
    def train(self, model, train_loader, valid_loader):
        """novelty_detection.py:88-127."""
        optimizer = torch.optim.Adam(model.parameters(), lr=1e-3)
        trainer = Engine(model.step)
        trainer.model, trainer.optimizer, trainer.config = model, optimizer, self.config
        trainer.train_history = []
        trainer.test_history = []
        evaluator = Engine(model.validate)
        evaluator.model, evaluator.config, evaluator.lowest_loss = model, self.config, np.inf
        evaluator.valid_history = []
        evaluator.best_model = None
        evaluator.best_epoch = 0
        model.attach(trainer, evaluator, self.config)

        def run_validation(engine, evaluator, valid_loader):
            evaluator.run(valid_loader, max_epochs=1)

        if getattr(model, "dist", None) is not None:
            # data parallel: per-shard BN running statistics averaged for eval
            # (and the sharded master weights gathered before any state_dict copy)
            trainer.add_event_handler(Events.EPOCH_COMPLETED,
                                      lambda engine: model.dist.epoch_end(model))
        trainer.add_event_handler(Events.EPOCH_COMPLETED, run_validation, evaluator, valid_loader)
        # every mini-batch's loss (the reference's step output), for trajectory checks
        self.step_losses = []
        trainer.add_event_handler(Events.ITERATION_COMPLETED,
                                  lambda engine: self.step_losses.append(float(engine.state.output[0])))

        @trainer.on(Events.EPOCH_COMPLETED)
        def append_train_loss_history(engine):
            engine.train_history += [float(engine.state.metrics["recon"])]

        @evaluator.on(Events.EPOCH_COMPLETED)
        def append_valid_loss_history(engine):
            loss = float(engine.state.metrics["recon"])
            if loss < engine.lowest_loss:
                engine.lowest_loss = loss
                engine.best_model = deepcopy(engine.model.state_dict())
                engine.best_epoch = trainer.state.epoch
            engine.valid_history += [loss]

        trainer.run(train_loader, max_epochs=self.config.n_epochs)
        if evaluator.best_model is not None:
            model.load_state_dict(evaluator.best_model)
        self.best_epoch = evaluator.best_epoch
        return trainer.train_history, evaluator.valid_history, trainer.test_history, model


def main(config):
    """novelty_detection.py:177-211 on the synthetic dataset (one process per
    GPU under torchrun: data parallel, dist.attach_data_parallel)."""
    from . import dist as mdist
    from .data_loaders import get_input_size, get_loaders
    from .model_builder import get_model
    if getattr(config, "input_size", None) is None:
        config.input_size = get_input_size(config)
    rank, world, _ = mdist.init_from_env()
    model = get_model(config)
    if world > 1:
        mdist.attach_data_parallel(model)
    detecter = NoveltyDetecter(config)
    dset_manager, train_loader, valid_loader, test_loader = get_loaders(config, rank=rank, world=world)
    _, _, _, model = detecter.train(model, train_loader, valid_loader)
    if getattr(config, "saved_name", None) and rank == 0:
        torch.save(model.state_dict(), config.saved_name)
    return detecter.test(model, dset_manager, train_loader, valid_loader, test_loader)[:3]
