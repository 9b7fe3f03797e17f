"""The nap_wc / teacher fixtures' configuration (plain data: no reference
import, safe to import from the GPU tests).  The generators
(gen_nap_wc.py, gen_teacher.py) and the tests read it from here."""
import types

NAPWC = dict(input_size=256, btl_size=20, n_layers=5, batch_size=500, n_epochs=10,
             n_normal=10000, n_novelty=1000, anomaly_strength=0.7, data="hsr_objectdrop",
             target_class=1, unimodal_normal=False, novelty_ratio=0.0, start_layer_index=0,
             end_layer_index=-1, sensor="All", verbose=0)
SEEDS = (0, 1, 2)


def config_for(seed):
    c = types.SimpleNamespace(**NAPWC)
    c.gpu_id = -1
    c.data_seed = 500 + seed
    c.sampler_seed = 600 + seed
    c.model_seed = 700 + seed
    return c
