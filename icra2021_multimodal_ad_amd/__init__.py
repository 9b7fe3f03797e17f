"""MI355X-native autoencoder train-and-score hot path of
Yoo-Youngjae/ICRA2021_multimodal_ad (FC autoencoder + RaPP scoring), behind
the reference's plugin surface (get_model / AbstractModel / AutoEncoder /
FCModule / FCLayer / get_diffs).  Compute runs in hand-written gfx950 HIP
kernels (libmmad.so, C-ABI in include/mmad.h); there is no CPU fallback.
"""
from .common_utils import get_hidden_layer_sizes, init_state_dict  # noqa: F401
from .data import get_input_size, synth_windows  # noqa: F401

__all__ = ["get_model", "AutoEncoder", "FCModule", "FCLayer", "get_diffs", "score_windows"]


def __getattr__(name):
    # lazy: importing the package must not require the native library
    if name == "get_model":
        from .model_builder import get_model
        return get_model
    if name == "AutoEncoder":
        from .auto_encoder import AutoEncoder
        return AutoEncoder
    if name in ("FCModule", "FCLayer", "Activation", "Loss"):
        from . import fc_module
        return getattr(fc_module, name)
    if name in ("get_diffs", "score_windows"):
        from . import reconstruction_aggregation
        return getattr(reconstruction_aggregation, name)
    raise AttributeError(name)
