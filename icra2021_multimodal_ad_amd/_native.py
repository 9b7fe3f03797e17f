"""ctypes binding of libmmad.so (the C-ABI declared in include/mmad.h).

There is no fallback: if the library is missing or no GPU is visible, calls
raise ``NativeUnavailable``.  Loading the library itself needs no GPU (the CPU
test-suite checks the exported symbols).
"""
import contextlib
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MMAD_LIB", os.path.join(HERE, "libmmad.so"))

MMAD_OK = 0
MMAD_EINVAL, MMAD_EUNSUPPORTED, MMAD_EHIP, MMAD_ERCCL = -1, -2, -3, -4
F32, BF16 = 0, 1
ACT = {None: 0, "leakyrelu": 1, "relu": 2, "sigmoid": 3, "tanh": 4}

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64

# name -> (restype, argtypes); mirrors include/mmad.h one-to-one
SIGNATURES = {
    "mmad_last_error_string": (ctypes.c_char_p, []),
    "mmad_abi_version": (_I, []),
    "mmad_pad_granule": (_I, []),
    "mmad_tune_set": (_I, [_I, _I]),
    "mmad_tune_get": (_I, [_I, ctypes.POINTER(_I)]),
    "mmad_gemm_splitk_for": (_I, [_I, _I, _I, _I, _I]),
    "mmad_gemm_ws_bytes": (ctypes.c_size_t, []),
    "mmad_gemm_set_workspace": (_I, [_P, ctypes.c_size_t]),
    "mmad_gemm_status": (_I, [_P]),
    "mmad_fc_fwd": (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _F, _P, _P, _P, _P, _P]),
    "mmad_fc_fwd_mse": (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _I, _F, _P, _P, _P]),
    "mmad_fc_fwd_score": (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _F, _P, _P, _P, _P,
                               _P, _P, _I, _P]),
    "mmad_bn_eval_affine": (_I, [_I, _I, _P, _P, _P, _P, _F, _P, _P, _P]),
    "mmad_bn_train_apply": (_I, [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P,
                                 _P]),
    "mmad_nap_score": (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "mmad_fc_bwd_data": (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "mmad_fc_bwd_weight": (_I, [_I, _I, _I, _I, _P, _P, _P, _P]),
    "mmad_fc_bwd_weight_adam": (_I, [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _F, _F, _F, _F, _F, _P]),
    "mmad_bn_act_bwd_ws": (ctypes.c_size_t, [_I, _I]),
    "mmad_bn_act_bwd": (_I, [_I, _I, _F, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                             _P]),
    "mmad_act_bwd": (_I, [_I, _I, _F, _I, _I, _I, _P, _P, _P, _P, _P]),
    "mmad_activation_fwd": (_I, [_I, _F, _I, _I, _P, _I64, _P, _I64, _P]),
    "mmad_activation_bwd": (_I, [_I, _F, _I, _I, _P, _I64, _P, _I64, _P, _I64, _P]),
    "mmad_colsum": (_I, [_I, _I, _I, _P, _I, _F, _P, _P]),
    "mmad_sum": (_I, [_I64, _P, _F, _P, _I, _P]),
    "mmad_mse_loss_ws_floats": (_I, []),
    "mmad_mse_loss": (_I, [_I64, _P, _P, _I, _P, _P, _P]),
    "mmad_mse_grad": (_I, [_I64, _P, _P, _P, _I, _P, _P, _P]),
    "mmad_pack_input": (_I, [_I, _I, _I, _I, _I, _P, _I, _P, _P]),
    "mmad_unpack_output": (_I, [_I, _I, _I, _I, _P, _P, _I, _P]),
    "mmad_adam": (_I, [_I64, _P, _P, _P, _P, _F, _F, _F, _F, _F, _P, _I64, _P]),
    "mmad_vib_reparam_fwd": (_I, [_I, _I, _I, _I, _P, _I, _P, _P, _U64, _U64, _I, _P, _I, _P, _P]),
    "mmad_vib_reparam_bwd": (_I, [_I, _I, _I, _I, _P, _I, _P, _P, _I, _F, _P, _I, _P, _P]),
    "mmad_ae_create": (_I, [ctypes.POINTER(_P), _I, _I, ctypes.POINTER(_I), _I,
                            ctypes.POINTER(_I), _I, _F, _F, _F]),
    "mmad_ae_destroy": (None, [_P]),
    "mmad_ae_layout": (_I, [_P, ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "mmad_ae_workspace_bytes": (_I64, [_P, _I, _I]),
    "mmad_ae_bind": (_I, [_P, _P, _P, _P, _P, _P, _P]),
    "mmad_ae_sync_shadow": (_I, [_P, _P]),
    "mmad_ae_set_shadow_pair": (_I, [_P, _P]),
    "mmad_ae_current_shadow": (_P, [_P]),
    "mmad_ae_train_fwd_bwd": (_I, [_P, _P, _I, _I, _I, _P, _U64, _U64, _F, _P, _P, _I64, _P]),
    "mmad_ae_train_step": (_I, [_P, _P, _I, _I, _I, _P, _U64, _U64, _F, _F, _F, _F, _F, _I, _P,
                                _P, _I64, _P]),
    "mmad_ae_train_step_graph": (_I, [_P, _P, _I, _I, _I, _P, _U64, _U64, _F, _F, _F, _F, _F, _I, _P,
                                      _P, _I64, _P]),
    "mmad_ae_train_graph_count": (_I, [_P]),
    "mmad_ae_backward": (_I, [_P, _P, _I, _I, _P, _I64, _P]),
    "mmad_ae_adam": (_I, [_P, _F, _F, _F, _F, _I, _P]),
    "mmad_ae_forward": (_I, [_P, _P, _I, _I, _I, _P, _I, _P, _P, _I64, _P]),
    "mmad_ae_score": (_I, [_P, _P, _I, _I, _P, _P, _P, _I64, _P]),
    "mmad_ae_score_stream": (_I, [_P, _P, _I, _I64, _I, _P, _I64, _P, _I64, _I, _P]),
    "mmad_ae_status": (_I, [_P, _P, _I64, _P]),
    "mmad_ae_probe": (_I, [_P, _I, _I, _I]),
    "mmad_ae_probe_read": (_I, [_P, ctypes.POINTER(_F), _I]),
    "mmad_ae_probe_layers": (_I, [_P]),
    "mmad_ae_graph_count": (_I, [_P]),
    "mmad_ae_clear_graphs": (_I, [_P]),
    "mmad_comm_unique_id_bytes": (_I, []),
    "mmad_comm_get_unique_id": (_I, [_P]),
    "mmad_comm_create": (_I, [ctypes.POINTER(_P), _P, _I, _I]),
    "mmad_comm_create_loopback": (_I, [ctypes.POINTER(_P), _F]),
    "mmad_comm_create_loopback_ranks": (_I, [ctypes.POINTER(_P), _F, _I, _I]),
    "mmad_comm_destroy": (None, [_P]),
    "mmad_allreduce_bucket": (_I, [_P, _P, _I64, _P]),
    "mmad_comm_rank": (_I, [_P]),
    "mmad_comm_size": (_I, [_P]),
    "mmad_reduce_scatter_bucket": (_I, [_P, _P, _I64, _P]),
    "mmad_all_gather_bucket": (_I, [_P, _P, _I64, _I, _P]),
    "mmad_ae_dp_sync_master": (_I, [_P, _P]),
    "mmad_ae_dp_master_stale": (_I, [_P]),
    "mmad_ae_set_comm": (_I, [_P, _P]),
    "mmad_ae_adam_range": (_I, [_P, _F, _F, _F, _F, _I, _I64, _I64, _P]),
    "mmad_ae_dw_events": (_I, [_P, _I]),
    "mmad_ae_set_grad_bf16": (_I, [_P, _P]),
    "mmad_reduce_scatter_bucket_bf16": (_I, [_P, _P, _I64, _P]),
    "mmad_ae_wait_dw": (_I, [_P, _I, _P]),
    "mmad_ae_dw_plan": (_I, [_P, _I, ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I)]),
    "mmad_nap_fit_ws_bytes": (ctypes.c_size_t, [_I64, _I]),
    "mmad_minmax_norm_ws_bytes": (ctypes.c_size_t, [_I64, _I]),
    "mmad_minmax_norm": (_I, [_I64, _I, _P, _I, _I, _P, _P, ctypes.c_size_t, _P]),
    "mmad_nap_fit": (_I, [_I64, _I, _P, _I64, _P, _P, _P, _P, _P, ctypes.c_size_t, _P]),
    "mmad_rank_metrics_ws_bytes": (ctypes.c_size_t, [_I64]),
    "mmad_rank_metrics": (_I, [_I64, _P, _P, _P, _P, ctypes.c_size_t, _P]),
    "mmad_threshold_metrics_ws_bytes": (ctypes.c_size_t, [_I64]),
    "mmad_threshold_metrics": (_I, [_I64, _P, _I64, _P, _P, ctypes.c_double, _P, _P, ctypes.c_size_t, _P]),
    "mmad_hsr_weight_count": (_I, []),
    "mmad_hsr_fuse": (_I, [_I, _P, _P, _P, _P, _P, _I, _P, _I, _P]),
}


# the library's tune table (include/mmad.h, mmad_tune_set): GEMM knobs are read
# per dispatch, the schedule knobs (14-31, 33-35) when a model handle is created
KNOB = dict(tile=0, group_m=1, autotune=2, dbg=3, splitk=4, tile_adam=5, tile_bwd_data=6,
            tile_fwd=7, tile_adam_main=8, splitk_dw=9, splitk_dw_blocks=10, splitk_dw_min_stages=11,
            persist=12, bn_apply_rb=13, side_cu_held=15,
            bn_mode=16, bn_mode_bwd=17, bn_fused_rows=18, dw_main=19, pair_rows=20, dw_main_ping=21,
            ev_every=22, loss_side=23, dp_small_at=24, keep_grads=25, side_prio=26,
            event_sysfence=27, dp_shard=28, side_hold=29, dp_bucket_mib=30, ev_on_kernel=31, dw_late=33, fork_on_kernel=34, fork_pair_below=35, dp_fork_rows=14,
            splitk_dw_f32_blocks=32)
# host-side schedule choices of the Python executor wrapper (engine.py), read
# when a model is built: a second bf16 weight shadow (ping-pong), and whether
# train_step replays one captured hipGraph per step instead of the eager enqueue
SCHEDULE = {"shadow_pair": True, "train_graph": False}


def tune_get(name):
    if name in SCHEDULE:
        return SCHEDULE[name]
    v = ctypes.c_int(0)
    check(load().mmad_tune_get(KNOB[name], ctypes.byref(v)), f"tune_get({name})")
    return v.value


def tune_set(name, value):
    if name in SCHEDULE:
        SCHEDULE[name] = value
        return
    check(load().mmad_tune_set(KNOB[name], int(value)), f"tune_set({name})")


@contextlib.contextmanager
def tune(**knobs):
    """Set tune-table knobs / host schedule options for the duration of a
    ``with`` block (models created inside keep their schedule), then restore."""
    old = {k: tune_get(k) for k in knobs}
    try:
        for k, v in knobs.items():
            tune_set(k, v)
        yield
    finally:
        for k, v in old.items():
            tune_set(k, v)


class NativeUnavailable(RuntimeError):
    pass


class NativeError(RuntimeError):
    pass


_lib = None


def load():
    """Load libmmad.so (no GPU needed).  Raises NativeUnavailable if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeUnavailable(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (or `make -C icra2021_multimodal_ad_amd/csrc`)")
    # torch must own the process's HIP runtime: import it before libmmad.so so
    # the dynamic loader resolves libamdhip64.so.7 to torch's copy (one runtime)
    import torch  # noqa: F401
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error():
    """This thread's last libmmad error string."""
    return load().mmad_last_error_string().decode(errors="replace")


def check(status, what=""):
    if status != MMAD_OK:
        raise NativeError(f"{what}: status {status}: {last_error()}")


def call(name, *args):
    """Call an mmad_* entry point and raise on a non-zero status."""
    fn = getattr(load(), name)
    check(fn(*args), name)


def require_gpu(t=None):
    """Fail loudly unless the HIP path can run (no CPU fallback exists)."""
    import torch
    load()
    if not torch.cuda.is_available():
        raise NativeUnavailable("icra2021_multimodal_ad_amd needs a ROCm GPU (MI355X); "
                                "torch.cuda.is_available() is False")
    if t is not None and not t.is_cuda:
        raise NativeUnavailable("tensor must live on the GPU (call model.cuda() / get_model with "
                                "gpu_id >= 0)")


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


_gemm_ws = {}


def enable_gemm_workspace(device=None):
    """Give this thread's layer-operator GEMMs (mmad_fc_*) a split-K workspace
    on ``device`` (zeroed; kept alive here).  Returns the tensor."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    ws = _gemm_ws.get(dev)
    if ws is None:
        n = int(load().mmad_gemm_ws_bytes())
        ws = torch.zeros(n, dtype=torch.uint8, device=dev)
        _gemm_ws[dev] = ws
    call("mmad_gemm_set_workspace", ptr(ws), ws.numel())
    return ws


def pad(n, g=128):
    return (int(n) + g - 1) // g * g
