"""Shape helpers and deterministic parameter init.

``get_hidden_layer_sizes`` restates utils/common_utils.py:22-31 of the
reference (it defines every GEMM shape on the path).  ``init_state_dict``
replaces the reference's unseeded torch init with a seeded numpy PCG64 draw of
the same distribution (nn.Linear: U(-1/sqrt(in), 1/sqrt(in)) for weight and
bias; BatchNorm1d: gamma=1, beta=0, running mean 0 / var 1), so the GPU path,
the CPU oracle and the reference can start from identical weights.
"""
import numpy as np


def get_hidden_layer_sizes(start_size, end_size, n_hidden_layers):
    """utils/common_utils.py:22-31: ``int(start - diff*(i+1))``, float diff."""
    sizes = []
    diff = (start_size - end_size) / (n_hidden_layers + 1)
    for idx in range(n_hidden_layers):
        sizes.append(int(start_size - (diff * (idx + 1))))
    return sizes


def flatten_input_size(input_size):
    """model_builder.py:14-19: (C,H,W) inputs are flattened."""
    if not isinstance(input_size, int):
        c, h, w = input_size
        return int(c * h * w)
    return int(input_size)


def ae_widths(input_size, btl_size, n_layers, enc_out=None):
    """Encoder / decoder width lists as built by model_builder.py:21-37.
    ``enc_out`` = 2*btl for the VIB head."""
    d = flatten_input_size(input_size)
    eo = btl_size if enc_out is None else enc_out
    enc = [d] + get_hidden_layer_sizes(d, eo, n_layers - 1) + [eo]
    dec = [btl_size] + get_hidden_layer_sizes(btl_size, d, n_layers - 1) + [d]
    return enc, dec


def state_dict_keys(n_layers, prefix):
    """Reference state_dict key layout of one FCModule (modules/fc_module.py:
    34-51 registers ``net``; layers/fc_layer.py:31-33 names layer/bn)."""
    keys = []
    for i in range(n_layers):
        keys += [f"{prefix}.net.{i}.layer.weight", f"{prefix}.net.{i}.layer.bias"]
        if i < n_layers - 1:
            keys += [f"{prefix}.net.{i}.bn.{n}" for n in
                     ("weight", "bias", "running_mean", "running_var", "num_batches_tracked")]
    return keys


def init_state_dict(input_size, btl_size, n_layers, seed=0, enc_out=None):
    """Seeded init in reference state_dict layout (numpy arrays)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    enc, dec = ae_widths(input_size, btl_size, n_layers, enc_out)
    sd = {}
    for prefix, widths in (("encoder", enc), ("decoder", dec)):
        for i, (fi, fo) in enumerate(zip(widths[:-1], widths[1:])):
            bound = 1.0 / np.sqrt(fi)
            sd[f"{prefix}.net.{i}.layer.weight"] = rng.uniform(-bound, bound, (fo, fi)).astype(np.float32)
            sd[f"{prefix}.net.{i}.layer.bias"] = rng.uniform(-bound, bound, (fo,)).astype(np.float32)
            if i < len(widths) - 2:
                sd[f"{prefix}.net.{i}.bn.weight"] = np.ones(fo, np.float32)
                sd[f"{prefix}.net.{i}.bn.bias"] = np.zeros(fo, np.float32)
                sd[f"{prefix}.net.{i}.bn.running_mean"] = np.zeros(fo, np.float32)
                sd[f"{prefix}.net.{i}.bn.running_var"] = np.ones(fo, np.float32)
                sd[f"{prefix}.net.{i}.bn.num_batches_tracked"] = np.zeros((), np.int64)
    return sd
