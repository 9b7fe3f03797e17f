"""get_model / ae_wrapper -- model_builder.py:6-53 of the reference.

Same config fields (input_size int or (C,H,W), btl_size, n_layers, gpu_id);
``config.models`` (parsed but ignored by the reference, model_builder.py:48-49)
selects 'ae' or 'vib_ae' here.  Build extras, all optional: ``dtype``
('f32' default = reference numerics, 'bf16' = throughput path), ``vib_k``,
``beta_kl``.
"""
from .auto_encoder import AutoEncoder
from .common_utils import get_hidden_layer_sizes, flatten_input_size
from .fc_module import FCModule, Loss


def ae_wrapper(config):
    input_size = flatten_input_size(config.input_size)
    btl_size = config.btl_size
    n_layers = config.n_layers
    vib = getattr(config, "models", "ae") == "vib_ae"
    enc_out = 2 * btl_size if vib else btl_size
    encoder = FCModule(
        input_size=input_size,
        output_size=enc_out,
        hidden_sizes=get_hidden_layer_sizes(input_size, enc_out, n_hidden_layers=n_layers - 1),
        use_batch_norm=True,
        act="leakyrelu",
        last_act=None,
    )
    decoder = FCModule(
        input_size=btl_size,
        output_size=input_size,
        hidden_sizes=get_hidden_layer_sizes(btl_size, input_size, n_hidden_layers=n_layers - 1),
        use_batch_norm=True,
        act="leakyrelu",
        last_act=None,
    )
    return AutoEncoder(
        encoder=encoder,
        decoder=decoder,
        recon_loss=Loss("mse", reduction="sum"),
        dtype=getattr(config, "dtype", "f32"),
        vib=vib,
        k=getattr(config, "vib_k", 1),
        beta_kl=getattr(config, "beta_kl", 1.0),
    )


def get_model(config):
    model = ae_wrapper(config)
    if config.gpu_id >= 0:
        model = model.cuda(config.gpu_id)
    return model
