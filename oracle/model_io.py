"""State-dict <-> oracle-model conversion (TEST INFRASTRUCTURE ONLY; see
ae_oracle.py header).  Key layout: model_builder.py:21-37 + modules/
fc_module.py:50-51 (``{encoder,decoder}.net.{i}.layer.*`` / ``.bn.*``)."""
import numpy as np


def model_from_state_dict(sd, prefix=""):
    model = {}
    for side, name in (("enc", "encoder"), ("dec", "decoder")):
        layers = []
        i = 0
        while f"{prefix}{name}.net.{i}.layer.weight" in sd:
            p = f"{prefix}{name}.net.{i}."
            layer = {"W": np.array(sd[p + "layer.weight"], np.float32),
                     "b": np.array(sd[p + "layer.bias"], np.float32),
                     "act": None, "bn": None}
            if p + "bn.weight" in sd:
                layer["act"] = "leakyrelu"
                layer["bn"] = {"gamma": np.array(sd[p + "bn.weight"], np.float32),
                               "beta": np.array(sd[p + "bn.bias"], np.float32),
                               "rm": np.array(sd[p + "bn.running_mean"], np.float32),
                               "rv": np.array(sd[p + "bn.running_var"], np.float32),
                               "nbt": int(np.asarray(sd.get(p + "bn.num_batches_tracked", 0)))}
            layers.append(layer)
            i += 1
        model[side] = layers
    return model


def state_dict_from_model(model):
    sd = {}
    for side, name in (("enc", "encoder"), ("dec", "decoder")):
        for i, layer in enumerate(model[side]):
            p = f"{name}.net.{i}."
            sd[p + "layer.weight"] = layer["W"]
            sd[p + "layer.bias"] = layer["b"]
            if layer["bn"] is not None:
                bn = layer["bn"]
                sd[p + "bn.weight"] = bn["gamma"]
                sd[p + "bn.bias"] = bn["beta"]
                sd[p + "bn.running_mean"] = bn["rm"]
                sd[p + "bn.running_var"] = bn["rv"]
                sd[p + "bn.num_batches_tracked"] = np.int64(bn["nbt"])
    return sd


def grads_to_flat(grads):
    """oracle grads {"enc":[{W,b,gamma,beta}...]} -> reference parameter names."""
    out = {}
    for side, name in (("enc", "encoder"), ("dec", "decoder")):
        for i, g in enumerate(grads[side]):
            p = f"{name}.net.{i}."
            out[p + "layer.weight"] = g["W"]
            out[p + "layer.bias"] = g["b"]
            if "gamma" in g:
                out[p + "bn.weight"] = g["gamma"]
                out[p + "bn.bias"] = g["beta"]
    return out
