"""Golden vectors for the HSR_Net multimodal fusion producer, made by running
the REFERENCE ``HSR_Net`` (utils/data_loaders.py:152-229) on CPU.

Runs only in the build container (needs /root/reference); the .npz it writes is
committed and travels instead of the reference.  Usage:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_hsr_golden.py

Shims: ``collections.Iterable`` for Python>=3.10 (utils/data_loaders.py:3);
``librosa`` is not installed and HSR_Net does not use it, so an empty module
stands in for the import at utils/data_loaders.py:12; ``HSR_Net.forward``
allocates its output with ``torch.Tensor().cuda(gpu_id)`` (:181), so
``Tensor.cuda`` is made the identity while the reference runs (CPU tensors).
Weights: the reference's own default init under ``torch.manual_seed``; inputs:
seeded U[0,1] in the shapes utils/data_loaders.py:369-396 hands to the net
(r [n,1,3,32,32], d [n,1,1,32,32], t [n,1], m [n,1,1,13]).
"""
import collections
import collections.abc
import os
import sys
import types

sys.dont_write_bytecode = True
collections.Iterable = collections.abc.Iterable
sys.modules.setdefault("librosa", types.ModuleType("librosa"))
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.set_num_threads(8)


def run_case(n, seed, unimodal, mods):
    from utils.data_loaders import HSR_Net
    torch.manual_seed(seed)
    cfg = types.SimpleNamespace(slicing_size=n, gpu_id=0)
    net = HSR_Net(unimodal, cfg)
    g = torch.Generator().manual_seed(seed + 1)
    inp = {
        "r": torch.rand(n, 1, 3, 32, 32, generator=g),
        "d": torch.rand(n, 1, 1, 32, 32, generator=g),
        "t": torch.rand(n, 1, generator=g),
        "m": torch.rand(n, 1, 1, 13, generator=g),
    }
    args = [inp["r"] if "r" in mods else None, inp["d"] if "d" in mods else None, None,
            inp["t"] if "t" in mods else None, inp["m"] if "m" in mods else None]
    cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self
    try:
        with torch.no_grad():
            out = net(*args)
    finally:
        torch.Tensor.cuda = cuda
    res = {f"in_{k}": v.numpy() for k, v in inp.items() if k in mods}
    res.update({"w_" + k: v.detach().numpy().copy() for k, v in net.state_dict().items()})
    res["out"] = out.reshape(n, -1).numpy()
    return res


def main():
    cases = {
        "all": dict(n=24, seed=11, unimodal=False, mods="rdtm"),
        "hand_camera": dict(n=6, seed=12, unimodal=True, mods="r"),
        "head_depth": dict(n=6, seed=13, unimodal=True, mods="d"),
        "force_torque": dict(n=6, seed=14, unimodal=True, mods="t"),
        "mic": dict(n=6, seed=15, unimodal=True, mods="m"),
    }
    blob = {}
    for name, c in cases.items():
        r = run_case(**c)
        for k, v in r.items():
            blob[f"{name}/{k}"] = v
        print(name, r["out"].shape, float(r["out"].mean()))
    np.savez_compressed(os.path.join(HERE, "hsr.npz"), **blob)


if __name__ == "__main__":
    main()
