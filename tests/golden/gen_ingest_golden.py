"""Golden vectors for the dataset ingest (TabularDataset, utils/data_loaders.py:
233-434), made by running the REFERENCE TabularDataset on CPU over the seeded
export tests/hsr_fixture.py writes.

Runs only in the build container (needs /root/reference); the .npz it writes is
committed and travels instead of the reference (the GPU test rewrites the same
export from the same seed).  Usage:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_ingest_golden.py

Shims (none changes what the reference computes):
* ``collections.Iterable`` for Python >= 3.10 (utils/data_loaders.py:3);
  ``librosa`` is not installed and the ingest does not use it (an empty module
  stands in for the import at :12);
* ``DataFrame.append`` was removed in pandas 2; the reference's calls
  (:263-282) get pandas 1.x's meaning, ``pd.concat([self, other],
  ignore_index=...)``;
* ``Tensor.cuda`` is the identity while the reference runs (CPU tensors);
* the hard-coded image root ``/data_ssd/hsr_dropobject/data/`` (:341, :348) is
  redirected to the fixture's image directory inside ``PIL.Image.open``;
* ``sklearn.utils.shuffle`` (no random_state, :287) draws from numpy's global
  RandomState, seeded here with the fixture's SHUFFLE_SEED right before the
  constructor -- the product takes the same seed as ``random_state``;
* HSR_Net's default init draws from torch's generator, seeded right before;
  its weights are saved with the outputs.
"""
import collections
import collections.abc
import os
import shutil
import sys
import tempfile
import types

sys.dont_write_bytecode = True
collections.Iterable = collections.abc.Iterable
sys.modules.setdefault("librosa", types.ModuleType("librosa"))
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

from tests.hsr_fixture import CASES, SHUFFLE_SEED, write_recordings  # noqa: E402

REF_ROOT = "/data_ssd/hsr_dropobject/data/"


def main():
    tmp = tempfile.mkdtemp(dir=os.path.join(REPO, "build") if os.path.isdir(
        os.path.join(REPO, "build")) else None)
    try:
        folder, img_root = write_recordings(tmp)
        pd.DataFrame.append = lambda self, other, ignore_index=False: pd.concat(
            [self, other], ignore_index=ignore_index)
        open_ = Image.open
        Image.open = lambda p, *a, **k: open_(p.replace(REF_ROOT, img_root), *a, **k)
        cuda = torch.Tensor.cuda
        torch.Tensor.cuda = lambda self, *a, **k: self
        from utils import data_loaders as dl
        captured = {}
        fwd = dl.HSR_Net.forward

        def spy(self, r, d, l, t, m):
            captured.update(r=r, d=d, t=t, m=m)
            return fwd(self, r, d, l, t, m)
        dl.HSR_Net.forward = spy
        blob = {}
        try:
            for name, c in CASES.items():
                cfg = types.SimpleNamespace(data_folder_name=folder, gpu_id=0, **c)
                captured.clear()
                np.random.seed(SHUFFLE_SEED)
                torch.manual_seed(100)
                with torch.no_grad():
                    ds = dl.TabularDataset(cfg)
                blob[f"{name}/data"] = ds.data.detach().numpy()
                blob[f"{name}/targets"] = ds.targets.numpy()
                for k, v in captured.items():
                    if v is not None:
                        blob[f"{name}/in_{k}"] = v.numpy()
                print(name, ds.data.shape, float(ds.data.mean()))
            # the HSR_Net weights every case above drew (same seed)
            torch.manual_seed(100)
            for k, v in dl.HSR_Net(False, types.SimpleNamespace(slicing_size=1)).state_dict().items():
                blob["w_" + k] = v.numpy().copy()
        finally:
            dl.HSR_Net.forward = fwd
            torch.Tensor.cuda = cuda
            Image.open = open_
        np.savez_compressed(os.path.join(HERE, "ingest.npz"), **blob)
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
