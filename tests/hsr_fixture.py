"""A small, seeded HSR object-drop export in the reference's on-disk format,
for the ingest tests (tests/test_hsr_ingest.py) and for the script that runs
the REFERENCE TabularDataset on it (tests/golden/gen_ingest_golden.py).

Layout written under ``root``:
  sum/data_sum{0..7}.csv   the schema of concatdata_maker.py:153-181 (index
                           column, 13 MFCCs, id, now_timegap, cur_depth_id,
                           cur_hand_id, cur_hand_weight, data_dir, 963 LiDAR,
                           label), ROWS rows each
  sum/data_small0.csv      a ninth file for the file_name != 'data_sum' path
  sum/objectsplit.csv      object type -> recording directories
  img/{dir}/data/img/hand/{id}.png   RGB  64x48 (uint8)
  img/{dir}/data/img/d/{id}.png      I;16 64x48 (uint16)
Column mfcc05 is constant (norm_vec_np's 0/0 -> 0 path).  Everything is a
function of the seed: the same bytes on every machine.
"""
import os

import numpy as np

ROWS = 6
DIRS = {"cracker": ["cracker_00", "cracker_01"], "book": ["book_00", "book_01"],
        "doll": ["doll_00", "doll_01"]}
IDS_PER_DIR = 5


def write_recordings(root, seed=0):
    import pandas as pd
    from PIL import Image

    rng = np.random.Generator(np.random.PCG64(seed))
    sum_dir = os.path.join(root, "sum")
    os.makedirs(sum_dir, exist_ok=True)
    dirs = [d for v in DIRS.values() for d in v]
    for dd in dirs:
        for kind in ("hand", "d"):
            os.makedirs(os.path.join(root, "img", dd, "data", "img", kind), exist_ok=True)
        for i in range(IDS_PER_DIR):
            rgb = rng.integers(0, 256, size=(48, 64, 3), dtype=np.uint8)
            Image.fromarray(rgb, mode="RGB").save(
                os.path.join(root, "img", dd, "data", "img", "hand", "%d.png" % i))
            dep = rng.integers(300, 4000, size=(48, 64), dtype=np.uint16)
            Image.fromarray(dep).save(os.path.join(root, "img", dd, "data", "img", "d", "%d.png" % i))

    def frame(n):
        cols = {}
        for j in range(13):
            cols["mfcc%02d" % j] = (np.full(n, 1.5) if j == 5 else rng.normal(0, 10, n))
        cols["id"] = rng.integers(0, 10 ** 6, n)
        cols["now_timegap"] = np.round(rng.uniform(0, 30, n), 1)
        cols["cur_depth_id"] = rng.integers(0, IDS_PER_DIR, n).astype(np.float64)
        cols["cur_hand_id"] = rng.integers(0, IDS_PER_DIR, n).astype(np.float64)
        cols["cur_hand_weight"] = rng.normal(0.5, 0.2, n)
        cols["data_dir"] = [dirs[k] for k in rng.integers(0, len(dirs), n)]
        for j in range(963):
            cols["LiDAR%03d" % j] = np.round(rng.uniform(0, 5, n), 3)
        cols["label"] = (rng.uniform(size=n) < 0.3).astype(np.int64)
        return pd.DataFrame(cols)

    for k in range(8):
        frame(ROWS).to_csv(os.path.join(sum_dir, "data_sum%d.csv" % k))
    frame(ROWS).to_csv(os.path.join(sum_dir, "data_small0.csv"))
    pd.DataFrame(DIRS).to_csv(os.path.join(sum_dir, "objectsplit.csv"), index=False)
    return sum_dir + "/", os.path.join(root, "img") + "/"


# ingest cases: name -> config fields (the reference's argparse names)
CASES = {
    "All": dict(sensor="All", file_name="data_sum", object_select_mode=False, slicing_size=40),
    "hand_camera": dict(sensor="hand_camera", file_name="data_sum", object_select_mode=False,
                        slicing_size=24),
    "head_depth": dict(sensor="head_depth", file_name="data_sum", object_select_mode=False,
                       slicing_size=24),
    "force_torque": dict(sensor="force_torque", file_name="data_sum", object_select_mode=False,
                         slicing_size=24),
    "mic": dict(sensor="mic", file_name="data_sum", object_select_mode=False, slicing_size=24),
    "All_objects": dict(sensor="All", file_name="data_sum", object_select_mode=True,
                        object_type="book", slicing_size=8),
    "All_small": dict(sensor="All", file_name="data_small", object_select_mode=False,
                      slicing_size=5),
}
SHUFFLE_SEED = 7
