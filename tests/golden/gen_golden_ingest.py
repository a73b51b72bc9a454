"""Golden vectors for the native ingest (reference utils/data_preprocess.py:18-26, :54-72).

Run in the build container only (imports /root/reference):

    python tests/golden/gen_golden_ingest.py

Input: tests/golden/ingest/tiny_train_head.csv (the first 1000 rows of the reference's
data/tiny_train_input.csv, a data fixture) and a feature map written the way SURVEY.md §8c's probe
synthesised the missing data/category_emb (one "field,value,index" line per index 1..max of each
categorical column, field ids 13..38 for feature_dim_start=0).  Output: the reference read_data's
label / value / index / feature_sizes as arrays.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CSV = os.path.join(HERE, "ingest", "tiny_train_head.csv")
FMAP = os.path.join(HERE, "ingest", "tiny_category_emb")


def write_feature_map():
    rows = [line.strip().split(",") for line in open(CSV)]
    with open(FMAP, "w") as f:
        for col in range(14, 40):
            mx = max(int(r[col]) for r in rows)
            for k in range(1, mx + 1):
                f.write(f"{col - 1},{k},{k}\n")


if __name__ == "__main__":
    sys.path.insert(0, os.environ.get("DFWFM_REF", "/root/reference"))
    from utils import data_preprocess  # noqa: E402
    write_feature_map()
    d = data_preprocess.read_data(CSV, FMAP, set(range(1, 14)), feature_dim_start=0, dim=39)
    np.savez_compressed(os.path.join(HERE, "ingest", "ingest_tiny.npz"), label=np.array(d["label"], dtype=np.int64),
                        value=np.array(d["value"], dtype=np.float64), index=np.array(d["index"], dtype=np.int64),
                        feature_sizes=np.array(d["feature_sizes"], dtype=np.int64))
    print("rows", len(d["label"]), "feature_sizes", d["feature_sizes"])
