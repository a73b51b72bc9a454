"""Data ingest of the reference harness (utils/data_preprocess.py, model/Datasets.py:get_dataset) on the
native reader (include/dfwfm_ingest.h).

``read_data`` / ``load_category_index`` / ``get_feature_sizes`` keep the reference's signatures and
return the same contents -- label, value (numerical columns), index (categorical columns),
feature_sizes -- as numpy arrays instead of lists of lists (``fit`` converts both the same way:
``np.array(Xi).reshape(-1, F - num, 1)``, ``np.array(Xv)``).  ``get_dataset`` follows
model/Datasets.py:22-80 for the Criteo datasets.
"""
from __future__ import annotations

import ctypes
import logging
import os

import numpy as np

from . import _lib

CRITEO_NUM_FEAT_DIM = set(range(1, 14))  # model/Datasets.py:23
_log = logging.getLogger("xsDeepFwFM")


def _threads():
    return max(1, min(len(os.sched_getaffinity(0)), 32))


def _check(rc, what):
    if rc != 0:
        msg = _lib.ingest_lib().dfwfm_ingest_last_error().decode(errors="replace")
        raise ValueError(f"{what}: {msg}")


def feature_map_counts(emb_file, feature_dim_start=0, dim=39):
    """Distinct values per field of a "field,value,index" feature map (load_category_index, :18-26)."""
    counts = np.zeros(dim, dtype=np.int64)
    _check(_lib.ingest_lib().dfwfm_feature_map_counts(os.fsencode(emb_file), int(feature_dim_start), int(dim),
                                                        counts.ctypes.data_as(ctypes.c_void_p)), emb_file)
    return counts


def feature_sizes_from_counts(counts, num_list):
    """[1] * len(num_list) + [count + 1 for every field whose 1-based column is not numerical] (:57-61)."""
    sizes = [1] * len(num_list)
    for num, c in enumerate(counts):
        if num + 1 not in num_list:
            sizes.append(int(c) + 1)
    return sizes


def load_category_index(file_path, feature_dim_start=0, dim=39):
    """Reference :18-26 returns one dict per field; the ingest only needs their sizes, so this returns
    a list of per-field distinct-value counts (len(cate_dict[f]))."""
    return feature_map_counts(file_path, feature_dim_start, dim).tolist()


def read_csv(file_path, num_list):
    """label int64 [n], value float64 [n, #num], index int64 [n, #cat] of a "label,c1,...,cC" CSV."""
    L = _lib.ingest_lib()
    h = ctypes.c_void_p()
    rows, cols = ctypes.c_int64(), ctypes.c_int32()
    _check(L.dfwfm_csv_open(os.fsencode(file_path), _threads(), ctypes.byref(h), ctypes.byref(rows),
                            ctypes.byref(cols)), file_path)
    try:
        n, C = rows.value, cols.value
        is_num = np.zeros(max(C, 1), dtype=np.uint8)
        for c in num_list:
            if 0 < c < C:
                is_num[c] = 1
        nv = int(is_num[1:].sum())
        labels = np.empty(n, dtype=np.int64)
        values = np.empty((n, nv), dtype=np.float64)
        index = np.empty((n, max(C - 1 - nv, 0)), dtype=np.int64)
        ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        _check(L.dfwfm_csv_parse(h, ptr(is_num), ptr(labels), ptr(values), ptr(index), _threads()), file_path)
    finally:
        L.dfwfm_csv_close(h)
    return labels, values, index


def read_data(file_path, emb_file, num_list, feature_dim_start=0, dim=39):
    """Reference utils/data_preprocess.py:54-72 (label, value, index, feature_sizes).  When the feature
    map is missing (the reference's tiny-criteo `data/category_emb` is not shipped) the
    sizes come from the largest index of each categorical column + 1 (= what a map with one entry per
    index 1..max gives), with a warning."""
    labels, values, index = read_csv(file_path, num_list)
    if emb_file is not None and os.path.exists(emb_file):
        sizes = feature_sizes_from_counts(feature_map_counts(emb_file, feature_dim_start, dim), num_list)
    else:
        _log.warning("feature map %s missing: feature sizes from the data's largest indices", emb_file)
        sizes = [1] * len(num_list) + [int(v) + 1 for v in (index.max(axis=0) if len(index) else
                                                               np.zeros(index.shape[1], np.int64))]
    return {"label": labels, "value": values, "index": index, "feature_sizes": sizes}


def get_feature_sizes(emb_file, num_list, feature_dim_start=0, dim=39, twitter=False):
    """Reference :127-138."""
    counts = feature_map_counts(emb_file, feature_dim_start, dim)
    if twitter:
        return {"label": [], "value": [], "index": [], "feature_sizes": [1] * len(num_list) +
                [int(c) + 1 for c in counts if c > 0]}
    return {"label": [], "value": [], "index": [], "feature_sizes": feature_sizes_from_counts(counts, num_list)}


def get_dataset(pars, root="."):
    """model/Datasets.py:22-80 for 'tiny-criteo' and 'criteo' (twitter / ali / avazu readers are out of
    scope: other datasets, not the Criteo-39 hot path).  Returns (field_size, train, valid, test);
    feature sizes are the union over the three splits when no feature map exists."""
    join = lambda *p: os.path.join(root, *p)  # noqa: E731
    if pars.dataset == "tiny-criteo":
        fm = join("data", "category_emb")
        tr = read_data(join("data", "tiny_train_input.csv"), fm, CRITEO_NUM_FEAT_DIM, 0, 39)
        va = read_data(join("data", "tiny_test_input.csv"), fm, CRITEO_NUM_FEAT_DIM, 0, 39)
        te = read_data(join("data", "tiny_test_input.csv"), fm, CRITEO_NUM_FEAT_DIM, 0, 39)
    elif pars.dataset == "criteo":
        fm = join("data", "large", "criteo_feature_map")
        tr = read_data(join("data", "large", "criteo_train.csv"), fm, CRITEO_NUM_FEAT_DIM, 1, 39)
        va = read_data(join("data", "large", "criteo_valid.csv"), fm, CRITEO_NUM_FEAT_DIM, 1, 39)
        te = read_data(join("data", "large", "criteo_test.csv"), fm, CRITEO_NUM_FEAT_DIM, 1, 39)
    else:
        raise NotImplementedError(f"dataset {pars.dataset!r}: only the Criteo-39 datasets are in scope")
    sizes = [max(a, b, c) for a, b, c in zip(tr["feature_sizes"], va["feature_sizes"], te["feature_sizes"])]
    for d in (tr, va, te):
        d["feature_sizes"] = sizes
    return 39, tr, va, te
