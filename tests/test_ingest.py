"""CPU: the native ingest (libdfwfm_ingest.so, include/dfwfm_ingest.h) against the reference's own
read_data output (tests/golden/ingest/ingest_tiny.npz, gen_golden_ingest.py) and a Python restatement of
utils/data_preprocess.py:54-72 on synthetic files (multi-threaded ranges, edge cases)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

NUM = set(range(1, 14))


@pytest.fixture(scope="module")
def ingest():
    from xsdeepfwfm_deprecated_amd import _lib, data
    _lib.build_ingest()
    return data


def write_map(csv, path):
    rows = [line.strip().split(",") for line in open(csv)]
    with open(path, "w") as f:
        for col in range(14, 40):
            for k in range(1, max(int(r[col]) for r in rows) + 1):
                f.write(f"{col - 1},{k},{k}\n")


def py_read(path, num_list):
    """utils/data_preprocess.py:54-72, restated (the oracle of the parser)."""
    lab, val, idx = [], [], []
    for line in open(path):
        d = line.strip().split(",")
        lab.append(int(d[0]))
        idx.append([int(x) for i, x in enumerate(d) if i not in num_list and i != 0])
        val.append([float(x) for i, x in enumerate(d) if i in num_list])
    return np.array(lab, np.int64), np.array(val, np.float64), np.array(idx, np.int64)


def test_tiny_criteo_matches_reference_read_data(ingest, tmp_path):
    z = np.load(os.path.join(GOLDEN, "ingest", "ingest_tiny.npz"))
    csv = os.path.join(GOLDEN, "ingest", "tiny_train_head.csv")
    fmap = str(tmp_path / "category_emb")
    write_map(csv, fmap)
    d = ingest.read_data(csv, fmap, NUM, feature_dim_start=0, dim=39)
    assert np.array_equal(d["label"], z["label"])
    assert np.array_equal(d["value"], z["value"]) and d["value"].dtype == np.float64
    assert np.array_equal(d["index"], z["index"])
    assert d["feature_sizes"] == z["feature_sizes"].tolist()
    # without the map: sizes from the data's largest index (the same numbers here)
    d2 = ingest.read_data(csv, str(tmp_path / "missing"), NUM, 0, 39)
    assert d2["feature_sizes"] == z["feature_sizes"].tolist()


def test_large_file_multithreaded_equals_python(ingest, tmp_path):
    rng = np.random.default_rng(0)
    n = 40000  # > 1 MiB: several parallel ranges
    path = tmp_path / "big.csv"
    with open(path, "w") as f:
        for i in range(n):
            vals = rng.integers(0, 300, 13)
            cats = rng.integers(0, 100000, 26)
            f.write(",".join([str(int(rng.random() < 0.25))] + [str(v) for v in vals] + [str(c) for c in cats]) + "\n")
    assert os.path.getsize(path) > (1 << 20)
    lab, val, idx = ingest.read_csv(str(path), NUM)
    pl, pv, pi = py_read(str(path), NUM)
    assert np.array_equal(lab, pl) and np.array_equal(val, pv) and np.array_equal(idx, pi)


def test_tokens_follow_python_int_and_float(ingest, tmp_path):
    path = tmp_path / "edge.csv"
    lines = ["1, 2.5,-3,1e3,  +4 ,0\r", "", "0,inf,-0.0,nan,7,  -12", "1,.5,5.,1E-2,8,9"]
    path.write_text("\n".join(lines))  # no trailing newline, a blank line, CRLF
    num = {1, 2, 3}
    lab, val, idx = ingest.read_csv(str(path), num)
    assert lab.tolist() == [1, 0, 1]
    assert val[0].tolist() == [2.5, -3.0, 1000.0]
    assert np.isinf(val[1][0]) and val[1][1] == 0.0 and np.signbit(val[1][1]) and np.isnan(val[1][2])
    assert val[2].tolist() == [0.5, 5.0, 0.01]
    assert idx.tolist() == [[4, 0], [7, -12], [8, 9]]


@pytest.mark.parametrize("bad,msg", [("1,2,x3\n", "line 2, column 2: invalid int"),
                                     ("1,2\n", "line 2: 2 columns, expected 3"),
                                     ("1,2.0,3\n", "invalid int '2.0'"),
                                     ("1,0x10,3\n", "invalid int")])
def test_malformed_rows_raise_with_line(ingest, tmp_path, bad, msg):
    path = tmp_path / "bad.csv"
    path.write_text("0,1,2\n" + bad)
    with pytest.raises(ValueError, match=msg):
        ingest.read_csv(str(path), set())


def test_float_column_rejects_hex_and_garbage(ingest, tmp_path):
    path = tmp_path / "bad.csv"
    for tok in ("0x10", "1.5abc", ""):
        path.write_text(f"0,{tok},2\n")
        with pytest.raises(ValueError, match="invalid float"):
            ingest.read_csv(str(path), {1})


def test_empty_file(ingest, tmp_path):
    path = tmp_path / "empty.csv"
    path.write_text("")
    lab, val, idx = ingest.read_csv(str(path), NUM)
    assert lab.shape == (0,)


def test_feature_map_counts_distinct_values(ingest, tmp_path):
    path = tmp_path / "fmap"
    path.write_text("14,a,1\n14,b,2\n14,a,3\n15,x,1\n\n39,z,9\n")
    counts = ingest.feature_map_counts(str(path), feature_dim_start=1, dim=39)
    assert counts[13] == 2 and counts[14] == 1 and counts[38] == 1 and counts.sum() == 4
    assert ingest.feature_sizes_from_counts(counts, NUM)[:15] == [1] * 13 + [3, 2]
    bad = tmp_path / "fmap_bad"
    bad.write_text("99,a,1\n")
    with pytest.raises(ValueError, match="outside"):
        ingest.feature_map_counts(str(bad), 1, 39)
