"""CPU: pin the oracle (float64 restatement) and the fp32 torch port to the reference's golden vectors."""
import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden, logit_close
from oracle import dfwfm_oracle, torch_port


@pytest.mark.parametrize("name", golden_names())
def test_oracle_matches_reference_float64(name):
    cfg, params, xi, xv, y, l32, l64, auc = load_golden(name)
    got = dfwfm_oracle.forward(cfg, params, xi, xv)
    # both are float64 evaluations of the same algebra: only summation order differs
    assert logit_close(got, l64, rtol=0) < 1e-11


@pytest.mark.parametrize("name", golden_names())
def test_oracle_vs_reference_fp32_within_parity_bar(name):
    cfg, params, xi, xv, y, l32, l64, auc = load_golden(name)
    got = dfwfm_oracle.forward(cfg, params, xi, xv)
    assert logit_close(got, l32) < 1e-5


@pytest.mark.parametrize("name", golden_names())
def test_torch_port_matches_reference_fp32(name):
    cfg, params, xi, xv, y, l32, l64, auc = load_golden(name)
    tp = {k: torch.from_numpy(v) for k, v in params.items()}
    got = torch_port.forward(cfg, tp, torch.from_numpy(xi), torch.from_numpy(xv)).numpy()
    assert logit_close(got, l32) < 1e-5


@pytest.mark.parametrize("name", ["tiny_fwfm_lw", "tiny_deepfwfm_lw"])
def test_oracle_auc_matches_reference(name):
    from sklearn.metrics import roc_auc_score
    cfg, params, xi, xv, y, l32, l64, auc = load_golden(name)
    got = roc_auc_score(y, dfwfm_oracle.sigmoid(dfwfm_oracle.forward(cfg, params, xi, xv)))
    assert abs(got - auc) <= 1e-4


def _latency_model_as_params(dims, emb=10):
    """The C++ latency model's init_FM weights (latency/criteo_latency.cpp:201-212) as a DeepFMs state."""
    params = {"bias": np.zeros(1, np.float32)}
    for f, n in enumerate(dims):
        j = np.arange(n, dtype=np.float64)
        params[f"fm_1st_embeddings.{f}.weight"] = (j * j * 1.11).astype(np.float32)[:, None]
        params[f"fm_2nd_embeddings.{f}.weight"] = np.repeat((1.2 * j).astype(np.float32)[:, None], emb, 1)
    params["field_cov.weight"] = np.ones((len(dims), len(dims)), np.float32)
    return params


def test_known_answer_cpp_latency_fwfm():
    """Known answer from the reference's own C++ FwFM (latency/criteo_latency.cpp:86-103) on its fixed
    sample (:231-232).  Numerical fields carry Xi = 0 there, so their rows (j = 0) are zero in both
    formulations and the C++ sum equals the Python model's FwFM-only, plain-sum first order."""
    Xi = [0] * 13 + [10, 10, 10, 10, 10, 10, 10, 10, 3, 10, 10, 10, 10, 10, 10, 10, 5, 10, 10, 4, 10, 10, 10, 100,
                     10, 10]
    Xv = [1.1, 2.1, 3.1, 4.1, 5.1, 6.1, 7.1, 8.1, 9.1, 10.1, 11.1, 12.1, 13.1] + [1.0] * 26
    dims = [1] * 13 + [max(x + 1, 2) for x in Xi[13:]]
    kat = dfwfm_oracle.latency_fwfm_known_answer(Xi, Xv, dims)
    cfg = dict(field_size=39, numerical=13, embedding_size=10, use_fwfm=1, use_deep=0, use_lw=0, use_fwlw=0)
    params = _latency_model_as_params(dims)
    got = dfwfm_oracle.forward(cfg, params, np.array([Xi[13:]]), np.array([Xv[:13]], np.float32))[0]
    # closed form: sum_cat 1.11 x^2 + 10 * 1.44 * sum_{i<j} x_i x_j
    x = np.array(Xi[13:], np.float64)
    closed = (1.11 * x * x).sum() + 14.4 * ((x.sum() ** 2 - (x * x).sum()) / 2)
    assert abs(got - closed) <= 1e-9 * closed
    assert abs(got - kat) <= 1e-5 * abs(kat)


def test_oracle_index_out_of_range_raises():
    cfg, params, xi, xv, *_ = load_golden("deepfwfm_lw")
    bad = xi[:4].copy()
    bad[2, 5] = cfg["feature_sizes"][13 + 5]
    with pytest.raises(IndexError):
        dfwfm_oracle.forward(cfg, params, bad, xv[:4])
