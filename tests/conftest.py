import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def golden_names():
    """Forward goldens (tests/golden/gen_golden.py)."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and not f.startswith("train_"))


def train_golden_names():
    """One-training-step goldens (tests/golden/gen_golden_train.py)."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and f.startswith("train_"))


def load_train_golden(name):
    """(cfg, params, Xi int64, Xv f32, y f32, loss, logits, ref) with ref[param] = (idx or None, grad, dp, gnorm)."""
    from xsdeepfwfm_deprecated_amd import synth
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    cfg = json.loads(str(z["config"]))
    shapes = {k: tuple(v) for k, v in cfg["param_shapes"].items()}
    use_second = bool(cfg["use_fwfm"] or cfg["use_fm"])
    params = synth.synth_state(shapes, cfg["field_size"], cfg["embedding_size"], cfg["deep_nodes"], use_second,
                               bool(cfg["use_deep"]), seed=cfg["seed"])
    ref = {}
    for pname, how in cfg["stored"].items():
        idx = z[f"idx/{pname}"] if how == "sample" else None
        ref[pname] = (idx, z[f"grad/{pname}"], z[f"dp/{pname}"], float(z[f"gnorm/{pname}"]))
    return (cfg, params, z["Xi"].astype(np.int64), z["Xv"], z["y"].astype(np.float32), float(z["loss"]),
            z["logits"], ref)


def load_golden(name):
    """(cfg, params, Xi int64, Xv f32, y, logits_ref32, logits_ref64, auc_ref); params regenerated."""
    from xsdeepfwfm_deprecated_amd import synth
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    cfg = json.loads(str(z["config"]))
    shapes = {k: tuple(v) for k, v in cfg["param_shapes"].items()}
    use_second = bool(cfg["use_fwfm"] or cfg["use_fm"])
    params = synth.synth_state(shapes, cfg["field_size"], cfg["embedding_size"], cfg["deep_nodes"], use_second,
                               bool(cfg["use_deep"]), seed=cfg["seed"])
    for pname, thr in cfg.get("thresholds", {}).items():
        w = params[pname].copy()
        mask = np.abs(0.5 * (w + w.T)) < thr if pname == "field_cov.weight" else np.abs(w) < thr
        w[mask] = 0
        params[pname] = w
    return (cfg, params, z["Xi"].astype(np.int64), z["Xv"], z["y"].astype(np.int64), z["logits_ref32"],
            z["logits_ref64"], float(z["auc_ref"]))


def model_kwargs(cfg):
    return dict(field_size=cfg["field_size"], feature_sizes=cfg["feature_sizes"],
                embedding_size=cfg["embedding_size"], use_fwfm=cfg["use_fwfm"], use_fm=cfg["use_fm"],
                use_logit=cfg["use_logit"], use_deep=cfg["use_deep"], use_lw=cfg["use_lw"],
                use_fwlw=cfg["use_fwlw"], h_depth=cfg["h_depth"], deep_nodes=cfg["deep_nodes"],
                numerical=cfg["numerical"], embedding_bag=cfg["embedding_bag"], qr_flag=cfg["qr_flag"],
                qr_operation=cfg["qr_operation"], qr_collisions=cfg["qr_collisions"],
                qr_threshold=cfg["qr_threshold"], use_cuda=False)


def logit_close(got, ref, rtol=1e-5):
    """The parity bar of BASELINE.json's north_star: |d| <= 1e-5 * max(1, |ref|) per logit (fp32)."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
    return float(err.max(initial=0.0))


def logit_close_scaled(got, ref, cfg, params, Xi, Xv, rtol=1e-5):
    """logit_close with the bar scaled by the row's sum of absolute first- and second-order terms and
    |deep|: where terms of magnitude ~1e2 cancel to a logit ~1e-1 (first-order weights ~N(0,1) times Xv
    up to 63, no lw), one fp32 ulp of the partial sums already exceeds 1e-5 * max(1, |ref|) in the
    reference itself, and the order of the fp32 additions decides the last bits."""
    from oracle import dfwfm_oracle
    _, parts = dfwfm_oracle.forward(cfg, params, Xi, Xv, return_parts=True)
    if cfg.get("use_fwlw"):
        fo = np.einsum("bfd,fd->bf", parts["E"], np.asarray(params["fwfm_linear.weight"], np.float64))
    else:
        fo = dfwfm_oracle.embeddings(cfg, params, Xi, Xv, prefix="fm_1st_embeddings")[:, :, 0]
    if cfg.get("use_lw") and (cfg.get("use_fwfm") or cfg.get("use_fm")):
        fo = fo * np.asarray(params["fm_1st.weight"], np.float64)[0]
    mag = np.abs(fo).sum(1) + np.abs(parts["deep"])
    if cfg.get("use_fwfm") or cfg.get("use_fm"):
        E = parts["E"]
        G = np.abs(np.einsum("bkd,bld->bkl", E, E))
        Rs = np.ones((E.shape[1],) * 2)
        if cfg.get("use_fwfm"):
            R = np.asarray(params["field_cov.weight"], np.float64)
            Rs = np.abs(0.5 * (R + R.T))
        mag = mag + 0.5 * (G * Rs[None]).sum((1, 2))
    # bar: 1e-5 * max(1, |ref|) or 2e-7 * sum|terms| (~3 fp32 ulps of the absolute sum), the larger
    scale = np.maximum(np.maximum(1.0, np.abs(np.asarray(ref, np.float64))), mag * 2e-2)
    err = np.abs(np.asarray(got, np.float64) - np.asarray(ref, np.float64)) / scale
    return float(err.max(initial=0.0))


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from xsdeepfwfm_deprecated_amd import _lib
    _lib.lib()  # must load: no fallback
    return torch.device("cuda:0")
