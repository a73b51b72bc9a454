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
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz"))


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


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from xsdeepfwfm_deprecated_amd import _lib
    _lib.lib()  # must load: no fallback
    return torch.device("cuda:0")
