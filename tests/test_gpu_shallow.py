"""GPU: the forward without a deep tower -- the FwFM-only config of BASELINE configs[0]: the default
MLP-free fwd_kernel (PART 3, per-sample Gram FwFM) and the generic fused kernel (DFWFM_DIAG=part3=0) against the
oracle."""
import numpy as np
import pytest
import torch

from conftest import logit_close, logit_close_scaled, model_kwargs
from oracle import dfwfm_oracle

pytestmark = pytest.mark.gpu


def _case(F, num, D, *, fwlw=0, lw=1, qr=0, qr_op="mult", fm=0, logit=0, bag=0, B=300, seed=0, big=False):
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    if big:
        sizes = [1] * num + list(synth.CRITEO_FEATURE_SIZES[13:13 + F - num])
    else:
        sizes = [1] * num + [int(x) for x in 40 + (np.arange(F - num) * 53) % 700]
    second = not logit
    cfg = dict(field_size=F, feature_sizes=sizes, embedding_size=D, use_fwfm=int(second and not fm),
               use_fm=int(fm), use_logit=int(logit), use_deep=0, use_lw=lw, use_fwlw=fwlw, h_depth=3,
               deep_nodes=400, numerical=num, embedding_bag=int(bag or qr), qr_flag=qr, qr_operation=qr_op,
               qr_collisions=4, qr_threshold=200)
    m = DeepFMs(**model_kwargs(cfg))
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    params = synth.synth_state(shapes, F, D, 400, second, False, seed=seed)
    xi, xv = synth.synth_inputs(sizes, num, B, seed=seed + 1)
    return cfg, params, xi, xv


def _err(got, ref, cfg, params, xi, xv):
    """The north-star bar |d| <= 1e-5 * max(1, |ref|) where the first-order terms are projected by lw (BASELINE
    configs[0]'s model: terms ~1e1 at the init_weights scales, no cancellation to tiny logits); the bar scaled by
    the row's absolute term sum (conftest.logit_close_scaled) where they are not: without lw the ~N(0, 1) table
    weights times Xv up to 63 cancel from ~1e2 to logits ~1e-1, below one fp32 ulp of the partial sums."""
    if cfg.get("use_lw") and not cfg.get("use_logit"):
        return logit_close(got, ref)
    return logit_close_scaled(got, ref, cfg, params, xi, xv)


def _model(cfg, params, dev, monkeypatch, unused=False):
    from xsdeepfwfm_deprecated_amd import DeepFMs
    m = DeepFMs(**model_kwargs(cfg))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    m = m.to(dev).eval()
    with torch.no_grad():
        m._sync_engine(dev)  # the engine (and its kernel choice) is created here
    return m


def _run(m, xi, xv, dev):
    with torch.no_grad():
        out = m(torch.from_numpy(xi).to(dev), torch.from_numpy(xv).to(dev))
    torch.cuda.synchronize()
    return out.cpu().numpy()


CASES = [
    dict(F=39, num=13, D=10),                           # BASELINE configs[0]: FwFM + lw
    dict(F=39, num=13, D=10, lw=0),                     # FwFM, plain first-order sum
    dict(F=39, num=13, D=10, fwlw=1),                   # fwlw first order
    dict(F=39, num=13, D=10, fwlw=1, lw=0),
    dict(F=39, num=13, D=10, qr=1),                     # QR mult (tables of > 200 rows)
    dict(F=39, num=13, D=10, qr=1, qr_op="add", fwlw=1),
    dict(F=39, num=13, D=10, bag=1),                    # EmbeddingBag
    dict(F=39, num=13, D=10, fm=1),                     # FM second order
    dict(F=39, num=13, D=10, logit=1),                  # first order only (no E gather)
    dict(F=39, num=13, D=4), dict(F=39, num=13, D=8), dict(F=39, num=13, D=16), dict(F=39, num=13, D=32),
    dict(F=39, num=13, D=32, qr=1),
    dict(F=64, num=16, D=10), dict(F=64, num=0, D=10),  # four FwFM row tiles; no numerical field
    dict(F=20, num=20, D=10),                           # only numerical fields (no Xi)
    dict(F=5, num=2, D=10), dict(F=48, num=13, D=16, qr=1),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_mlp_free_kernels_match_oracle(gpu, monkeypatch, case):
    """The default MLP-free kernel (per-sample Gram FwFM) and the generic fused kernel (DFWFM_DIAG part3=0: the
    piece-wise FwFM) against the oracle over the configs without a deep tower."""
    cfg, params, xi, xv = _case(**case, seed=len(str(case)))
    ref = dfwfm_oracle.forward(cfg, params, xi, xv)
    part3 = _run(_model(cfg, params, gpu, monkeypatch), xi, xv, gpu)
    assert _err(part3, ref, cfg, params, xi, xv) < 1e-5
    monkeypatch.setenv("DFWFM_DIAG", "part3=0")
    fused = _run(_model(cfg, params, gpu, monkeypatch), xi, xv, gpu)
    monkeypatch.delenv("DFWFM_DIAG")
    assert _err(fused, ref, cfg, params, xi, xv) < 1e-5


@pytest.mark.parametrize("B", [1, 17, 4096 + 3])
def test_default_mlp_free_kernel_ragged_and_full_size(gpu, monkeypatch, B):
    """The default FwFM-only forward (fwd_kernel PART 3) at ragged batches and the Criteo-39 tables;
    a row's logit does not depend on its tile or slot."""
    cfg, params, xi, xv = _case(39, 13, 10, B=B, big=B > 4096, seed=B + 1)
    m = _model(cfg, params, gpu, monkeypatch, False)
    got = _run(m, xi, xv, gpu)
    ref = dfwfm_oracle.forward(cfg, params, xi, xv)
    assert _err(got, ref, cfg, params, xi, xv) < 1e-5
    one = _run(m, xi[B - 1:], xv[B - 1:], gpu)
    assert one[0] == got[B - 1]


@pytest.mark.parametrize("case", [dict(F=39, num=13, D=10), dict(F=39, num=13, D=10, fwlw=1, lw=0),
                                  dict(F=64, num=0, D=16), dict(F=5, num=2, D=4), dict(F=39, num=13, D=32)],
                         ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_mlp_free_four_and_eight_waves_bit_identical(gpu, monkeypatch, case):
    """PART 3 on eight waves (the default) and on four (DFWFM_DIAG p3ng=4, no QR operands): each sample's Gram sum
    is formed by one wave in the same order, so the logits are bit-identical."""
    cfg, params, xi, xv = _case(**case, B=4096 + 5, seed=11)
    got8 = _run(_model(cfg, params, gpu, monkeypatch, False), xi, xv, gpu)
    monkeypatch.setenv("DFWFM_DIAG", "p3ng=4")
    got4 = _run(_model(cfg, params, gpu, monkeypatch, False), xi, xv, gpu)
    monkeypatch.delenv("DFWFM_DIAG")
    assert np.array_equal(got4, got8)
    ref = dfwfm_oracle.forward(cfg, params, xi, xv)
    assert _err(got4, ref, cfg, params, xi, xv) < 1e-5


@pytest.mark.parametrize("bad", [-1, "n"])
def test_default_mlp_free_kernel_index_out_of_range_raises(gpu, monkeypatch, bad):
    cfg, params, xi, xv = _case(39, 13, 10, B=64, seed=3)
    xi = xi.copy()
    xi[37, 5] = -1 if bad == -1 else cfg["feature_sizes"][13 + 5]
    m = _model(cfg, params, gpu, monkeypatch, False)
    with pytest.raises(IndexError):
        _run(m, xi, xv, gpu)


def _prune_r(params, keep=0.1, seed=0):
    """The reference's R mask (model/DeepFMs.py:661-666): entries whose |(R + R^T)/2| is below the threshold are
    zeroed, so the mask is symmetric; `keep` of the off-diagonal pairs survive."""
    p = dict(params)
    W = p["field_cov.weight"].copy()
    sym = np.abs(0.5 * (W + W.T))
    F = W.shape[0]
    iu = np.triu_indices(F, 1)
    thr = np.quantile(sym[iu], 1.0 - keep)
    W[sym < thr] = 0.0
    p["field_cov.weight"] = W
    return p, int((sym[iu] >= thr).sum())


@pytest.mark.parametrize("case", [dict(F=39, num=13, D=10), dict(F=39, num=13, D=10, fwlw=1, lw=0),
                                  dict(F=64, num=0, D=16), dict(F=5, num=2, D=4), dict(F=39, num=13, D=32)],
                         ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
@pytest.mark.parametrize("B", [17, 4096 + 3])
def test_pruned_fwfm_pair_path_matches_oracle_and_gram(gpu, monkeypatch, case, B):
    """A pruned R (8 % of the pairs) takes the pair path (dfwfm_model_build_fwfm_pairs) in the MLP-free forward;
    its logits equal the oracle's and the dense Gram path's (fwfm_pair_max = 0) within the 1e-5 bar."""
    cfg, params, xi, xv = _case(**case, B=B, seed=B + 3)
    params, npairs = _prune_r(params, 0.08)
    m = _model(cfg, params, gpu, monkeypatch, False)
    m.fwfm_pair_max = 192  # opt-in (default 0: measured no faster)
    got = _run(m, xi, xv, gpu)
    assert m._engine._pairs_on and npairs <= m.fwfm_pair_max
    ref = dfwfm_oracle.forward(cfg, params, xi, xv)
    assert _err(got, ref, cfg, params, xi, xv) < 1e-5
    m.fwfm_pair_max = 0
    dense = _run(m, xi, xv, gpu)
    assert not m._engine._pairs_on
    assert _err(dense, ref, cfg, params, xi, xv) < 1e-5
    one = _run(m, xi[B - 1:], xv[B - 1:], gpu)  # a row's logit does not depend on its tile or slot
    assert one[0] == dense[B - 1]


def test_pair_list_follows_weight_updates(gpu, monkeypatch):
    """set_dense (a weight change) turns the pair path off until the list is rebuilt from the new R; a dense R
    (more than fwfm_pair_max pairs) keeps the Gram path."""
    cfg, params, xi, xv = _case(39, 13, 10, B=300, seed=21)
    pruned, _ = _prune_r(params, 0.1)
    m = _model(cfg, pruned, gpu, monkeypatch, False)
    m.fwfm_pair_max = 192
    _run(m, xi, xv, gpu)
    assert m._engine._pairs_on
    pruned2, _ = _prune_r(params, 0.05)
    with torch.no_grad():
        m.field_cov.weight.copy_(torch.from_numpy(pruned2["field_cov.weight"]))
    got = _run(m, xi, xv, gpu)
    assert m._engine._pairs_on
    ref = dfwfm_oracle.forward(cfg, pruned2, xi, xv)
    assert _err(got, ref, cfg, pruned2, xi, xv) < 1e-5
    with torch.no_grad():
        m.field_cov.weight.copy_(torch.from_numpy(params["field_cov.weight"]))  # dense R: 741 pairs
    got = _run(m, xi, xv, gpu)
    assert not m._engine._pairs_on
    ref = dfwfm_oracle.forward(cfg, params, xi, xv)
    assert _err(got, ref, cfg, params, xi, xv) < 1e-5
