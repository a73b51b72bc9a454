"""GPU: the HIP forward (through the C ABI) against the reference's golden vectors and the oracle."""
import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden, logit_close, model_kwargs
from oracle import dfwfm_oracle

pytestmark = pytest.mark.gpu


def make_model(cfg, params, device):
    from xsdeepfwfm_deprecated_amd import DeepFMs
    m = DeepFMs(**model_kwargs(cfg))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    return m.to(device).eval()


def run(m, xi, xv, device):
    with torch.no_grad():
        out = m(torch.from_numpy(xi).to(device), torch.from_numpy(xv).to(device))
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("name", golden_names())
def test_forward_matches_reference(gpu, name):
    cfg, params, xi, xv, y, l32, l64, auc = load_golden(name)
    m = make_model(cfg, params, gpu)
    got = run(m, xi.reshape(len(xi), -1, 1), xv, gpu)
    assert got.dtype == np.float32 and got.shape == l32.shape
    assert logit_close(got, l32) < 1e-5, name
    assert logit_close(got, l64) < 1e-5, name


@pytest.mark.parametrize("name", ["tiny_fwfm_lw", "tiny_deepfwfm_lw"])
def test_auc_matches_reference(gpu, name):
    from sklearn.metrics import roc_auc_score
    cfg, params, xi, xv, y, l32, l64, auc = load_golden(name)
    m = make_model(cfg, params, gpu)
    got = run(m, xi, xv, gpu)
    assert abs(roc_auc_score(y, dfwfm_oracle.sigmoid(got)) - auc) <= 1e-4


@pytest.mark.parametrize("B", [1, 2, 15, 16, 17, 37, 100, 255])
def test_ragged_batches(gpu, B):
    cfg, params, xi, xv, y, l32, l64, auc = load_golden("deepfwfm_qr_mult")
    m = make_model(cfg, params, gpu)
    got = run(m, xi[:B], xv[:B], gpu)
    assert logit_close(got, l32[:B]) < 1e-5
    # a row's logit does not depend on its batch-mates or its slot in the 16-row tile
    full = run(m, xi, xv, gpu)
    off = run(m, xi[3:3 + B], xv[3:3 + B], gpu)
    assert np.array_equal(full[:B], got) and np.array_equal(full[3:3 + B], off)


def test_empty_batch(gpu):
    cfg, params, xi, xv, *_ = load_golden("deepfwfm_lw")
    m = make_model(cfg, params, gpu)
    assert run(m, xi[:0], xv[:0], gpu).shape == (0,)


@pytest.mark.parametrize("bad", [-1, "n"])
def test_index_out_of_range_raises(gpu, bad):
    cfg, params, xi, xv, *_ = load_golden("deepfwfm_lw")
    m = make_model(cfg, params, gpu)
    x = xi[:8].copy()
    x[5, 3] = cfg["feature_sizes"][13 + 3] if bad == "n" else -1
    with pytest.raises(IndexError):
        run(m, x, xv[:8], gpu)
    # the flag is sticky only until read: a clean batch afterwards passes
    run(m, xi[:8], xv[:8], gpu)


def test_batched_callers_read_the_index_flag_once(gpu, monkeypatch):
    """eval_by_batch / predict_proba / run_benchmark do not synchronise on the index flag per batch: one read
    at the end, which still raises IndexError for a bad row in any batch."""
    cfg, params, xi, xv, y, *_ = load_golden("deepfwfm_lw")
    m = make_model(cfg, params, gpu)
    reads = []
    orig = m.check_index_errors
    monkeypatch.setattr(m, "check_index_errors", lambda: (reads.append(1), orig())[1])
    n = len(xi)
    m.eval_by_batch(xi, xv, y, n)
    assert len(reads) == 1
    m.predict_proba(xi, xv)
    assert len(reads) == 2
    bad = xi.copy()
    bad[n - 1, 2] = -1  # in the last batch
    with pytest.raises(IndexError):
        m.eval_by_batch(bad, xv, y, n)
    m.eval_by_batch(xi, xv, y, n)  # the flag was cleared by the raising read


def test_qr_index_range_follows_quotient_table(gpu):
    # QREmbeddingBag rejects only i // c >= ceil(n/c): i = n (inside the last quotient row) is valid
    cfg, params, xi, xv, l32, *_ = load_golden("deepfwfm_qr_mult")[:5]
    sizes = cfg["feature_sizes"]
    f = next(j for j in range(13, 39) if sizes[j] > cfg["qr_threshold"] and sizes[j] % cfg["qr_collisions"])
    m = make_model(cfg, params, gpu)
    x = xi[:4].copy()
    x[1, f - 13] = sizes[f]
    got = run(m, x, xv[:4], gpu)
    ref = dfwfm_oracle.forward(cfg, params, x, xv[:4])
    assert logit_close(got, ref) < 1e-5


def test_layouts_and_strides(gpu):
    cfg, params, xi, xv, y, l32, *_ = load_golden("deepfwfm_fwlw_lw")
    m = make_model(cfg, params, gpu)
    wide = np.concatenate([xv, np.full((len(xv), 26), 7.0, np.float32)], axis=1)  # Xv with 39 columns
    got = run(m, xi[:, :, None], wide, gpu)
    assert logit_close(got, l32) < 1e-5
    # non-contiguous Xi view (every other row)
    xt = torch.from_numpy(xi).to(gpu)[::2]
    with torch.no_grad():
        g2 = m(xt, torch.from_numpy(xv).to(gpu)[::2]).cpu().numpy()
    assert logit_close(g2, l32[::2]) < 1e-5


def test_weight_update_is_picked_up(gpu):
    cfg, params, xi, xv, y, l32, *_ = load_golden("deepfwfm_lw")
    m = make_model(cfg, params, gpu)
    run(m, xi, xv, gpu)
    with torch.no_grad():
        m.field_cov.weight.mul_(0.5)
        m.net_1_linear_2.weight.mul_(-1.0)
        m.fm_2nd_embeddings[20].weight.add_(0.125)
    p2 = dict(params)
    p2["field_cov.weight"] = params["field_cov.weight"] * 0.5
    p2["net_1_linear_2.weight"] = -params["net_1_linear_2.weight"]
    p2["fm_2nd_embeddings.20.weight"] = params["fm_2nd_embeddings.20.weight"] + np.float32(0.125)
    got = run(m, xi, xv, gpu)
    assert logit_close(got, dfwfm_oracle.forward(cfg, p2, xi, xv)) < 1e-5


# ---------------------------------------------------------------- full Criteo-39 size
@pytest.fixture(scope="module")
def criteo(gpu):
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = synth.CRITEO_FEATURE_SIZES
    m = DeepFMs(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_deep=1, use_lw=1,
                use_fwlw=0, use_fm=0, numerical=13, use_cuda=False)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    params = synth.synth_state(shapes, 39, 10, 400, True, True, seed=1234)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    m = m.to(gpu).eval()
    cfg = dict(field_size=39, numerical=13, embedding_size=10, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1,
               use_fwlw=0, h_depth=3, deep_nodes=400)
    return m, cfg, params, sizes


def test_criteo_size_vs_oracle(criteo, gpu):
    from xsdeepfwfm_deprecated_amd import synth
    m, cfg, params, sizes = criteo
    xi, xv = synth.synth_inputs(sizes, 13, 4096, seed=7)
    got = run(m, xi, xv, gpu)
    sel = np.arange(0, 4096, 8)
    ref = dfwfm_oracle.forward(cfg, params, xi[sel], xv[sel])
    assert logit_close(got[sel], ref) < 1e-5


def test_criteo_size_properties_large_batch(criteo, gpu):
    """Size-independent properties at 64k rows: deterministic, permutation-equivariant, split-invariant."""
    from xsdeepfwfm_deprecated_amd import synth
    m, cfg, params, sizes = criteo
    xi, xv = synth.zipf_inputs(sizes, 13, 65536, seed=3)
    a = run(m, xi, xv, gpu)
    b = run(m, xi, xv, gpu)
    assert np.array_equal(a, b)
    perm = np.random.default_rng(0).permutation(len(xi))
    c = run(m, xi[perm], xv[perm], gpu)
    assert np.array_equal(c, a[perm])
    d = np.concatenate([run(m, xi[:12345], xv[:12345], gpu), run(m, xi[12345:], xv[12345:], gpu)])
    assert np.array_equal(d, a)
    sel = np.arange(0, 65536, 997)
    assert logit_close(a[sel], dfwfm_oracle.forward(cfg, params, xi[sel], xv[sel])) < 1e-5


@pytest.mark.parametrize("n,levels,rate", [(1000, 0, 0.3), (50000, 64, 0.25), (123457, 0, 0.02), (4097, 3, 0.5)])
def test_device_metrics_match_sklearn(gpu, n, levels, rate):
    """DeviceMetrics == sklearn roc_auc_score / precision_recall_curve+auc / log_loss / RCE (the reference's
    eval_by_batch metrics, :777-800), including heavily tied predictions."""
    from sklearn.metrics import auc, log_loss, precision_recall_curve, roc_auc_score
    from xsdeepfwfm_deprecated_amd.metrics import DeviceMetrics
    rng = np.random.default_rng(n)
    z = rng.normal(size=n).astype(np.float32) * 2
    if levels:
        z = np.round(z * levels / 4) / (levels / 4)  # many exact ties
    y = (rng.random(n) < 1 / (1 + np.exp(-(z + rng.normal(size=n))))) * 1.0
    y = np.where(rng.random(n) < rate, y, 0.0).astype(np.float32)
    m = DeviceMetrics(gpu)(torch.from_numpy(z).to(gpu), torch.from_numpy(y).to(gpu))
    # the device's f32 sigmoid may differ from torch-CPU's by an ulp per element, which can merge or split
    # near-equal predictions: the AUCs agree to ~1e-7 here (exactly on separated logits, next test), the
    # log-loss to ~1e-9 relative
    pred = torch.sigmoid(torch.from_numpy(z)).numpy().astype("float64")
    assert abs(m["auc"] - roc_auc_score(y, pred)) < 1e-6
    prec, rec, _ = precision_recall_curve(y, pred)
    assert abs(m["prauc"] - auc(rec, prec)) < 1e-6
    ll = log_loss(y, pred)
    assert abs(m["log_loss"] - ll) < 1e-7 * max(1.0, ll)
    c = float(np.mean(y == 1))
    rce = (1.0 - ll / log_loss(y, [c] * n)) * 100.0
    assert abs(m["rce"] - rce) < 1e-5
    assert m["n"] == n and m["positives"] == float((y == 1).sum())


def test_device_metrics_deterministic_and_degenerate(gpu):
    """The hand-written ranking (radix passes, scans) gives the same bits on every call (no float atomics), and the
    degenerate cases match sklearn: one sample, every prediction tied, tiles ending inside a tie group."""
    from sklearn.metrics import auc, precision_recall_curve, roc_auc_score
    from xsdeepfwfm_deprecated_amd.metrics import DeviceMetrics
    dm = DeviceMetrics(gpu)
    rng = np.random.default_rng(9)
    n = 3 * 4096 + 77
    z = np.round(rng.normal(size=n) * 3).astype(np.float32)  # 20-odd distinct values: groups span many tiles
    y = (rng.random(n) < 1 / (1 + np.exp(-z))).astype(np.float32)
    zt, yt = torch.from_numpy(z).to(gpu), torch.from_numpy(y).to(gpu)
    a, b = dm(zt, yt), dm(zt, yt)
    assert a == b
    pred = torch.sigmoid(torch.from_numpy(z)).numpy().astype("float64")
    assert a["distinct_predictions"] == len(np.unique(pred))
    assert abs(a["auc"] - roc_auc_score(y, pred)) < 1e-12
    prec, rec, _ = precision_recall_curve(y, pred)
    assert abs(a["prauc"] - auc(rec, prec)) < 1e-12
    # every prediction tied: one group, AUC 0.5
    zc = torch.full((5000,), 0.25, device=gpu)
    yc = torch.from_numpy((np.arange(5000) % 7 == 0).astype(np.float32)).to(gpu)
    c = dm(zc, yc)
    assert c["distinct_predictions"] == 1 and abs(c["auc"] - 0.5) < 1e-15
    prec, rec, _ = precision_recall_curve(yc.cpu().numpy(), np.full(5000, 0.5))
    assert abs(c["prauc"] - auc(rec, prec)) < 1e-12
    one = dm(torch.tensor([0.3], device=gpu), torch.tensor([1.0], device=gpu))
    assert one["n"] == 1 and one["positives"] == 1 and one["distinct_predictions"] == 1


def test_eval_by_batch_matches_reference_auc(gpu):
    """eval_by_batch (device logits + device metrics) reproduces the reference's AUC on tiny-criteo."""
    cfg, params, xi, xv, y, l32, l64, auc_ref = load_golden("tiny_deepfwfm_lw")
    m = make_model(cfg, params, gpu)
    loss, auc_got, prauc, rce = m.eval_by_batch(xi, xv, y, len(y))
    assert abs(auc_got - auc_ref) <= 1e-4
    from sklearn.metrics import log_loss
    assert abs(loss - log_loss(y, dfwfm_oracle.sigmoid(l64))) < 1e-4


def test_device_metrics_exact_on_separated_logits(gpu):
    """With logits far enough apart that every platform's f32 sigmoid orders them the same, and exact
    repeats for ties, the device AUC / PR-AUC equal sklearn's to rounding."""
    from sklearn.metrics import auc, precision_recall_curve, roc_auc_score
    from xsdeepfwfm_deprecated_amd.metrics import DeviceMetrics
    rng = np.random.default_rng(3)
    levels = np.linspace(-4, 4, 401).astype(np.float32)
    z = levels[rng.integers(0, len(levels), size=20000)]
    y = (rng.random(20000) < 1 / (1 + np.exp(-z))).astype(np.float32)
    m = DeviceMetrics(gpu)(torch.from_numpy(z).to(gpu), torch.from_numpy(y).to(gpu))
    pred = torch.sigmoid(torch.from_numpy(z)).numpy().astype("float64")
    assert m["distinct_predictions"] == len(np.unique(pred))
    assert abs(m["auc"] - roc_auc_score(y, pred)) < 1e-12
    prec, rec, _ = precision_recall_curve(y, pred)
    assert abs(m["prauc"] - auc(rec, prec)) < 1e-12


def _sweep_case(F, num, D, N, H, fwlw, seed):
    """A synthetic DeepFwFM config (small tables) and its params / inputs, for shape sweeps."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = [1] * num + [int(x) for x in 50 + (np.arange(F - num) * 37) % 400]
    cfg = dict(field_size=F, feature_sizes=sizes, embedding_size=D, use_fwfm=1, use_fm=0, use_logit=0,
               use_deep=1, use_lw=1, use_fwlw=int(fwlw), h_depth=H, deep_nodes=N, numerical=num,
               embedding_bag=0, qr_flag=0, qr_operation="mult", qr_collisions=4, qr_threshold=200)
    m = DeepFMs(**model_kwargs(cfg))
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    params = synth.synth_state(shapes, F, D, N, True, True, seed=seed)
    xi, xv = synth.synth_inputs(sizes, num, 48, seed=seed)
    return cfg, params, xi, xv


# deep_nodes covers the eight-wave kernel with the split 25th tile (400: 3 + tail; 144: 1 + tail),
# without it (256: 2 per wave; 512: 4; 96: 6 tiles; 340: 22 ragged), and the four-wave fallback (D = 32:
# 78 layer-1 chunks)
@pytest.mark.parametrize("ng", ["8", "4"])
@pytest.mark.parametrize("D,N,H,fwlw", [(10, 400, 3, 0), (10, 144, 2, 1), (4, 256, 1, 0), (16, 512, 2, 0),
                                        (8, 96, 3, 1), (32, 400, 1, 0), (10, 340, 2, 0)])
def test_forward_shape_sweep_matches_oracle(gpu, monkeypatch, ng, D, N, H, fwlw):
    monkeypatch.setenv("DFWFM_DIAG", f"ng={ng}")
    cfg, params, xi, xv = _sweep_case(39, 13, D, N, H, fwlw, seed=D * 1000 + N + H)
    m = make_model(cfg, params, gpu)
    got = run(m, xi, xv, gpu)
    ref = dfwfm_oracle.forward(cfg, params, xi, xv)
    assert logit_close(got, ref) < 1e-5


@pytest.mark.parametrize("inputs", ["uniform", "zipf"])
def test_full_size_criteo_batch_matches_oracle(gpu, inputs):
    """The bench workload at full size (Criteo-39 tables, 1.33 M rows; B = 4096): a sample of rows vs the
    float64 oracle, and every sampled row bit-identical when run alone (no dependence on batch-mates)."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = synth.CRITEO_FEATURE_SIZES
    cfg = dict(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_fm=0, use_logit=0,
               use_deep=1, use_lw=1, use_fwlw=0, h_depth=3, deep_nodes=400, numerical=13, embedding_bag=0,
               qr_flag=0, qr_operation="mult", qr_collisions=4, qr_threshold=200)
    m = DeepFMs(**model_kwargs(cfg))
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    params = synth.synth_state(shapes, 39, 10, 400, True, True, seed=1234)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    m = m.to(gpu).eval()
    gen = synth.zipf_inputs if inputs == "zipf" else synth.synth_inputs
    xi, xv = gen(sizes, 13, 4096, seed=11)
    full = run(m, xi, xv, gpu)
    rows = np.random.default_rng(0).choice(4096, 96, replace=False)
    ref = dfwfm_oracle.forward(cfg, params, xi[rows], xv[rows])
    assert logit_close(full[rows], ref) < 1e-5
    alone = run(m, xi[rows], xv[rows], gpu)
    assert np.array_equal(alone, full[rows])


@pytest.mark.parametrize("op", ["mult", "add"])
@pytest.mark.parametrize("inputs", ["uniform", "zipf"])
def test_full_size_qr_batch_matches_oracle(gpu, inputs, op):
    """BASELINE configs[2] at full size: Criteo-39 tables as QR embedding bags (c = 4, threshold 200:
    18 of the 26 categorical fields, e.g. 245,197 rows -> 61,300 quotient rows), B = 4096; every logit against
    the float64 oracle at the north-star bar (reference model/DeepFMs.py:1071-1073, model/QREmbeddingBag.py:
    156-174), and rows run alone bit-identical."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = synth.CRITEO_FEATURE_SIZES
    cfg = dict(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_fm=0, use_logit=0,
               use_deep=1, use_lw=1, use_fwlw=0, h_depth=3, deep_nodes=400, numerical=13, embedding_bag=1,
               qr_flag=1, qr_operation=op, qr_collisions=4, qr_threshold=200)
    m = DeepFMs(**model_kwargs(cfg))
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert sum(k.endswith("weight_q") for k in shapes) == 2 * 18  # first- and second-order QR bags
    assert shapes["fm_2nd_embeddings.15.weight_q"] == (61300, 10)
    params = synth.synth_state(shapes, 39, 10, 400, True, True, seed=4321)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    m = m.to(gpu).eval()
    gen = synth.zipf_inputs if inputs == "zipf" else synth.synth_inputs
    xi, xv = gen(sizes, 13, 4096, seed=12)
    xi[0] = np.asarray(sizes[13:]) - 1  # the last row of every table
    xi[1] = 0
    full = run(m, xi, xv, gpu)
    ref = dfwfm_oracle.forward(cfg, params, xi, xv)
    assert logit_close(full, ref) < 1e-5
    rows = np.random.default_rng(1).choice(4096, 64, replace=False)
    alone = run(m, xi[rows], xv[rows], gpu)
    assert np.array_equal(alone, full[rows])


def test_custom_op_opcheck_and_matches_engine(gpu):
    """torch.ops.dfwfm.forward passes torch.library.opcheck (schema, fake tensor, autograd
    registration) and returns the engine's logits bit for bit."""
    from xsdeepfwfm_deprecated_amd import torch_ops
    cfg, params, xi, xv, *_ = load_golden("deepfwfm_lw")
    m = make_model(cfg, params, gpu)
    xi_t = torch.from_numpy(xi[:64]).to(gpu)
    xv_t = torch.from_numpy(xv[:64]).to(gpu)
    with torch.no_grad():
        ref = m(xi_t, xv_t)  # syncs the engine
    plist = [p for p in m.parameters() if p.requires_grad]
    mid = torch_ops.register(m)
    torch.library.opcheck(torch.ops.dfwfm.forward.default, (mid, xi_t, xv_t, plist, False, 0.0, 0),
                          test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))
    with torch.no_grad():
        out, tok = torch.ops.dfwfm.forward(mid, xi_t, xv_t, plist, False, 0.0, 0)
    assert torch.equal(out.cpu(), ref.cpu())


@pytest.mark.parametrize("F,num,D,N,H", [(64, 16, 10, 256, 5), (20, 0, 8, 128, 2), (39, 39, 4, 64, 1)])
def test_forward_extreme_shapes_match_oracle(gpu, F, num, D, N, H):
    """The limits of the layout: 64 fields (four FwFM row tiles), no numerical field, only numerical
    fields (no Xi at all), five hidden layers."""
    cfg, params, xi, xv = _sweep_case(F, num, D, N, H, 0, seed=F + num + D + N + H)
    m = make_model(cfg, params, gpu)
    got = run(m, xi, xv, gpu)
    ref = dfwfm_oracle.forward(cfg, params, xi, xv)
    assert logit_close(got, ref) < 1e-5


@pytest.mark.parametrize("qr", [0, 1])
@pytest.mark.parametrize("B", [1, 31, 33, 4096 + 17])
def test_fwd32_bit_identical_to_fwd_kernel(gpu, monkeypatch, qr, B):
    """The 32-sample-workgroup forward (fwd32_kernel, DFWFM_DIAG=r32=1: both 16-row tiles per wave in the MLP) gives the
    same bits as fwd_kernel's static 3x400 form at Criteo-39 sizes (ragged tails, QR fields) and the oracle's
    logits at the north-star bar."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = synth.CRITEO_FEATURE_SIZES
    cfg = dict(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_fm=0, use_logit=0,
               use_deep=1, use_lw=1, use_fwlw=0, h_depth=3, deep_nodes=400, numerical=13, embedding_bag=qr,
               qr_flag=qr, qr_operation="mult", qr_collisions=4, qr_threshold=200)
    m = DeepFMs(**model_kwargs(cfg))
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    params = synth.synth_state(shapes, 39, 10, 400, True, True, seed=55 + qr)
    xi, xv = synth.synth_inputs(sizes, 13, B, seed=B)
    outs = {}
    for r32 in ("0", "1"):
        monkeypatch.setenv("DFWFM_DIAG", f"r32={r32}")
        mm = make_model(cfg, params, gpu)
        outs[r32] = run(mm, xi, xv, gpu)
    assert np.array_equal(outs["0"], outs["1"])
    rows = np.arange(B) if B < 200 else np.random.default_rng(3).choice(B, 128, replace=False)
    assert logit_close(outs["1"][rows], dfwfm_oracle.forward(cfg, params, xi[rows], xv[rows])) < 1e-5


@pytest.mark.parametrize("name", ["deepfwfm_lw", "deepfwfm_fwlw_lw", "deepfwfm_qr_mult", "deepfwfm_qr_add_fwlw",
                                  "deepfwfm_embbag", "deepfwfm_pruned", "fm_deep"])
def test_fwd32_matches_reference_goldens(gpu, monkeypatch, name):
    monkeypatch.setenv("DFWFM_DIAG", "r32=1")
    cfg, params, xi, xv, y, l32, l64, auc = load_golden(name)
    m = make_model(cfg, params, gpu)
    got = run(m, xi, xv, gpu)
    assert logit_close(got, l32) < 1e-5 and logit_close(got, l64) < 1e-5


@pytest.mark.parametrize("name", ["deepfwfm_lw", "deepfwfm_qr_mult", "deepfwfm_fwlw_lw"])
def test_forward_gather_matches_oracle_and_fused(gpu, name):
    """dfwfm_forward_gather (the gather / shallow half alone, bench.py's roofline_gather): deep_emb equals the
    oracle's embeddings (exact products of the tables' fp32 values), first + second within the north-star bar,
    and deep_emb zero padded past F * D; a model without a deep tower is refused."""
    from xsdeepfwfm_deprecated_amd._lib import DfwfmError
    cfg, params, xi, xv, *_ = load_golden(name)
    m = make_model(cfg, params, gpu)
    B = min(len(xi), 300)
    eng = m._sync_engine(gpu)
    with torch.no_grad():
        E, fs = eng.forward_gather(torch.from_numpy(xi[:B]).to(gpu), torch.from_numpy(xv[:B]).to(gpu))
    E, fs = E.cpu().numpy(), fs.cpu().numpy()
    _, parts = dfwfm_oracle.forward(cfg, params, xi[:B], xv[:B], return_parts=True)
    F_, D_ = cfg["field_size"], cfg["embedding_size"]
    ref_e = parts["E"].reshape(B, F_ * D_)
    assert np.abs(E[:, :F_ * D_] - ref_e).max() <= 1e-6 * max(1.0, np.abs(ref_e).max())
    assert not E[:, F_ * D_:].any()
    assert logit_close(fs, parts["first"] + parts["second"]) < 1e-5
    fwfm_cfg = dict(cfg, use_deep=0)
    mf = make_model(fwfm_cfg, {k: v for k, v in params.items() if not k.startswith("net_1")}, gpu)
    with pytest.raises(DfwfmError, match="deep tower"):
        mf._sync_engine(gpu).forward_gather(torch.from_numpy(xi[:B]).to(gpu), torch.from_numpy(xv[:B]).to(gpu))
