"""GPU: dfwfm_forward_batches -- the forward of several resident batches in one launch (one grid over all of
them, each batch its own Xi / Xv / logits) -- against dfwfm_forward on each batch alone (bit-identical) and the
float64 oracle (north-star bar).  The reference runs these batches one forward call at a time
(model/DeepFMs.py:285-469, eval_by_batch's loop)."""
import numpy as np
import pytest
import torch

from conftest import load_golden, logit_close, logit_close_scaled, model_kwargs
from oracle import dfwfm_oracle

pytestmark = pytest.mark.gpu


def _criteo_model(gpu, deep=1, qr=0, seed=77):
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = synth.CRITEO_FEATURE_SIZES
    cfg = dict(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_fm=0, use_logit=0,
               use_deep=deep, use_lw=1, use_fwlw=0, h_depth=3, deep_nodes=400, numerical=13, embedding_bag=qr,
               qr_flag=qr, qr_operation="mult", qr_collisions=4, qr_threshold=200)
    m = DeepFMs(**model_kwargs(cfg))
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    params = synth.synth_state(shapes, 39, 10, 400, True, bool(deep), seed=seed)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    return cfg, params, m.to(gpu).eval()


def _inputs(sizes, nb, B, seed):
    from xsdeepfwfm_deprecated_amd import synth
    return [synth.synth_inputs(sizes, 13, B, seed=seed + i) for i in range(nb)]


def _check(cfg, params, m, gpu, host, scaled=False):
    """Every batch of the set bit-identical to its own forward; the first and the last batch -- every row (the
    float64 oracle takes ~0.3 s per 4096 rows) -- against the oracle at the north-star bar (scaled: the bar widened
    by the row's absolute term sum, conftest.logit_close_scaled, for first-order sums without lw that cancel)."""
    eng = m._sync_inference(gpu)  # MLP-free models: the tables' serving copy (dfwfm_model_pack_tables)
    dev = [(torch.from_numpy(xi).to(gpu), torch.from_numpy(xv).to(gpu)) for xi, xv in host]
    B = host[0][0].shape[0]
    with torch.no_grad():
        outs = [torch.full((B,), float("nan"), device=gpu) for _ in dev]
        eng.forward_batches(dev, outs)
        alone = [eng.forward(xi, xv) for xi, xv in dev]
    torch.cuda.synchronize()
    for i, ((xi, xv), o, a) in enumerate(zip(host, outs, alone)):
        got = o.cpu().numpy()
        assert np.array_equal(got, a.cpu().numpy()), f"batch {i}: set vs alone"
        if i in (0, len(host) - 1):
            ref = dfwfm_oracle.forward(cfg, params, xi, xv)
            err = logit_close_scaled(got, ref, cfg, params, xi, xv) if scaled else logit_close(got, ref)
            assert err < 1e-5, f"batch {i} vs oracle"


@pytest.mark.parametrize("qr", [0, 1])
@pytest.mark.parametrize("nb,B", [(2, 4096), (5, 4096), (3, 4096 + 17), (4, 33), (35, 256)])
def test_batch_set_deep_bit_identical(gpu, qr, nb, B):
    """DeepFwFM at Criteo-39 sizes (the 32-sample forward once the set covers the chip, else the 16-sample one):
    every batch of the set equals its own forward, ragged tails included, more batches than one launch holds
    (35 > 32: two launches)."""
    cfg, params, m = _criteo_model(gpu, 1, qr, seed=77 + qr)
    _check(cfg, params, m, gpu, _inputs(cfg["feature_sizes"], nb, B, seed=100 * nb + B))


@pytest.mark.parametrize("nb,B", [(3, 4096), (6, 1000), (35, 256), (3, 4096 + 17), (2, 5), (20, 4096)])
def test_batch_set_fwfm_only_bit_identical(gpu, nb, B):
    """The MLP-free forward (BASELINE configs[0]'s model at Criteo-39 sizes) as a batch set (ragged tails, tiny
    batches, two launches): bit-identical to each batch's own forward, every row of the first and last batch vs the
    oracle."""
    cfg, params, m = _criteo_model(gpu, 0, 0, seed=91)
    _check(cfg, params, m, gpu, _inputs(cfg["feature_sizes"], nb, B, seed=7 * nb + B))


@pytest.mark.parametrize("name", ["deepfwfm_lw", "deepfwfm_qr_mult", "tiny_fwfm_lw", "fm_deep"])
def test_batch_set_goldens(gpu, name):
    """Reference goldens split into a set of equal batches (small tables, the generic kernels)."""
    cfg, params, xi, xv, y, l32, l64, auc = load_golden(name)
    from xsdeepfwfm_deprecated_amd import DeepFMs
    m = DeepFMs(**model_kwargs(cfg))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    m = m.to(gpu).eval()
    nb = 4
    B = xi.shape[0] // nb
    eng = m._sync_engine(gpu)
    dev = [(torch.from_numpy(np.ascontiguousarray(xi[i * B:(i + 1) * B])).to(gpu),
            torch.from_numpy(np.ascontiguousarray(xv[i * B:(i + 1) * B])).to(gpu)) for i in range(nb)]
    outs = [torch.empty(B, device=gpu) for _ in range(nb)]
    with torch.no_grad():
        eng.forward_batches(dev, outs)
    got = torch.cat(outs).cpu().numpy()
    assert logit_close(got, l32[:nb * B]) < 1e-5 and logit_close(got, l64[:nb * B]) < 1e-5


def test_batch_set_strided_inputs_and_errors(gpu):
    """Row strides other than the field count (slices of wider resident arrays), an out-of-range index in one
    batch of the set (the sticky flag, rows clamped, never a fault), and the argument checks."""
    from xsdeepfwfm_deprecated_amd._lib import DfwfmError
    cfg, params, m = _criteo_model(gpu, 1, 0, seed=5)
    sizes = cfg["feature_sizes"]
    host = _inputs(sizes, 3, 512, seed=3)
    eng = m._sync_engine(gpu)
    wide = [(torch.zeros(512, 40, dtype=torch.int64, device=gpu), torch.zeros(512, 20, device=gpu))
            for _ in host]
    for (wi, wv), (xi, xv) in zip(wide, host):
        wi[:, :26] = torch.from_numpy(xi).to(gpu)
        wv[:, :13] = torch.from_numpy(xv).to(gpu)
    dev = [(wi[:, :26], wv[:, :13]) for wi, wv in wide]
    outs = [torch.empty(512, device=gpu) for _ in dev]
    with torch.no_grad():
        eng.forward_batches(dev, outs)
        alone = [eng.forward(torch.from_numpy(xi).to(gpu), torch.from_numpy(xv).to(gpu)) for xi, xv in host]
    for o, a in zip(outs, alone):
        assert torch.equal(o, a)
    assert eng.read_error_flag() == 0
    wide[1][0][7, 4] = sizes[13 + 4]  # one past the last row of field 17
    with torch.no_grad():
        eng.forward_batches(dev, outs)
    assert eng.read_error_flag() != 0
    assert eng.read_error_flag() == 0  # cleared by the read
    with pytest.raises(ValueError):
        eng.forward_batches([dev[0], (dev[1][0][:100], dev[1][1][:100])], outs[:2])
    with pytest.raises((DfwfmError, ValueError)):
        eng.forward_batches(dev, outs[:2])
    assert eng.forward_batches([], []) == []


@pytest.mark.parametrize("deep", [1, 0])
def test_eval_by_batch_batch_sets_identical(gpu, deep):
    """eval_by_batch's full 8192-row batches as batch sets give the same loss and metrics as one forward per batch
    (reference model/DeepFMs.py:750-784), and an out-of-range index in one of them still raises IndexError."""
    from xsdeepfwfm_deprecated_amd import synth
    cfg, params, m = _criteo_model(gpu, deep, 0, seed=31)
    n = 3 * 8192 + 100
    xi, xv = synth.synth_inputs(cfg["feature_sizes"], 13, n, seed=8)
    y = (np.random.default_rng(2).random(n) < 0.3).astype(np.float32)
    res = {}
    for on in (True, False):
        m.eval_batch_sets = on
        res[on] = m.eval_by_batch(xi.reshape(n, 26, 1), xv, y, n)
    # loss and AUC exactly; PR-AUC / RCE up to the device metrics' own float64 summation order
    assert res[True][:2] == res[False][:2]
    assert np.allclose(res[True][2:], res[False][2:], rtol=1e-12, atol=0)
    m.eval_batch_sets = True
    bad = xi.copy()
    bad[8192 + 5, 2] = -1
    with pytest.raises(IndexError):
        m.eval_by_batch(bad.reshape(n, 26, 1), xv, y, n)


def test_batch_set_full_size_pruned_dense(gpu):
    """BASELINE configs[3] on the path the bench runs: Criteo-39 tables, 3x400, the reference's magnitude masks
    (prune_step(0.90, emb_r 0.444, prune_r 1), reference model/DeepFMs.py:647-673) applied on the device, the dense
    32-sample forward (sparse tower off) over a set of 3 batches of 4096: every batch equals its own forward and the
    float64 oracle at 1e-5 * max(1, |ref|)."""
    from xsdeepfwfm_deprecated_amd.training import prune_step
    cfg, _, m = _criteo_model(gpu, 1, 0, seed=1234)
    m.sparse_mlp_max_density = 0.0
    prune_step(m, 0.90, 1, 1, 1, 0.444, 1.0)
    torch.cuda.synchronize()
    params = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    # the masks are the reference's: ~90 % of every hidden layer and 44.4 % * 0.9 of the second-order rows zero
    for h in (1, 2, 3):
        z = float(np.mean(params[f"net_1_linear_{h}.weight"] == 0))
        assert 0.89 < z < 0.91, (h, z)
    eng = m._sync_engine(gpu)
    assert not eng.sync_sparse(m.sparse_mlp_max_density)
    _check(cfg, params, m, gpu, _inputs(cfg["feature_sizes"], 3, 4096, seed=4242))


def test_forward_rejects_column_major_inputs(gpu):
    """A column-major batch (np.asarray of a DataFrame keeps Fortran order through torch.as_tensor / .to()) must not
    be read as row-major: the engine refuses it, and eval_by_batch / forward make their inputs row-major first."""
    from xsdeepfwfm_deprecated_amd import synth
    cfg, params, m = _criteo_model(gpu, 1, 0, seed=13)
    n = 2 * 8192 + 50
    xi, xv = synth.synth_inputs(cfg["feature_sizes"], 13, n, seed=21)
    eng = m._sync_engine(gpu)
    fi = torch.as_tensor(np.asfortranarray(xi)).to(gpu)
    fv = torch.as_tensor(np.asfortranarray(xv)).to(gpu)
    assert fi.stride(1) != 1 and fv.stride(1) != 1
    with torch.no_grad():
        with pytest.raises(ValueError):
            eng.forward(fi, fv)
        with pytest.raises(ValueError):
            eng.forward_batches([(fi[:8192], fv[:8192]), (fi[8192:16384], fv[8192:16384])],
                                [torch.empty(8192, device=gpu) for _ in range(2)])
        with pytest.raises(ValueError):
            eng.forward(torch.from_numpy(xi).to(gpu).to(torch.int32), torch.from_numpy(xv).to(gpu))
        a = m(fi, fv).cpu().numpy()
        b = m(torch.from_numpy(xi).to(gpu), torch.from_numpy(xv).to(gpu)).cpu().numpy()
    assert np.array_equal(a, b)
    y = (np.random.default_rng(3).random(n) < 0.3).astype(np.float32)
    m.eval_batch_sets = True
    rf = m.eval_by_batch(np.asfortranarray(xi), np.asfortranarray(xv), y, n)
    rc = m.eval_by_batch(xi, xv, y, n)
    assert rf[:2] == rc[:2]


def _fwfm_only_case(F, num, D, lw, fm, seed):
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = [1] * num + [int(x) for x in 7 + (np.arange(F - num) * 389 + seed) % 20000]
    cfg = dict(field_size=F, feature_sizes=sizes, embedding_size=D, use_fwfm=1 - fm, use_fm=fm, use_logit=0,
               use_deep=0, use_lw=lw, use_fwlw=0, h_depth=1, deep_nodes=16, numerical=num, embedding_bag=0,
               qr_flag=0, qr_operation="mult", qr_collisions=4, qr_threshold=200)
    m = DeepFMs(**model_kwargs(cfg))
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    params = synth.synth_state(shapes, F, D, 16, True, False, seed=seed)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    return cfg, params, m


# (F, numerical, D, lw, FM): FwFM row tiles 1 / 2 / 3 and every last-tile step count (S = 4 (MT - 1) + 1..4), no
# numerical fields, plain first-order sum, FM instead of FwFM, D 4 / 8 / 10 / 16
@pytest.mark.parametrize("F,num,D,lw,fm", [(39, 13, 10, 1, 0), (39, 13, 16, 1, 0), (48, 16, 8, 0, 0),
                                           (20, 5, 4, 1, 1), (30, 0, 10, 1, 0), (9, 1, 10, 0, 0),
                                           (33, 13, 10, 1, 0), (42, 2, 4, 1, 0), (16, 3, 16, 0, 1)])
def test_fwfm_only_set_shapes_bit_identical(gpu, F, num, D, lw, fm):
    """The MLP-free batch-set forward over model shapes: bit-identical to each batch alone, and within the
    north-star bar of the float64 oracle (scaled for first-order sums without lw)."""
    cfg, params, m = _fwfm_only_case(F, num, D, lw, fm, seed=F * 100 + D)
    m = m.to(gpu).eval()
    from xsdeepfwfm_deprecated_amd import synth
    host = [synth.synth_inputs(cfg["feature_sizes"], num, 1000 + F, seed=F + D + i) for i in range(5)]
    _check(cfg, params, m, gpu, host, scaled=not lw)


def test_fwfm_only_set_strided_inputs_and_out_of_range(gpu):
    """The MLP-free batch-set forward reads Xi / Xv through any row stride and clamps an out-of-range index to row 0
    with the sticky flag (nn.Embedding's IndexError, raised by DeepFMs.forward)."""
    cfg, params, m = _criteo_model(gpu, 0, 0, seed=13)
    sizes = cfg["feature_sizes"]
    host = _inputs(sizes, 4, 700, seed=9)
    eng = m._sync_engine(gpu)
    wide = [(torch.zeros(700, 31, dtype=torch.int64, device=gpu), torch.zeros(700, 17, device=gpu)) for _ in host]
    for (wi, wv), (xi, xv) in zip(wide, host):
        wi[:, :26] = torch.from_numpy(xi).to(gpu)
        wv[:, :13] = torch.from_numpy(xv).to(gpu)
    dev = [(wi[:, :26], wv[:, :13]) for wi, wv in wide]
    outs = [torch.empty(700, device=gpu) for _ in dev]
    with torch.no_grad():
        eng.forward_batches(dev, outs)
        alone = [eng.forward(torch.from_numpy(xi).to(gpu), torch.from_numpy(xv).to(gpu)) for xi, xv in host]
    for o, a in zip(outs, alone):
        assert torch.equal(o, a)
    assert eng.read_error_flag() == 0
    wide[2][0][123, 7] = sizes[13 + 7]  # one past the last row of field 20
    wide[3][0][699, 0] = -1
    with torch.no_grad():
        eng.forward_batches(dev, outs)
    assert eng.read_error_flag() != 0
    clamped = [t.clone() for t, _ in wide]
    clamped[2][123, 7] = 0
    clamped[3][699, 0] = 0
    with torch.no_grad():
        ref = [eng.forward(c[:, :26], wv[:, :13]) for c, (_, wv) in zip(clamped, wide)]
    for o, a in zip(outs, ref):
        assert torch.equal(o, a)


@pytest.mark.parametrize("deep", [0, 1])
def test_packed_tables_bit_identical_and_refreshed(gpu, deep):
    """The serving copy of the categorical tables (second-order row + first-order weight in one 64-B row) gives
    the same bits as the plain tables, lone batch and batch set (MLP-free kernel; deep: the 32-sample set kernel
    and the 16-sample lone one); an in-place table update re-packs it (the next forward matches the oracle on the
    new weights)."""
    cfg, params, m = _criteo_model(gpu, deep, 0, seed=17)
    host = _inputs(cfg["feature_sizes"], 3, 4096 + 3, seed=4)
    dev = [(torch.from_numpy(xi).to(gpu), torch.from_numpy(xv).to(gpu)) for xi, xv in host]
    outs = {}
    for packed in (False, True):
        m.pack_tables = packed
        eng = m._sync_inference(gpu)
        assert eng._packed_on == packed
        with torch.no_grad():
            sets = eng.forward_batches(dev, [torch.empty(4096 + 3, device=gpu) for _ in dev])
            lone = [m(xi, xv) for xi, xv in dev]
        outs[packed] = (torch.stack(sets).cpu().numpy(), torch.stack(lone).cpu().numpy())
    assert np.array_equal(outs[False][0], outs[True][0]) and np.array_equal(outs[False][1], outs[True][1])
    assert np.array_equal(outs[True][0], outs[True][1])
    # an in-place update (torch bumps the tables' version counters) -> the next forward re-packs
    with torch.no_grad():
        m.fm_2nd_embeddings[20].weight.mul_(-0.5)
        m.fm_1st_embeddings[30].weight.add_(0.25)
        got = m(*dev[0]).cpu().numpy()
    new = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    assert logit_close(got, dfwfm_oracle.forward(cfg, new, *host[0])) < 1e-5
    assert m._engine._packed_on


def test_packed_tables_after_fused_training_steps(gpu):
    """The fused training step updates the tables inside captured graphs (no version bump): it drops the serving
    copy's key, so the next inference forward re-packs and equals the plain-table forward bit for bit."""
    from xsdeepfwfm_deprecated_amd.training import FusedTrainStep
    cfg, params, m = _criteo_model(gpu, 0, 0, seed=29)
    host = _inputs(cfg["feature_sizes"], 3, 1024, seed=8)
    dev = [(torch.from_numpy(xi).to(gpu), torch.from_numpy(xv).to(gpu)) for xi, xv in host]
    with torch.no_grad():
        before = m(*dev[0]).clone()  # packs
    m.train()
    t = FusedTrainStep(m, 1024, lr=1e-2, weight_decay=0.0)
    for xi, xv in dev[1:]:
        t.step(xi, xv, (torch.arange(1024, device=gpu) % 3 == 0).float())
    t.close()
    m.eval()
    with torch.no_grad():
        packed = m(*dev[0]).cpu().numpy()
        m.pack_tables = False
        plain = m(*dev[0]).cpu().numpy()
    assert not np.array_equal(packed, before.cpu().numpy())
    assert np.array_equal(packed, plain)
