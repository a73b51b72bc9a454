"""CPU: the training-step oracle (oracle/torch_port.train_step) is pinned to the reference's own one-step
goldens (tests/golden/train_*.npz, written by gen_golden_train.py from the reference model), and the
host-side training logic (pruning threshold, DP gradient all-reduce over gloo) behaves as the reference."""
import os

import numpy as np
import pytest
import torch

from conftest import load_train_golden, train_golden_names
from oracle import torch_port


def compare_step(cfg, params, ref, grads, newp, g_tol=1e-5, dp_tol=1e-4):
    """Worst relative gradient error (per tensor, vs its max |grad|) and parameter-update error in lr units."""
    worst_g = worst_dp = 0.0
    for k, (idx, gr, dp, gn) in ref.items():
        g = np.asarray(grads[k], np.float64).reshape(-1)
        d = (np.asarray(newp[k], np.float64) - params[k]).reshape(-1)
        if idx is not None:
            g, d = g[idx], d[idx]
        worst_g = max(worst_g, float(np.abs(g - gr).max() / (np.abs(gr).max() + 1e-30)))
        worst_dp = max(worst_dp, float(np.abs(d - dp).max() / cfg["lr"]))
    return worst_g, worst_dp


@pytest.mark.parametrize("name", train_golden_names())
def test_oracle_train_step_matches_reference(name):
    cfg, params, xi, xv, y, loss, logits, ref = load_train_golden(name)
    out, l, grads, newp = torch_port.train_step(cfg, params, xi, xv, y, cfg["lr"], cfg["l2"])
    assert abs(l - loss) <= 1e-6 * max(1.0, abs(loss))
    assert np.abs(out - logits).max() <= 1e-5
    wg, wdp = compare_step(cfg, params, ref, grads, newp)
    assert wg <= 1e-5 and wdp <= 1e-3, (wg, wdp)
    for k, (_, _, _, gn) in ref.items():
        assert abs(np.linalg.norm(grads[k].astype(np.float64)) - gn) <= 1e-5 * gn + 1e-12, k


def test_dropout_masks_are_bernoulli_and_deterministic():
    a = torch_port.dropout_masks(1234, 0.5, 512, [390, 400])
    b = torch_port.dropout_masks(1234, 0.5, 512, [390, 400])
    c = torch_port.dropout_masks(1235, 0.5, 512, [390, 400])
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    assert not torch.equal(a[0], c[0])
    for m in a:
        assert abs(m.float().mean().item() - 0.5) < 0.01
    assert not torch.equal(a[0][:, :390], a[1][:, :390])  # layers decorrelated
    # row offsets select the same global rows
    d = torch_port.dropout_masks(1234, 0.5, 100, [400], row0=17)
    e = torch_port.dropout_masks(1234, 0.5, 117, [400])
    assert torch.equal(d[0], e[0][17:])


def test_dropout_changes_the_step():
    cfg, params, xi, xv, y, *_ = load_train_golden("train_small_mlp")
    widths = [cfg["field_size"] * cfg["embedding_size"]] + [cfg["deep_nodes"]] * cfg["h_depth"]
    masks = torch_port.dropout_masks(7, 0.5, len(xi), widths)
    o1, *_ = torch_port.train_step(cfg, params, xi, xv, y, 1e-3, 0.0)
    o2, *_ = torch_port.train_step(cfg, params, xi, xv, y, 1e-3, 0.0, masks, 0.5)
    assert not np.allclose(o1, o2)


def test_binary_search_threshold_hits_target():
    from xsdeepfwfm_deprecated_amd.training import binary_search_threshold
    g = torch.Generator().manual_seed(0)
    w = torch.randn(100000, generator=g) * 0.01
    thr = binary_search_threshold(w, 0.4, w.numel())
    assert abs((w.abs() < thr).float().mean().item() - 0.4) < 1e-3


def _dp_worker(rank, world, port, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        from xsdeepfwfm_deprecated_amd.training import allreduce_grads
        m = torch.nn.Module()
        m.a = torch.nn.Parameter(torch.zeros(3))
        m.b = torch.nn.Parameter(torch.zeros(2, 2))
        flat = torch.arange(7, dtype=torch.float32) * (rank + 1)
        m.a.grad = flat[:3]
        m.b.grad = flat[3:].view(2, 2)
        m._grad_flat = flat
        allreduce_grads(m)  # the single flat all-reduce
        r1 = (m.a.grad.numpy().copy(), m.b.grad.numpy().copy())  # by value: the worker may exit before the read
        m._grad_flat = None
        m.a.grad = torch.ones(3) * (rank + 1)
        m.b.grad = torch.ones(2, 2) * 10 * (rank + 1)
        allreduce_grads(m)  # the coalesced fallback
        q.put((rank, r1, (m.a.grad.numpy().copy(), m.b.grad.numpy().copy())))
    finally:
        dist.destroy_process_group()


def test_dp_grad_allreduce_gloo_world2():
    import tempfile
    import torch.multiprocessing as mp
    port = os.path.join(tempfile.mkdtemp(), "store")  # a file rendezvous: no port to race for under pytest -n
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, tuple(tuple(torch.from_numpy(x) for x in ab) for ab in (a, b)))
               for r, a, b in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    base = torch.arange(7, dtype=torch.float32) * 3
    for r in range(2):
        (a1, b1), (a2, b2) = res[r]
        assert torch.equal(a1, base[:3]) and torch.equal(b1, base[3:].view(2, 2))
        assert torch.equal(a2, torch.full((3,), 3.0)) and torch.equal(b2, torch.full((2, 2), 30.0))


def _sparse_protocol_worker(rank, world, port, q):
    """One rank of the touched-row exchange at oracle level: its local table gradients (torch_port, loss
    normalised by the global batch) -> (dest, row) lists of both table families (second-order rows of width D,
    first-order rows of width 1) at the product's fixed capacity (sum over tables of min(rows per rank, table
    rows)), packed with training.packed_layout into one byte buffer -> training.gather_packed over gloo -> every
    rank's lists added in rank order (the order FusedTrainStep._apply_sparse uses)."""
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        from xsdeepfwfm_deprecated_amd.training import gather_packed, packed_layout
        cfg, params, xi, xv, y, *_ = load_train_golden("train_deepfwfm_lw")
        n = 64
        lo = rank * (n // world)
        hi = lo + n // world
        _, _, g, _ = torch_port.train_step(cfg, params, xi[lo:hi], xv[lo:hi], y[lo:hi], 1e-3, 0.0)
        scale = np.float32((hi - lo) / n)  # the rank's mean-loss gradient -> its share of the global mean
        num, D, F = cfg["numerical"], cfg["embedding_size"], cfg["field_size"]
        fams = []
        for prefix, w in (("fm_2nd_embeddings", D), ("fm_1st_embeddings", 1)):
            names = [f"{prefix}.{f}.weight" for f in range(num, F)]
            if not all(k in params for k in names):
                continue
            offs = np.cumsum([0] + [params[k].shape[0] for k in names])
            cap = sum(min(hi - lo, params[k].shape[0]) for k in names)
            fams.append(dict(names=names, offs=offs, cap=cap, w=w))
        nbytes = packed_layout(fams)
        send = torch.zeros(nbytes, dtype=torch.uint8)
        for f in fams:
            dest = np.full(f["cap"], -1, np.int64)
            rows = np.zeros((f["cap"], f["w"]), np.float32)
            c = 0
            for j, k in enumerate(f["names"]):
                touched = np.unique(xi[lo:hi, j])
                dest[c:c + len(touched)] = (f["offs"][j] + touched) * f["w"]
                rows[c:c + len(touched)] = g[k].reshape(-1, f["w"])[touched] * scale
                c += len(touched)
            assert c <= f["cap"]
            send[f["o_dest"]:f["o_dest"] + 8 * f["cap"]] = torch.from_numpy(dest).view(torch.uint8)
            send[f["o_rows"]:f["o_rows"] + 4 * f["cap"] * f["w"]] = torch.from_numpy(rows).view(-1).view(torch.uint8)
            send[f["o_cnt"]:f["o_cnt"] + 4] = torch.tensor([c], dtype=torch.int32).view(torch.uint8)
        recv = torch.zeros(world, nbytes, dtype=torch.uint8)
        gather_packed(dist, send, recv, async_op=False)
        out = []
        for f in fams:
            flat = torch.zeros(int(f["offs"][-1]) * f["w"])
            for r in range(world):  # rank order, one list after the other
                b = recv[r]
                cnt = int(b[f["o_cnt"]:f["o_cnt"] + 4].view(torch.int32)[0])
                d = b[f["o_dest"]:f["o_dest"] + 8 * f["cap"]].view(torch.int64)[:cnt]
                v = b[f["o_rows"]:f["o_rows"] + 4 * f["cap"] * f["w"]].view(torch.float32).view(f["cap"], f["w"])[:cnt]
                for j in range(f["w"]):  # destinations unique within one list
                    flat[d + j] += v[:, j]
            out.append(flat.numpy())
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])  # 8: BASELINE configs[4] is DP = 8
def test_touched_row_exchange_protocol_gloo(world):
    """configs[4] exchange at oracle level on CPU: `world` gloo ranks' touched-row lists of both table families,
    all-gathered at fixed capacity in training.packed_layout's buffer and added in rank order, equal the dense
    table gradients of one process on the global batch, and every rank's result is bit-identical."""
    import tempfile
    import torch.multiprocessing as mp
    port = os.path.join(tempfile.mkdtemp(), "store")  # a file rendezvous: no port to race for under pytest -n
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sparse_protocol_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r in range(1, world):
        assert all(np.array_equal(a, b) for a, b in zip(res[0], res[r]))
    cfg, params, xi, xv, y, *_ = load_train_golden("train_deepfwfm_lw")
    _, _, g, _ = torch_port.train_step(cfg, params, xi[:64], xv[:64], y[:64], 1e-3, 0.0)
    assert len(res[0]) == 2
    for got, prefix in zip(res[0], ("fm_2nd_embeddings", "fm_1st_embeddings")):
        dense = np.concatenate([g[f"{prefix}.{f}.weight"].reshape(-1) for f in range(13, 39)])
        assert np.abs(got - dense).max() <= 2e-5 * np.abs(dense).max()


def _criteo_fams(B, world=1):
    """The two table families' exchange capacities at Criteo-39 (sum over the 26 categorical tables of min(rows,
    per-rank batch), as dfwfm_sparse_grads_size reports them) and their packed layout."""
    from xsdeepfwfm_deprecated_amd import synth
    from xsdeepfwfm_deprecated_amd.training import packed_layout
    cap = sum(min(B, n) for n in synth.CRITEO_FEATURE_SIZES[13:])
    fams = [dict(cap=cap, w=10), dict(cap=cap, w=1)]
    return fams, packed_layout(fams)


def test_exchange_workspace_fits_dp8_and_refuses_oversize():
    """configs[4]: eight ranks of B = 4096 at Criteo-39 fit the exchange workspace (3.45 MB of packed lists per rank,
    DESIGN.md section 6); a world whose all-gathered buffer would not fit is refused with a clear error before
    anything is captured (FusedTrainStep._setup_sparse calls the same check)."""
    from xsdeepfwfm_deprecated_amd.training import check_exchange
    fams, nbytes = _criteo_fams(4096)
    assert fams[0]["cap"] == 57531 and 3.4e6 < nbytes < 3.5e6
    assert check_exchange(8, nbytes, fams) == 8 * nbytes
    with pytest.raises(ValueError, match="exceed the exchange workspace"):
        check_exchange(8, nbytes, fams, max_bytes=8 * nbytes - 1)
    with pytest.raises(ValueError, match="exceed the exchange workspace"):
        check_exchange(1024, nbytes, fams)  # 3.5 GB of receive buffer
    with pytest.raises(ValueError, match="32-bit grid"):
        check_exchange(1, 16, [dict(cap=2 ** 28, w=10)], max_bytes=2 ** 62)
