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
    normalised by the global batch) -> (dest, row) list at fixed capacity packed into one byte buffer ->
    training.gather_packed over gloo -> every rank's lists added in rank order."""
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        from xsdeepfwfm_deprecated_amd.training import gather_packed
        cfg, params, xi, xv, y, *_ = load_train_golden("train_deepfwfm_lw")
        n = 64
        lo = rank * (n // world)
        hi = lo + n // world
        _, _, g, _ = torch_port.train_step(cfg, params, xi[lo:hi], xv[lo:hi], y[lo:hi], 1e-3, 0.0)
        scale = (hi - lo) / n  # the rank's mean-loss gradient -> its share of the global mean
        num, D = cfg["numerical"], cfg["embedding_size"]
        names = [f"fm_2nd_embeddings.{f}.weight" for f in range(num, cfg["field_size"])]
        offs = np.cumsum([0] + [params[k].shape[0] for k in names])
        cap = len(names) * (n // world)
        dest = np.full(cap, -1, np.int64)
        rows = np.zeros((cap, D), np.float32)
        c = 0
        for j, k in enumerate(names):
            touched = np.unique(xi[lo:hi, j])
            dest[c:c + len(touched)] = offs[j] + touched
            rows[c:c + len(touched)] = g[k][touched] * scale
            c += len(touched)
        send = torch.cat([torch.from_numpy(dest).view(torch.uint8), torch.from_numpy(rows).view(-1).view(torch.uint8),
                          torch.tensor([c, 0], dtype=torch.int32).view(torch.uint8)])
        recv = torch.zeros(world, send.numel(), dtype=torch.uint8)
        gather_packed(dist, send, recv, async_op=False)
        flat = torch.zeros(int(offs[-1]), D)
        for r in range(world):
            b = recv[r]
            cnt = int(b[-8:].view(torch.int32)[0])
            d = b[:8 * cap].view(torch.int64)[:cnt]
            v = b[8 * cap:8 * cap + 4 * cap * D].view(torch.float32).view(cap, D)[:cnt]
            flat[d] += v  # destinations unique within one list
        q.put((rank, flat.numpy()))
    finally:
        dist.destroy_process_group()


def test_touched_row_exchange_protocol_gloo_world2():
    """configs[4] exchange at oracle level on CPU: two gloo ranks' touched-row lists, all-gathered at fixed
    capacity and added in rank order, equal the dense table gradients of one process on the global batch,
    identically on both ranks."""
    import tempfile
    import torch.multiprocessing as mp
    port = os.path.join(tempfile.mkdtemp(), "store")  # a file rendezvous: no port to race for under pytest -n
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sparse_protocol_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert np.array_equal(res[0], res[1])
    cfg, params, xi, xv, y, *_ = load_train_golden("train_deepfwfm_lw")
    _, _, g, _ = torch_port.train_step(cfg, params, xi[:64], xv[:64], y[:64], 1e-3, 0.0)
    dense = np.concatenate([g[f"fm_2nd_embeddings.{f}.weight"] for f in range(13, 39)])
    assert np.abs(res[0] - dense).max() <= 2e-5 * np.abs(dense).max()
