"""GPU: one HIP training step (fused forward in train mode -> HIP backward -> HIP Adam), through the C ABI,
against the reference's one-step goldens and the training oracle (with the kernels' dropout masks)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import load_train_golden, logit_close, logit_close_scaled, model_kwargs, train_golden_names
from oracle import torch_port
from test_train_oracle import compare_step

pytestmark = pytest.mark.gpu

# fp32 with atomically accumulated (order-free) sums: gradients to 2e-5 of each tensor's largest entry;
# Adam's first step is ~ -lr * sign(g), so the update is checked in lr units where |g + l2*p| is not tiny
G_TOL, DP_TOL = 2e-5, 2e-3


def build(cfg, params, device, **kw):
    from xsdeepfwfm_deprecated_amd import DeepFMs
    m = DeepFMs(**model_kwargs(cfg), **kw)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    return m.to(device).train()


def hip_step(m, xi, xv, y, device, lr, l2):
    from xsdeepfwfm_deprecated_amd.training import Adam
    opt = Adam(m.parameters(), lr=lr, weight_decay=l2)
    opt.zero_grad()
    out = m(torch.from_numpy(xi).to(device), torch.from_numpy(xv).to(device))
    loss = F.binary_cross_entropy_with_logits(out, torch.from_numpy(y).to(device))
    loss.backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu().numpy() for k, p in m.named_parameters()}
    opt.step()
    torch.cuda.synchronize()
    newp = {k: p.detach().cpu().numpy() for k, p in m.named_parameters()}
    return out.detach().cpu().numpy(), float(loss.item()), grads, newp


def check_dp(cfg, params, grads, newp, ref_grads, ref_newp, lr, l2):
    """Update error in lr units over entries whose effective Adam gradient is not within noise of 0."""
    worst = 0.0
    for k in ref_grads:
        geff = (ref_grads[k] + l2 * params[k]).reshape(-1)
        big = np.abs(geff) > 1e-6
        d = (newp[k] - params[k]).reshape(-1)[big]
        dr = (ref_newp[k] - params[k]).reshape(-1)[big]
        if d.size:
            worst = max(worst, float(np.abs(d - dr).max() / lr))
    return worst


@pytest.mark.parametrize("name", train_golden_names())
def test_train_step_matches_reference(gpu, name):
    cfg, params, xi, xv, y, loss_ref, logits_ref, ref = load_train_golden(name)
    m = build(cfg, params, gpu, is_deep_dropout=False)
    out, loss, grads, newp = hip_step(m, xi, xv, y, gpu, cfg["lr"], cfg["l2"])
    # strict north-star bar with lw (the first-order terms do not cancel); without it (train_fwfm_nolw) the
    # bar scaled by the row's absolute term sum (conftest.logit_close_scaled)
    if cfg["use_lw"]:
        assert logit_close(out, logits_ref) < 1e-5
    else:
        assert logit_close_scaled(out, logits_ref, cfg, params, xi, xv) < 1e-5
    assert abs(loss - loss_ref) <= 1e-5 * max(1.0, abs(loss_ref))
    worst_g = 0.0
    for k, (idx, gr, dp, gn) in ref.items():
        g = grads[k].reshape(-1).astype(np.float64)
        assert abs(np.linalg.norm(g) - gn) <= 1e-4 * gn + 1e-12, k
        gs = g[idx] if idx is not None else g
        worst_g = max(worst_g, float(np.abs(gs - gr).max() / (np.abs(gr).max() + 1e-30)))
    assert worst_g <= G_TOL, worst_g
    # the full update against the oracle's (the goldens store a sample of large tensors)
    _, _, og, onew = torch_port.train_step(cfg, params, xi, xv, y, cfg["lr"], cfg["l2"])
    assert check_dp(cfg, params, grads, newp, og, onew, cfg["lr"], cfg["l2"]) <= DP_TOL


@pytest.mark.parametrize("B", [1, 15, 17, 100])
def test_train_step_ragged_batches(gpu, B):
    cfg, params, xi, xv, y, *_ = load_train_golden("train_deepfwfm_fwlw")
    m = build(cfg, params, gpu, is_deep_dropout=False)
    out, loss, grads, newp = hip_step(m, xi[:B], xv[:B], y[:B], gpu, 1e-3, 3e-7)
    o_out, o_loss, og, onew = torch_port.train_step(cfg, params, xi[:B], xv[:B], y[:B], 1e-3, 3e-7)
    assert logit_close(out, o_out) < 1e-5
    for k in og:
        sc = np.abs(og[k]).max()
        assert np.abs(grads[k] - og[k]).max() <= G_TOL * sc + 1e-12, k


@pytest.mark.parametrize("name", ["train_small_mlp", "train_deepfwfm_lw"])
def test_train_step_with_dropout_matches_oracle_masks(gpu, name):
    """Deep-tower dropout (p = 0.5): the oracle rebuilds the kernels' counter-hash masks."""
    cfg, params, xi, xv, y, *_ = load_train_golden(name)
    m = build(cfg, params, gpu, is_deep_dropout=True)
    torch.manual_seed(99)
    seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())  # what train_forward draws next
    torch.manual_seed(99)
    out, loss, grads, newp = hip_step(m, xi, xv, y, gpu, 1e-3, 0.0)
    widths = [cfg["field_size"] * cfg["embedding_size"]] + [cfg["deep_nodes"]] * cfg["h_depth"]
    masks = torch_port.dropout_masks(seed, 0.5, len(xi), widths)
    o_out, o_loss, og, onew = torch_port.train_step(cfg, params, xi, xv, y, 1e-3, 0.0, masks, 0.5)
    assert logit_close(out, o_out) < 1e-5
    for k in og:
        sc = np.abs(og[k]).max()
        assert np.abs(grads[k] - og[k]).max() <= G_TOL * sc + 1e-12, k
    assert check_dp(cfg, params, grads, newp, og, onew, 1e-3, 0.0) <= DP_TOL


def test_adam_matches_torch_over_steps(gpu):
    """Five HIP Adam steps on fixed gradients equal torch.optim.Adam's single-tensor (CPU) updates."""
    from xsdeepfwfm_deprecated_amd.training import Adam
    g = torch.Generator().manual_seed(3)
    shapes = [(1000,), (37, 11), (5000, 10), (1,)]
    ps = [torch.randn(s, generator=g) for s in shapes]
    gs = [[torch.randn(s, generator=g) * 10 ** float(torch.randint(-8, 1, (1,), generator=g)) for s in shapes]
          for _ in range(5)]
    cpu = [p.clone().requires_grad_(True) for p in ps]
    dev = [torch.nn.Parameter(p.clone().to(gpu)) for p in ps]
    o_cpu = torch.optim.Adam(cpu, lr=1e-3, weight_decay=3e-7, foreach=False)
    o_dev = Adam(dev, lr=1e-3, weight_decay=3e-7)
    for step in range(5):
        for p, q, gg in zip(cpu, dev, gs[step]):
            p.grad = gg.clone()
            q.grad = gg.clone().to(gpu)
        o_cpu.step()
        o_dev.step()
    for p, q in zip(cpu, dev):
        # within 2 ulp of the parameter, or 2e-6 lr (sqrt / division rounding of the two implementations)
        np.testing.assert_allclose(q.detach().cpu().numpy(), p.detach().numpy(), rtol=2.4e-7, atol=2e-9)
    sd = o_dev.state_dict()
    assert sd["state"][0]["step"].item() == 5.0 and set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}


def test_backward_of_stale_forward_raises(gpu):
    cfg, params, xi, xv, y, *_ = load_train_golden("train_small_mlp")
    m = build(cfg, params, gpu, is_deep_dropout=False)
    a = m(torch.from_numpy(xi[:32]).to(gpu), torch.from_numpy(xv[:32]).to(gpu))
    m(torch.from_numpy(xi[32:64]).to(gpu), torch.from_numpy(xv[32:64]).to(gpu))
    with pytest.raises(RuntimeError, match="stale"):
        a.sum().backward()


def test_fit_learns(gpu):
    """fit(): the reference's loop (init, Adam, shuffle, per-epoch eval) on the HIP kernels; training AUC
    rises on a learnable synthetic target."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = [1] * 13 + [50, 300, 7, 1000, 20, 5, 64, 9, 100, 3, 11, 17, 250, 4, 6, 30, 8, 2, 40, 12, 90, 5, 15,
                        300, 7, 60]
    xi, xv = synth.synth_inputs(sizes, 13, 8192, seed=5)
    logit = ((xi[:, 0] % 7) - 3) * 0.6 + (xv[:, 0] > 30) * 1.0 - 0.5
    y = (np.random.default_rng(1).random(8192) < 1 / (1 + np.exp(-logit))).astype(np.float32)
    m = DeepFMs(field_size=39, feature_sizes=sizes, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1, n_epochs=3,
                batch_size=256, learning_rate=1e-2, weight_decay=3e-7, h_depth=2, deep_nodes=64).to(gpu)
    train_res, _ = m.fit(xi.reshape(-1, 26, 1), xv, y, [], [], [])
    assert len(train_res) == 3 and train_res[-1] > 0.6 and train_res[-1] > train_res[0]


def _batches(cfg, xi, xv, y, B, k):
    return [(xi[i * B:(i + 1) * B], xv[i * B:(i + 1) * B], y[i * B:(i + 1) * B]) for i in range(k)]


def _param_err(m, onew, lr):
    worst = 0.0
    for k, p in m.named_parameters():
        worst = max(worst, float(np.abs(p.detach().cpu().numpy() - onew[k]).max() / lr))
    return worst


@pytest.mark.parametrize("name", ["train_deepfwfm_lw", "train_qr_mult"])
def test_fused_graph_steps_match_oracle(gpu, name):
    """FusedTrainStep: step 1 eager, steps 2-4 replayed from the captured HIP graph; parameters after
    4 steps equal 4 reference steps (torch.optim.Adam carried across steps) within a fraction of lr."""
    from xsdeepfwfm_deprecated_amd.training import FusedTrainStep
    cfg, params, xi, xv, y, *_ = load_train_golden(name)
    B, K = 64, 4
    m = build(cfg, params, gpu, is_deep_dropout=False)
    t = FusedTrainStep(m, B, lr=1e-3, weight_decay=3e-7)
    logits = []
    for xb, vb, yb in _batches(cfg, xi, xv, y, B, K):
        t.step(torch.from_numpy(xb).to(gpu), torch.from_numpy(vb).to(gpu), torch.from_numpy(yb).to(gpu))
        logits.append(t.out[:B].detach().cpu().numpy().copy())
    torch.cuda.synchronize()
    assert t.graphs is not None  # steps 2.. replayed
    outs, onew = torch_port.train_steps(cfg, params, _batches(cfg, xi, xv, y, B, K), 1e-3, 3e-7)
    for k in range(K):
        assert logit_close(logits[k], outs[k]) < 1e-4, k
    # Adam's early steps move by ~lr * sign(g): near-zero gradients may flip, so the bar is 1% of lr
    # over all entries and a tight one on the median
    errs = [np.abs(p.detach().cpu().numpy() - onew[k]).reshape(-1) / 1e-3 for k, p in m.named_parameters()]
    e = np.concatenate(errs)
    assert np.median(e) < 1e-3 and np.quantile(e, 0.999) < 0.05, (np.median(e), np.quantile(e, 0.999))
    # the loss sum the kernels accumulated equals the oracle's
    ref_loss = sum(float(torch.nn.functional.binary_cross_entropy_with_logits(
        torch.from_numpy(o), torch.from_numpy(yb), reduction="sum")) for o, (_, _, yb) in
        zip(outs, _batches(cfg, xi, xv, y, B, K)))
    assert abs(t.loss_sum.item() - ref_loss) <= 1e-4 * abs(ref_loss)


def test_fused_step_dropout_uses_device_step_seed(gpu):
    """Graph-replayable dropout: step k draws masks from seed ^ mix(k - 1) (device counter)."""
    from xsdeepfwfm_deprecated_amd.training import FusedTrainStep
    cfg, params, xi, xv, y, *_ = load_train_golden("train_small_mlp")
    B, K = 32, 3
    m = build(cfg, params, gpu, is_deep_dropout=True)
    t = FusedTrainStep(m, B, lr=1e-3, weight_decay=0.0)
    for xb, vb, yb in _batches(cfg, xi, xv, y, B, K):
        t.step(torch.from_numpy(xb).to(gpu), torch.from_numpy(vb).to(gpu), torch.from_numpy(yb).to(gpu))
    torch.cuda.synchronize()
    widths = [cfg["field_size"] * cfg["embedding_size"]] + [cfg["deep_nodes"]] * cfg["h_depth"]
    mask_fn = lambda k, n: torch_port.dropout_masks(torch_port.step_seed(t.seed, k), 0.5, n, widths)  # noqa: E731
    outs, onew = torch_port.train_steps(cfg, params, _batches(cfg, xi, xv, y, B, K), 1e-3, 0.0, mask_fn, 0.5)
    e = np.concatenate([np.abs(p.detach().cpu().numpy() - onew[k]).reshape(-1) / 1e-3
                        for k, p in m.named_parameters()])
    assert np.median(e) < 1e-3 and np.quantile(e, 0.999) < 0.05


def test_fit_fused_matches_autograd_fit(gpu):
    """fit() with the fused graph step and with the autograd path (fused_fit=False) train the same
    model to the same AUC (same init seed, same shuffles; no dropout so the paths are comparable)."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = [1] * 13 + [50, 300, 7, 1000, 20, 5, 64, 9, 100, 3, 11, 17, 250, 4, 6, 30, 8, 2, 40, 12, 90, 5, 15,
                        300, 7, 60]
    xi, xv = synth.synth_inputs(sizes, 13, 4096, seed=5)
    logit = ((xi[:, 0] % 7) - 3) * 0.6 + (xv[:, 0] > 30) * 1.0 - 0.5
    y = (np.random.default_rng(1).random(4096) < 1 / (1 + np.exp(-logit))).astype(np.float32)
    res = []
    for fused in (True, False):
        m = DeepFMs(field_size=39, feature_sizes=sizes, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1, n_epochs=2,
                    batch_size=512, learning_rate=1e-2, weight_decay=3e-7, h_depth=2, deep_nodes=64,
                    is_deep_dropout=False, random_seed=3).to(gpu)
        m.fused_fit = fused
        tr, _ = m.fit(xi.reshape(-1, 26, 1), xv, y, [], [], [])
        res.append(tr)
    assert abs(res[0][-1] - res[1][-1]) < 2e-3, res


def _ref_prune(params, adaptive, emb_r, emb_corr):
    """The reference's pruning loop (:647-673) on CPU copies, with binary_search_threshold (:807-823)."""
    from xsdeepfwfm_deprecated_amd.training import binary_search_threshold
    out = {k: torch.from_numpy(v.copy()) for k, v in params.items()}
    stacked = torch.cat([v for k, v in out.items() if "fm_2nd_embeddings" in k], 0)
    emb_thr = binary_search_threshold(stacked, adaptive * emb_r, stacked.numel())
    thr = {"emb": emb_thr}
    for k, v in out.items():
        if "fm_2nd_embeddings" in k:
            v[v.abs() < emb_thr] = 0
        if "linear" in k and "weight" in k:
            t = binary_search_threshold(v, adaptive, v.numel())
            thr[k] = t
            v[v.abs() < t] = 0
        if k == "field_cov.weight":
            symm = 0.5 * (v + v.t())
            t = binary_search_threshold(symm, adaptive * emb_corr, v.numel())
            thr[k] = t
            v[symm.abs() < t] = 0
    return out, thr


@pytest.mark.parametrize("name,adaptive", [("train_deepfwfm_fwlw", 0.3), ("train_qr_mult", 0.55),
                                           ("train_small_mlp", 0.9)])
def test_device_pruning_matches_reference_bisection(gpu, name, adaptive):
    """prune_step on the device zeroes exactly what the reference's host bisection zeroes."""
    from xsdeepfwfm_deprecated_amd.training import prune_step
    cfg, params, *_ = load_train_golden(name)
    m = build(cfg, params, gpu)
    prune_step(m, adaptive, prune_fm=1, prune_r=1, prune_deep=1, emb_r=0.444, emb_corr=1.0)
    torch.cuda.synchronize()
    ref, _ = _ref_prune(params, adaptive, 0.444, 1.0)
    for k, p in m.named_parameters():
        assert torch.equal(p.detach().cpu(), ref[k]), k


def test_device_threshold_equals_reference_value(gpu):
    from xsdeepfwfm_deprecated_amd.training import DevicePruner, binary_search_threshold
    g = torch.Generator().manual_seed(7)
    pr = DevicePruner(gpu)
    for n, scale, target in [(1000, 0.01, 0.4), (100000, 1.0, 0.9), (37, 3.0, 0.2), (250000, 1e-3, 0.05)]:
        x = torch.randn(n, generator=g) * scale
        ref = binary_search_threshold(x, target, n)
        got = pr.threshold([(x.to(gpu), 0)], target).item()
        assert got == ref, (n, got, ref)
    # symmetric R
    W = torch.randn(39, 39, generator=g) * 0.2
    ref = binary_search_threshold(0.5 * (W + W.t()), 0.7, W.numel())
    assert pr.threshold([(W.to(gpu), 39)], 0.7).item() == ref


@pytest.mark.parametrize("extra,name", [([], "DeepFwFM"), (["-use_deep", "0", "-c", "FwFM"], "FwFM")])
def test_main_all_tiny_criteo_end_to_end(gpu, tmp_path, extra, name):
    """main_all.py (the reference entry point) on the tiny-criteo fixture rows: native ingest, fit with the
    fused HIP step (one epoch), save, reload, print_size_of_model, run_benchmark (device metrics) -- for
    DeepFwFM and for BASELINE configs[0] (FwFM only, use_deep 0)."""
    import shutil
    import subprocess
    import sys
    from conftest import GOLDEN, REPO
    data = tmp_path / "data"
    data.mkdir()
    src = os.path.join(GOLDEN, "ingest", "tiny_train_head.csv")
    shutil.copy(src, data / "tiny_train_input.csv")
    shutil.copy(src, data / "tiny_test_input.csv")
    r = subprocess.run([sys.executable, os.path.join(REPO, "main_all.py"), "-dataset", "tiny-criteo", "-n_epochs",
                        "1", "-batch_size", "256", "-data_root", str(tmp_path), "-time_on_cuda", "1"] + extra,
                       cwd=str(tmp_path),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "Training [1] loss" in r.stdout and "Acc:" in r.stdout and "Avg forward pass time" in r.stdout
    assert any(f.startswith(name + "_l2_") for f in os.listdir(tmp_path / "saved_models"))


def _dp_fit_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = _fit_small(batch_size=256)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _fit_small(batch_size):
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = [1] * 13 + [50, 300, 7, 1000, 20, 5, 64, 9, 100, 3, 11, 17, 250, 4, 6, 30, 8, 2, 40, 12, 90, 5, 15,
                        300, 7, 60]
    xi, xv = synth.synth_inputs(sizes, 13, 4096, seed=5)
    logit = ((xi[:, 0] % 7) - 3) * 0.6 + (xv[:, 0] > 30) * 1.0 - 0.5
    y = (np.random.default_rng(1).random(4096) < 1 / (1 + np.exp(-logit))).astype(np.float32)
    m = DeepFMs(field_size=39, feature_sizes=sizes, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1, n_epochs=2,
                batch_size=batch_size, learning_rate=1e-2, weight_decay=3e-7, h_depth=2, deep_nodes=64,
                is_deep_dropout=False, random_seed=3).to("cuda:0")
    tr, _ = m.fit(xi.reshape(-1, 26, 1), xv, y, [], [], [])
    torch.cuda.synchronize()
    return tr, {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}


def test_data_parallel_fit_two_ranks(gpu):
    """config 5 semantics on one GPU: two gloo ranks (both on cuda:0) run fit with batch 256 each; every
    rank ends with bit-identical weights, and training matches one process on the global batch of 512
    (same init and shuffles; float summation order differs) to ~1e-6."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_fit_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (tr0, w0), (tr1, w1) = res[0], res[1]
    assert all(np.array_equal(w0[k], w1[k]) for k in w0)  # replicas stay identical
    tr_single, w_single = _fit_small(batch_size=512)
    num = sum(float(np.abs(w0[k] - w_single[k]).sum()) for k in w0)
    den = sum(float(np.abs(w_single[k]).sum()) for k in w0)
    # measured on MI355X (profiles/r03/r03bj_dp_fit.log): final train loss 1.2e-7 apart, parameters 7.7e-8 relative
    # L1 after 2 epochs (16 steps; only the fp32 summation order of the exchange differs) -- bars ~25-100x that
    assert abs(tr0[-1] - tr_single[-1]) < 1e-5 * max(1.0, abs(tr_single[-1])), (tr0, tr_single)
    assert num / den < 2e-6, num / den


@pytest.mark.parametrize("F,D,N,H,fwlw", [(39, 4, 256, 1, 0), (39, 16, 512, 2, 0), (39, 8, 96, 3, 1),
                                          (39, 10, 144, 2, 1), (39, 16, 340, 1, 1),
                                          # the backward LDS envelope: 149.4 KiB with the field_cov Gram in the G
                                          # buffer (a separate Gram region made it 167.4 KiB and refused it)
                                          (45, 16, 400, 1, 0)])
def test_train_step_shape_sweep_matches_oracle(gpu, F, D, N, H, fwlw):
    """Gradients of one HIP step vs the training oracle over embedding sizes and MLP shapes."""
    from test_gpu_parity import _sweep_case
    cfg, params, xi, xv = _sweep_case(F, 13, D, N, H, fwlw, seed=7 * D + N + H)
    y = (np.arange(len(xi)) % 3 == 0).astype(np.float32)
    m = build(cfg, params, gpu, is_deep_dropout=False)
    out, loss, grads, newp = hip_step(m, xi, xv, y, gpu, 1e-3, 3e-7)
    o_out, o_loss, og, onew = torch_port.train_step(cfg, params, xi, xv, y, 1e-3, 3e-7)
    assert logit_close(out, o_out) < 1e-5
    assert abs(loss - o_loss) <= 1e-5 * max(1.0, abs(o_loss))
    for k in og:
        sc = np.abs(og[k]).max()
        assert np.abs(grads[k] - og[k]).max() <= G_TOL * sc + 1e-12, k


def test_train_step_unsupported_shape_raises(gpu):
    """D = 32 with a 400-wide MLP needs more than 160 KiB of backward LDS: refused loudly, never run."""
    from test_gpu_parity import _sweep_case
    from xsdeepfwfm_deprecated_amd._lib import DfwfmError
    cfg, params, xi, xv = _sweep_case(39, 13, 32, 400, 1, 0, seed=5)
    m = build(cfg, params, gpu, is_deep_dropout=False)
    y = np.zeros(len(xi), np.float32)
    with pytest.raises(DfwfmError, match="unsupported"):
        hip_step(m, xi, xv, y, gpu, 1e-3, 0.0)


def test_autograd_dropout_step_after_fused_fit_uses_host_seed(gpu):
    """After fit() (fused graph step) returns, the engine no longer reads the trainer's freed device step
    counter: an autograd training step with dropout draws the host seed's masks, which the oracle rebuilds
    (use-after-free of the step source)."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = [1] * 13 + [50, 300, 7, 1000, 20, 5, 64, 9, 100, 3, 11, 17, 250, 4, 6, 30, 8, 2, 40, 12, 90, 5, 15,
                        300, 7, 60]
    xi, xv = synth.synth_inputs(sizes, 13, 1024, seed=5)
    y = (np.arange(1024) % 3 == 0).astype(np.float32)
    m = DeepFMs(field_size=39, feature_sizes=sizes, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1, n_epochs=1,
                batch_size=256, learning_rate=1e-2, weight_decay=0.0, h_depth=2, deep_nodes=64,
                is_deep_dropout=True, random_seed=3).to(gpu)
    m.fit(xi.reshape(-1, 26, 1), xv, y, [], [], [])
    torch.cuda.synchronize()
    # churn the caching allocator so the trainer's old counter block is reused by other data
    junk = [torch.full((4096,), 7, dtype=torch.int64, device=gpu) for _ in range(8)]
    params = {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}
    cfg = dict(field_size=39, numerical=13, embedding_size=10, use_fwfm=1, use_fm=0, use_logit=0, use_deep=1,
               use_lw=1, use_fwlw=0, h_depth=2, deep_nodes=64, embedding_bag=0, qr_flag=0, qr_operation="mult",
               qr_collisions=1, qr_threshold=200, feature_sizes=sizes)
    m.train()
    xb, vb, yb = xi[:128], xv[:128], y[:128]
    torch.manual_seed(99)
    seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
    torch.manual_seed(99)
    out, loss, grads, newp = hip_step(m, xb, vb, yb, gpu, 1e-3, 0.0)
    del junk
    masks = torch_port.dropout_masks(seed, 0.5, len(xb), [390, 64, 64])
    o_out, o_loss, og, onew = torch_port.train_step(cfg, params, xb, vb, yb, 1e-3, 0.0, masks, 0.5)
    assert logit_close(out, o_out) < 1e-5
    for k in og:
        sc = np.abs(og[k]).max()
        assert np.abs(grads[k] - og[k]).max() <= G_TOL * sc + 1e-12, k


def test_fused_step_recaptures_after_workspace_growth(gpu):
    """A larger autograd train forward re-allocates the engine's activation workspace; the fused step's
    graphs (which baked the old pointers in) are re-captured and stay equal to the oracle."""
    from xsdeepfwfm_deprecated_amd.training import FusedTrainStep
    cfg, params, xi, xv, y, *_ = load_train_golden("train_small_mlp")
    B = 32
    m = build(cfg, params, gpu, is_deep_dropout=False)
    t = FusedTrainStep(m, B, lr=1e-3, weight_decay=3e-7)
    bats = _batches(cfg, xi, xv, y, B, 4)
    for k, (xb, vb, yb) in enumerate(bats):
        if k == 2:
            key0 = t._graph_key
            with torch.no_grad():  # a train forward at 2B rows from outside (no backward needed)
                m._engine.train_forward(torch.from_numpy(xi[:2 * B]).to(gpu), torch.from_numpy(xv[:2 * B]).to(gpu),
                                        torch.empty(2 * B, device=gpu), 0.0, 1)
        t.step(torch.from_numpy(xb).to(gpu), torch.from_numpy(vb).to(gpu), torch.from_numpy(yb).to(gpu))
    torch.cuda.synchronize()
    assert t._graph_key != key0  # re-captured
    outs, onew = torch_port.train_steps(cfg, params, bats, 1e-3, 3e-7)
    e = np.concatenate([np.abs(p.detach().cpu().numpy() - onew[k]).reshape(-1) / 1e-3
                        for k, p in m.named_parameters()])
    assert np.median(e) < 1e-3 and np.quantile(e, 0.999) < 0.05
    t.close()
    with pytest.raises(RuntimeError, match="after close"):
        t.step(torch.from_numpy(xi[:B]).to(gpu), torch.from_numpy(xv[:B]).to(gpu), torch.from_numpy(y[:B]).to(gpu))


def test_fit_raises_index_error_on_out_of_range_xi(gpu):
    """nn.Embedding raises IndexError in the reference's training forward; fit() reads the kernels' sticky
    flag after the first step and per epoch."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = [1] * 13 + [50] * 26
    xi, xv = synth.synth_inputs(sizes, 13, 512, seed=2)
    xi[3, 5] = 50  # one past the end of field 18's table
    y = np.zeros(512, np.float32)
    m = DeepFMs(field_size=39, feature_sizes=sizes, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1, n_epochs=1,
                batch_size=256, h_depth=1, deep_nodes=32, is_deep_dropout=False).to(gpu)
    with pytest.raises(IndexError):
        m.fit(xi.reshape(-1, 26, 1), xv, y, [], [], [])


def test_kd_under_data_parallel_is_refused(gpu):
    """loss_fn_kd softmaxes over the batch (reference :1060-1061): fit refuses KD under DP."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_kd_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
    assert res[0] == res[1] == "NotImplementedError"


def _kd_dp_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from xsdeepfwfm_deprecated_amd import DeepFMs, synth
        sizes = [1] * 13 + [20] * 26
        xi, xv = synth.synth_inputs(sizes, 13, 256, seed=2)
        kw = dict(field_size=39, feature_sizes=sizes, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1, n_epochs=1,
                  batch_size=64, h_depth=1, deep_nodes=32, is_deep_dropout=False)
        m, teacher = DeepFMs(**kw).to("cuda:0"), DeepFMs(**kw).to("cuda:0")
        try:
            m.fit(xi.reshape(-1, 26, 1), xv, np.zeros(256, np.float32), [], [], [], teacher_model=teacher)
            q.put((rank, "ok"))
        except NotImplementedError:
            q.put((rank, "NotImplementedError"))
    finally:
        dist.destroy_process_group()


# ----------------------------------------------------------------------------------------------------------
# touched-row (sparse) gradients of the categorical tables: the data-parallel exchange
def _sparse_setup(m, gpu):
    """FusedTrainStep-free driver of the C ABI: train forward + DFWFM_BWD_TABLES backward with the categorical
    fields' grads in a local buffer, then dfwfm_sparse_grads_local for both families (_local_lists_step)."""
    import ctypes
    from xsdeepfwfm_deprecated_amd import _lib
    fields, dense = m._param_layout()
    params = [p for p in m.parameters() if p.requires_grad]
    flat = torch.zeros(sum(p.numel() for p in params), device=gpu)
    views, off = {}, 0
    for p in params:
        views[id(p)] = (off, flat[off:off + p.numel()].view_as(p))
        off += p.numel()
    return fields, dense, views, flat, _lib, ctypes


def _sparse_step(m, gpu, xi, xv, y, sparse, split=False, bce_fused=False, extras=None):
    """One backward of m on (xi, xv, y) with the dense scatter (sparse=False; the touched-row lists are
    _local_lists_step's).  Returns {param name: grad}, [] and the logits; bce_fused: the loss gradient formed inside
    the per-tile backward (dfwfm_backward_phases_bce); extras (a dict) receives dlogit and the loss sum."""
    fields, dense, views, flat, _lib, ctypes = _sparse_setup(m, gpu)
    L, eng = _lib.lib(), m._sync_engine(gpu)
    st = ctypes.c_void_p(torch.cuda.current_stream(gpu).cuda_stream)
    xi_d, xv_d, y_d = (torch.from_numpy(a).to(gpu) for a in (xi.reshape(len(xi), -1), xv, y))
    out = torch.empty(len(xi), device=gpu)
    eng.train_forward(xi_d, xv_d, out, 0.0, 0)
    dl = torch.empty(len(xi), device=gpu)
    loss = torch.zeros(1, device=gpu)
    if not bce_fused:
        _lib.check(L.dfwfm_bce_grad(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(y_d.data_ptr()), len(xi),
                                    float(len(xi)), ctypes.c_void_p(dl.data_ptr()), ctypes.c_void_p(loss.data_ptr()),
                                    st), "bce")
    ptr = lambda t, f: None if (t is None or (sparse and f >= m.num)) else views[id(t)][1].data_ptr()  # noqa
    fg = (_lib.dfwfm_field_grads * len(fields))(*[_lib.dfwfm_field_grads(*[ptr(t, f) for t in tup])
                                                  for f, tup in enumerate(fields)])
    H = len(dense["lin_w"])
    gW = (ctypes.c_void_p * max(H, 1))(*[views[id(t)][1].data_ptr() for t in dense["lin_w"]])
    gB = (ctypes.c_void_p * max(H, 1))(*[views[id(t)][1].data_ptr() for t in dense["lin_b"]])
    dp = lambda k: None if dense[k] is None else views[id(dense[k])][1].data_ptr()  # noqa
    grads = _lib.dfwfm_grads(fg, dp("field_cov"), dp("fwfm_lin"), dp("fm_1st"), dp("bias"), gW if H else None,
                             gB if H else None, dp("fc_w"))
    if split:  # the per-tile backward, then the weight GEMM on a side stream beside the reductions + scatter
        ph = lambda bits, s_: _lib.check(L.dfwfm_backward_phases(  # noqa: E731
            eng.handle, ctypes.c_void_p(dl.data_ptr()), ctypes.byref(grads), bits, s_), "bwd phases")
        if bce_fused:  # the loss gradient in the per-tile backward; its loss sum is formed by the later REDUCE
            _lib.check(L.dfwfm_backward_phases_bce(eng.handle, ctypes.c_void_p(out.data_ptr()),
                                                   ctypes.c_void_p(y_d.data_ptr()), float(len(xi)),
                                                   ctypes.c_void_p(dl.data_ptr()), ctypes.c_void_p(loss.data_ptr()),
                                                   ctypes.byref(grads), _lib.BWD_TILES, st), "bwd bce tiles")
        else:
            ph(_lib.BWD_TILES, st)
        side = torch.cuda.Stream(gpu)
        side.wait_stream(torch.cuda.current_stream(gpu))
        ph(_lib.BWD_MLP_WEIGHTS, ctypes.c_void_p(side.cuda_stream))
        ph(_lib.BWD_SPREAD, st)
        torch.cuda.current_stream(gpu).wait_stream(side)
    elif bce_fused:
        _lib.check(L.dfwfm_backward_phases_bce(eng.handle, ctypes.c_void_p(out.data_ptr()),
                                               ctypes.c_void_p(y_d.data_ptr()), float(len(xi)),
                                               ctypes.c_void_p(dl.data_ptr()), ctypes.c_void_p(loss.data_ptr()),
                                               ctypes.byref(grads), _lib.BWD_TABLES | _lib.BWD_MLP_WEIGHTS, st),
                   "bwd bce")
    else:
        _lib.check(L.dfwfm_backward(eng.handle, ctypes.c_void_p(dl.data_ptr()), ctypes.byref(grads), st), "bwd")
    if extras is not None:
        torch.cuda.synchronize()
        extras["dlogit"] = dl.cpu().numpy()
        extras["loss"] = float(loss.item())
    lists = []
    torch.cuda.synchronize()
    names = {id(p): k for k, p in m.named_parameters()}
    g = {names[i]: v.detach().cpu().numpy().copy() for i, (o, v) in views.items()}
    return g, lists, out.detach().cpu().numpy()


def test_local_lists_hot_rows(gpu):
    """A field where every sample hits one of 3 rows (thousands of (table, sample) pairs race for one stamp) and one
    with all-distinct rows: dfwfm_sparse_grads_local lists each touched row once, with the dense gradient's sum."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = [1] * 13 + [3] + [5000] * 25
    B = 3000
    xi, xv = synth.synth_inputs(sizes, 13, B, seed=4)
    xi[:, 1] = np.arange(B)  # field 14: every sample its own row
    y = (np.arange(B) % 2).astype(np.float32)
    m = DeepFMs(field_size=39, feature_sizes=sizes, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1, h_depth=1,
                deep_nodes=32, is_deep_dropout=False).to(gpu).train()
    m.init_weights()
    gd, _, _ = _sparse_step(m, gpu, xi, xv, y, sparse=False)
    gl, lists, local, _ = _local_lists_step(m, gpu, xi, xv, y)
    assert float(local.abs().max()) == 0.0
    for k in gd:
        sc = np.abs(gd[k]).max()
        assert np.abs(gl[k] - gd[k]).max() <= G_TOL * sc + 1e-12, k
    fam0 = lists[0]
    assert fam0[0] == 0 and int(fam0[4].item()) == sum(len(np.unique(xi[:, j])) for j in range(26))


def _dp_step_worker(rank, world, port, q, name, sparse, steps):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _dp_steps(name, sparse, steps, dist, rank, world)))
    finally:
        dist.destroy_process_group()


def _dp_steps(name, sparse, steps, dist, rank, world, deterministic=False):
    """`steps` FusedTrainSteps on the global batches of train golden `name` (64 rows each), this rank taking
    its contiguous share; returns first-step grads / logits and the final parameters."""
    from xsdeepfwfm_deprecated_amd.training import FusedTrainStep
    cfg, params, xi, xv, y, *_ = load_train_golden(name)
    dev = torch.device("cuda:0")
    G = 64
    bs = G // world
    m = build(cfg, params, dev, is_deep_dropout=False)
    t = FusedTrainStep(m, bs, lr=1e-3, weight_decay=3e-7, dist=dist, sparse_exchange=sparse,
                       deterministic=deterministic)
    first = None
    for k in range(steps):
        lo = k * G + rank * bs
        xb, vb, yb = (torch.from_numpy(a[lo:lo + bs]).to(dev) for a in (xi, xv, y))
        t.step(xb, vb, yb, G if dist is not None else None)
        if k == 0:
            torch.cuda.synchronize()
            first = ({n: p.grad.detach().cpu().numpy().copy() for n, p in m.named_parameters()},
                     t.out[:bs].detach().cpu().numpy().copy())
    torch.cuda.synchronize()
    t.close()
    return first, {n: p.detach().cpu().numpy().copy() for n, p in m.named_parameters()}


def _run_dp(name, sparse, steps, world=2):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_step_worker, args=(r, world, port, q, name, sparse, steps)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("name", ["train_deepfwfm_lw", "train_qr_mult"])
def test_data_parallel_step_equals_single_process_global_batch(gpu, name):
    """configs[4] semantics, tight: two gloo ranks (both on cuda:0), each with half of every
    64-row global batch, through FusedTrainStep with the touched-row exchange.  After step 1 every gradient
    equals one process's on the whole batch to 2e-5 of the tensor's largest entry and the ranks' logits equal
    its rows to 1e-5 * max(1, |ref|); the two replicas' gradients and, after 3 steps, parameters are
    bit-identical; the dense all-reduce exchange gives the same gradients to fp32 reassociation."""
    steps = 3
    res = _run_dp(name, True, steps)
    (g0, o0), p0 = res[0]
    (g1, o1), p1 = res[1]
    for k in g0:
        assert np.array_equal(g0[k], g1[k]), k
        assert np.array_equal(p0[k], p1[k]), k
    (gs, os_), ps = _dp_steps(name, True, steps, None, 0, 1)  # one process, global batch (no exchange)
    assert logit_close(np.concatenate([o0, o1]), os_) < 1e-5
    for k in gs:
        sc = np.abs(gs[k]).max()
        assert np.abs(g0[k] - gs[k]).max() <= G_TOL * sc + 1e-12, k
    e = np.concatenate([np.abs(p0[k] - ps[k]).reshape(-1) / 1e-3 for k in ps])
    # parameters after 3 steps in lr units (measured, profiles/r03/r03bk_dp_step.log: median 0, 99.9th percentile
    # 7.5e-6, max 3.1e-4 -- Adam's m / sqrt(v) magnifies the exchange's fp32 reassociation on near-zero gradients)
    assert np.median(e) < 1e-6 and np.quantile(e, 0.999) < 1e-4 and e.max() < 2e-3, \
        (np.median(e), np.quantile(e, 0.999), e.max())
    resd = _run_dp(name, False, 1)  # dense exchange (all-reduce of the whole buffer)
    (gd, od), _ = resd[0]
    for k in gs:
        sc = np.abs(gs[k]).max()
        assert np.abs(gd[k] - g0[k]).max() <= G_TOL * sc + 1e-12, k


def test_resident_inputs_graphs_equal_copied_inputs(gpu):
    """FusedTrainStep(resident_inputs=True) replays one captured graph set per resident (xi, xv, y) buffer set,
    reading the batches in place; the parameters after 6 steps over 3 resident batches are bit-identical to the
    copying path's (the same kernels on the same values, dropout included with the same seed)."""
    from xsdeepfwfm_deprecated_amd.training import FusedTrainStep
    cfg, params, xi, xv, y, *_ = load_train_golden("train_deepfwfm_lw")
    B = 64
    bat = [tuple(torch.from_numpy(a).to(gpu) for a in b) for b in _batches(cfg, xi, xv, y, B, 3)]
    res = []
    for resident in (False, True):
        m = build(cfg, params, gpu, is_deep_dropout=True)
        m.train()
        torch.manual_seed(5)
        t = FusedTrainStep(m, B, lr=1e-3, weight_decay=3e-7, resident_inputs=resident, deterministic=True)
        for k in range(6):
            t.step(*bat[k % 3])
        torch.cuda.synchronize()
        if resident:
            assert len(t._graph_sets) == 3  # one graph set per resident batch
        res.append({n: p.detach().cpu().numpy().copy() for n, p in m.named_parameters()})
        t.close()
    for n in res[0]:  # the same kernels on the same values, and a deterministic step: the same bits
        assert np.array_equal(res[0][n], res[1][n]), n


def test_step_many_equals_single_steps(gpu):
    """FusedTrainStep.step_many captures consecutive steps over a ring of resident batches as ONE graph; the
    parameters and the running loss after 1 + 2 x 3 steps are bit-identical to seven step() calls (same kernels,
    dropout seeds and Adam counts from the device counter, and a deterministic step)."""
    from xsdeepfwfm_deprecated_amd.training import FusedTrainStep
    cfg, params, xi, xv, y, *_ = load_train_golden("train_deepfwfm_lw")
    B = 64
    bat = [tuple(torch.from_numpy(a).to(gpu) for a in b) for b in _batches(cfg, xi, xv, y, B, 3)]
    res, losses = [], []
    for many in (False, True):
        m = build(cfg, params, gpu, is_deep_dropout=True)
        m.train()
        torch.manual_seed(5)
        t = FusedTrainStep(m, B, lr=1e-3, weight_decay=3e-7, resident_inputs=True, deterministic=True)
        t.step(*bat[0])
        for _ in range(2):
            if many:
                t.step_many([bat[1], bat[2], bat[0]])
            else:
                for k in (1, 2, 0):
                    t.step(*bat[k])
        torch.cuda.synchronize()
        assert t.steps == 7
        if many:
            assert any(k[0] == "many" for k in t._many_sets) and not any(k[0] == "many" for k in t._graph_sets)
        losses.append(float(t.loss_sum.item()))
        res.append({n: p.detach().cpu().numpy().copy() for n, p in m.named_parameters()})
        t.close()
    # deterministic mode: every sum of the step is formed in a fixed order (sorted scatter, split-K slices,
    # tile-ordered reductions and loss): the same bits
    for n in res[0]:
        assert np.array_equal(res[0][n], res[1][n]), n
    assert losses[0] == losses[1], losses


def _nccl_world1_worker(port, q, name, graph_comm, det=False):
    """A world-size-1 RCCL process group (backend "nccl" is RCCL on ROCm): the packed touched-row all-gather
    (all_gather_into_tensor branch of gather_packed) and FusedTrainStep's bucketed exchange run over RCCL --
    captured into the step's graph (graph_comm) or issued between its graphs."""
    import torch.distributed as dist
    os.environ["DFWFM_DP_GRAPH_COMM"] = "1" if graph_comm else "0"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from xsdeepfwfm_deprecated_amd.training import gather_packed
        assert dist.get_backend() == "nccl"
        send = torch.arange(1000, dtype=torch.int32, device=dev).view(torch.uint8)[:3992]  # odd-sized byte buffer
        recv = torch.zeros(1, send.numel(), dtype=torch.uint8, device=dev)
        gather_packed(dist, send, recv, async_op=True).wait()
        gathered_ok = bool(torch.equal(recv[0], send))
        sparse = _dp_steps(name, True, 3, dist, 0, 1, det)   # touched-row lists over all_gather_into_tensor
        dense = _dp_steps(name, False, 3, dist, 0, 1, det)   # bucketed all-reduces of the whole buffer
        q.put(("ok", gathered_ok, sparse, dense))
    except Exception as e:  # report, do not hang the parent
        q.put(("error", repr(e), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("graph_comm", [True, False])
@pytest.mark.parametrize("name", ["train_deepfwfm_lw", "train_qr_mult"])
def test_rccl_exchange_world_one_matches_single_process(gpu, name, graph_comm):
    """The RCCL branch of the data-parallel exchange runs: with a world-size-1 nccl group the packed
    all-gather returns the buffer, and three FusedTrainSteps (eager, captured, replayed) through the sparse and
    the dense exchange give the single-process gradients (2e-5 of each tensor's largest entry), logits
    (1e-5 * max(1, |ref|)) and parameters, with the collectives inside the step's graph or between its graphs."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_world1_worker, args=(port, q, name, graph_comm))
    p.start()
    status, gathered_ok, sparse, dense = q.get(timeout=300)
    p.join(60)
    assert status == "ok", gathered_ok
    assert p.exitcode == 0
    assert gathered_ok
    (gs, os_), ps = _dp_steps(name, True, 3, None, 0, 1)
    for (g, o), pr in (sparse, dense):
        assert logit_close(o, os_) < 1e-5
        for k in gs:
            sc = np.abs(gs[k]).max()
            assert np.abs(g[k] - gs[k]).max() <= G_TOL * sc + 1e-12, k
        e = np.concatenate([np.abs(pr[k] - ps[k]).reshape(-1) / 1e-3 for k in ps])
        assert np.median(e) < 1e-4 and np.quantile(e, 0.999) < 0.02


@pytest.mark.parametrize("name", ["train_deepfwfm_lw", "train_qr_mult"])
def test_rccl_world_one_deterministic_bit_identical(gpu, name):
    """with deterministic steps the world-size-1 RCCL group's three FusedTrainSteps (sparse and dense
    exchange, collectives inside the step's graph) give the single-process step's gradients, logits and parameters
    bit for bit -- the exchange adds nothing to one rank's sums and reorders none of them."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_world1_worker, args=(port, q, name, True, True))
    p.start()
    status, gathered_ok, sparse, dense = q.get(timeout=300)
    p.join(60)
    assert status == "ok", gathered_ok
    assert p.exitcode == 0
    (gs, os_), ps = _dp_steps(name, True, 3, None, 0, 1, True)
    for which, ((g, o), pr) in (("sparse", sparse), ("dense", dense)):
        assert np.array_equal(o, os_), which
        for k in gs:
            assert np.array_equal(g[k], gs[k]), (which, k)
        for k in ps:
            assert np.array_equal(pr[k], ps[k]), (which, k)


def test_sparse_exchange_capacity_is_per_table_rows(gpu):
    """The exchanged list capacity is sum over tables of min(batch, rows), with q and r
    tables of QR fields counted separately; at Criteo-39 / B = 4096 the packed per-rank buffer shrinks by
    ~46 % against tables x batch."""
    import ctypes
    from xsdeepfwfm_deprecated_amd import DeepFMs, _lib, synth
    sizes = synth.CRITEO_FEATURE_SIZES
    for qr in (0, 1):
        m = DeepFMs(field_size=39, feature_sizes=sizes, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1,
                    embedding_bag=qr, qr_flag=qr, qr_collisions=4, qr_threshold=200, h_depth=1, deep_nodes=16,
                    is_deep_dropout=False).to(gpu)
        eng = m._sync_engine(gpu)
        B = 4096
        want = 0
        for n in sizes[13:]:
            if qr and n > 200:
                want += min(B, -(-n // 4)) + min(B, 4)
            else:
                want += min(B, n)
        cap, w, ws = ctypes.c_int64(0), ctypes.c_int32(0), ctypes.c_int64(0)
        _lib.check(_lib.lib().dfwfm_sparse_grads_size(eng.handle, 0, B, ctypes.byref(cap), ctypes.byref(w),
                                                      ctypes.byref(ws)), "size")
        assert cap.value == want and w.value == 10
        if not qr:
            assert cap.value / (26 * B) < 0.56  # vs the round-2 tables x batch


def test_full_size_criteo_training_step_matches_oracle(gpu):
    """One fused training step (FusedTrainStep, what fit() runs) at full size: Criteo-39 tables
    (1.33 M rows, 13.3 M second-order table elements: row offsets well past 2^24 into the flat gradient buffer),
    3x400 MLP, B = 4096, dropout off -- logits at the north-star bar, the loss, every gradient (2e-5 of each
    tensor's largest entry, over the whole tensor) and the Adam update against the training oracle
    (oracle/torch_port.train_step: the reference's op sequence + torch.optim.Adam on the CPU)."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    from xsdeepfwfm_deprecated_amd.training import FusedTrainStep
    sizes = synth.CRITEO_FEATURE_SIZES
    cfg = dict(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_fm=0, use_logit=0,
               use_deep=1, use_lw=1, use_fwlw=0, h_depth=3, deep_nodes=400, numerical=13, embedding_bag=0,
               qr_flag=0, qr_operation="mult", qr_collisions=4, qr_threshold=200)
    m = DeepFMs(**model_kwargs(cfg), is_deep_dropout=False)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    params = synth.synth_state(shapes, 39, 10, 400, True, True, seed=77)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    m = m.to(gpu).train()
    B, lr, l2 = 4096, 1e-3, 3e-7
    xi, xv = synth.synth_inputs(sizes, 13, B, seed=31)
    y = synth.synth_labels(B, seed=31).astype(np.float32)
    t = FusedTrainStep(m, B, lr=lr, weight_decay=l2)
    loss_sum = t.step(torch.from_numpy(xi).to(gpu), torch.from_numpy(xv).to(gpu), torch.from_numpy(y).to(gpu))
    torch.cuda.synchronize()
    out = t.out.detach().cpu().numpy()
    loss = float(loss_sum.item()) / B
    grads = {k: p.grad.detach().cpu().numpy().copy() for k, p in m.named_parameters()}
    newp = {k: p.detach().cpu().numpy().copy() for k, p in m.named_parameters()}
    t.close()
    o_out, o_loss, og, onew = torch_port.train_step(cfg, params, xi, xv, y, lr, l2)
    assert logit_close(out, o_out) < 1e-5
    assert abs(loss - o_loss) <= 1e-5 * max(1.0, abs(o_loss))
    for k in og:
        sc = np.abs(og[k]).max()
        assert np.abs(grads[k] - og[k]).max() <= G_TOL * sc + 1e-12, k
    assert check_dp(cfg, params, grads, newp, og, onew, lr, l2) <= DP_TOL


def _local_lists_step(m, gpu, xi, xv, y):
    """Backward with the categorical tables scattered into a local buffer, then dfwfm_sparse_grads_local for both
    families and the lists applied to a zero buffer: returns {param: grad}, the lists, the local buffer after."""
    fields, dense, views, flat, _lib, ctypes = _sparse_setup(m, gpu)
    L, eng = _lib.lib(), m._sync_engine(gpu)
    st = ctypes.c_void_p(torch.cuda.current_stream(gpu).cuda_stream)
    xi_d, xv_d, y_d = (torch.from_numpy(a).to(gpu) for a in (xi.reshape(len(xi), -1), xv, y))
    out = torch.empty(len(xi), device=gpu)
    eng.train_forward(xi_d, xv_d, out, 0.0, 0)
    dl = torch.empty(len(xi), device=gpu)
    _lib.check(L.dfwfm_bce_grad(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(y_d.data_ptr()), len(xi),
                                float(len(xi)), ctypes.c_void_p(dl.data_ptr()), None, st), "bce")
    local = torch.zeros_like(flat)
    stamp = torch.zeros(flat.numel() + 1, dtype=torch.int32, device=gpu)
    lb, fb = local.data_ptr(), flat.data_ptr()
    ptr = lambda t, f: None if t is None else ((lb if f >= m.num else fb) + views[id(t)][0] * 4)  # noqa: E731
    fg = (_lib.dfwfm_field_grads * len(fields))(*[_lib.dfwfm_field_grads(*[ptr(t, f) for t in tup])
                                                  for f, tup in enumerate(fields)])
    H = len(dense["lin_w"])
    gW = (ctypes.c_void_p * max(H, 1))(*[views[id(t)][1].data_ptr() for t in dense["lin_w"]])
    gB = (ctypes.c_void_p * max(H, 1))(*[views[id(t)][1].data_ptr() for t in dense["lin_b"]])
    dp = lambda k: None if dense[k] is None else views[id(dense[k])][1].data_ptr()  # noqa
    grads = _lib.dfwfm_grads(fg, dp("field_cov"), dp("fwfm_lin"), dp("fm_1st"), dp("bias"), gW if H else None,
                             gB if H else None, dp("fc_w"))
    _lib.check(L.dfwfm_backward(eng.handle, ctypes.c_void_p(dl.data_ptr()), ctypes.byref(grads), st), "bwd")
    lists = []
    for fam, (iq, ir) in ((0, (0, 1)), (1, (2, 3))):
        o = lambda t: -1 if t is None else views[id(t)][0]  # noqa
        dest = (_lib.dfwfm_sparse_dest * len(fields))(
            *[_lib.dfwfm_sparse_dest(o(tup[iq]) if f >= m.num else -1, o(tup[ir]) if f >= m.num else -1)
              for f, tup in enumerate(fields)])
        cap, w, wsb = ctypes.c_int64(0), ctypes.c_int32(0), ctypes.c_int64(0)
        _lib.check(L.dfwfm_sparse_grads_size(eng.handle, fam, len(xi), ctypes.byref(cap), ctypes.byref(w),
                                             ctypes.byref(wsb)), "size")
        if cap.value == 0:
            continue
        od = torch.full((cap.value,), -7, dtype=torch.int64, device=gpu)
        orow = torch.zeros(cap.value * w.value, device=gpu)
        cnt = torch.zeros(1, dtype=torch.int32, device=gpu)
        _lib.check(L.dfwfm_sparse_grads_local(eng.handle, fam, dest, cap.value, ctypes.c_void_p(lb),
                                              ctypes.c_void_p(stamp.data_ptr()), local.numel(),
                                              ctypes.c_void_p(od.data_ptr()), ctypes.c_void_p(orow.data_ptr()),
                                              ctypes.c_void_p(cnt.data_ptr()), st), "local lists")
        _lib.check(L.dfwfm_sparse_grads_apply(ctypes.c_void_p(fb), w.value, ctypes.c_void_p(od.data_ptr()),
                                              ctypes.c_void_p(orow.data_ptr()), ctypes.c_void_p(cnt.data_ptr()),
                                              cap.value, st), "apply")
        lists.append((fam, w.value, od, orow, cnt))
    torch.cuda.synchronize()
    names = {id(p): k for k, p in m.named_parameters()}
    g = {names[i]: v.detach().cpu().numpy().copy() for i, (o, v) in views.items()}
    return g, lists, local, stamp


@pytest.mark.parametrize("name", ["train_deepfwfm_lw", "train_qr_mult", "train_deepfwfm_fwlw", "train_fwfm_nolw"])
def test_local_row_lists_equal_dense_table_grads(gpu, name):
    """dfwfm_sparse_grads_local (the data-parallel step's list builder: claim + copy of the rank's dense table
    gradients, no sort) gives the categorical tables' gradients back through apply, one entry per touched row, and
    leaves the local buffer zero (the data-parallel tests run it over several steps with one stamp array)."""
    cfg, params, xi, xv, y, *_ = load_train_golden(name)
    m = build(cfg, params, gpu, is_deep_dropout=False)
    gd, _, _ = _sparse_step(m, gpu, xi, xv, y, sparse=False)
    for rep in range(2):
        gl, lists, local, stamp = _local_lists_step(m, gpu, xi, xv, y)
        assert float(local.abs().max()) == 0.0
        for k in gd:
            sc = np.abs(gd[k]).max()
            assert np.abs(gl[k] - gd[k]).max() <= G_TOL * sc + 1e-12, (k, rep)
        ncat = cfg["field_size"] - cfg["numerical"]
        for fam, w, od, orow, cnt in lists:
            n = int(cnt.item())
            d = od[:n].cpu().numpy()
            assert n > 0 and len(np.unique(d)) == n
            assert n <= len(xi) * ncat * 2


@pytest.mark.parametrize("name", ["train_deepfwfm_lw", "train_qr_mult", "train_deepfwfm_fwlw", "train_fwfm_nolw"])
def test_backward_with_fused_bce_equals_separate(gpu, name):
    """dfwfm_backward_phases_bce (the loss gradient formed in the per-tile backward's staging) against
    dfwfm_bce_grad + dfwfm_backward: the same dlogit bits, the same gradients, the loss sum to f32 rounding."""
    cfg, params, xi, xv, y, *_ = load_train_golden(name)
    m = build(cfg, params, gpu, is_deep_dropout=False)
    e0, e1 = {}, {}
    g0, _, o0 = _sparse_step(m, gpu, xi, xv, y, sparse=False, extras=e0)
    g1, _, o1 = _sparse_step(m, gpu, xi, xv, y, sparse=False, bce_fused=True, extras=e1)
    assert np.array_equal(o0, o1)
    assert np.array_equal(e0["dlogit"], e1["dlogit"])
    assert abs(e0["loss"] - e1["loss"]) <= 1e-5 * max(1.0, abs(e0["loss"]))
    for k in g0:
        sc = np.abs(g0[k]).max()
        assert np.abs(g1[k] - g0[k]).max() <= G_TOL * sc + 1e-12, k


@pytest.mark.parametrize("name", ["train_deepfwfm_lw", "train_fwfm_nolw"])
def test_backward_bce_tiles_then_spread_forms_loss(gpu, name):
    """with the loss gradient fused into DFWFM_BWD_TILES, the tiles' losses are partials that the REDUCE
    phase of a LATER call (DFWFM_BWD_SPREAD) sums into loss_sum: the split form gives the whole call's loss and
    dlogit bits (include/dfwfm.h, dfwfm_backward_phases_bce)."""
    cfg, params, xi, xv, y, *_ = load_train_golden(name)
    m = build(cfg, params, gpu, is_deep_dropout=False)
    e0, e1 = {}, {}
    g0, _, o0 = _sparse_step(m, gpu, xi, xv, y, sparse=False, bce_fused=True, extras=e0)
    g1, _, o1 = _sparse_step(m, gpu, xi, xv, y, sparse=False, bce_fused=True, split=True, extras=e1)
    assert np.array_equal(o0, o1)
    assert np.array_equal(e0["dlogit"], e1["dlogit"])
    assert e1["loss"] != 0.0
    assert abs(e0["loss"] - e1["loss"]) <= 1e-6 * max(1.0, abs(e0["loss"]))
    for k in g0:
        sc = np.abs(g0[k]).max()
        assert np.abs(g1[k] - g0[k]).max() <= G_TOL * sc + 1e-12, k


@pytest.mark.parametrize("name", ["train_deepfwfm_lw", "train_qr_mult", "train_fwfm_nolw"])
def test_backward_tiles_spread_split_equals_whole(gpu, name):
    """DFWFM_BWD_TILES, then DFWFM_BWD_MLP_WEIGHTS on a second stream beside DFWFM_BWD_SPREAD (the one-GPU step's
    fork) gives dfwfm_backward's gradients; SPREAD without a per-tile backward for the last forward is refused."""
    import ctypes
    from xsdeepfwfm_deprecated_amd import _lib
    cfg, params, xi, xv, y, *_ = load_train_golden(name)
    m = build(cfg, params, gpu, is_deep_dropout=False)
    g0, _, o0 = _sparse_step(m, gpu, xi, xv, y, sparse=False)
    g1, _, o1 = _sparse_step(m, gpu, xi, xv, y, sparse=False, split=True)
    assert np.array_equal(o0, o1)
    for k in g0:
        sc = np.abs(g0[k]).max()
        assert np.abs(g1[k] - g0[k]).max() <= G_TOL * sc + 1e-12, k
    L, eng = _lib.lib(), m._sync_engine(gpu)
    xi_d, xv_d = (torch.from_numpy(a).to(gpu) for a in (xi.reshape(len(xi), -1), xv))
    out = torch.empty(len(xi), device=gpu)
    eng.train_forward(xi_d, xv_d, out, 0.0, 0)
    grads = _lib.dfwfm_grads(None, None, None, None, None, None, None, None)
    rc = L.dfwfm_backward_phases(eng.handle, ctypes.c_void_p(out.data_ptr()), ctypes.byref(grads), _lib.BWD_SPREAD,
                                 ctypes.c_void_p(torch.cuda.current_stream(gpu).cuda_stream))
    torch.cuda.synchronize()
    assert rc != 0  # every golden model gathers second-order embeddings (needs the per-tile backward)


# ----------------------------------------------------------------------------------------------------------
# determinism: every sum of the training step in a fixed order
def _hot_case(B, seed=4):
    """Tables from 3 rows (every sample in one of three rows) to 5000, one field with all-distinct rows."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = [1] * 13 + [3, 10 ** 6, 7, 60, 500] + [5000] * 21
    xi, xv = synth.synth_inputs(sizes, 13, B, seed=seed)
    xi[:, 1] = np.arange(B)  # field 14: every sample its own row
    y = (np.arange(B) % 3 == 0).astype(np.float32)
    m = DeepFMs(field_size=39, feature_sizes=sizes, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1, h_depth=2,
                deep_nodes=64, is_deep_dropout=False)
    return m, xi, xv, y


@pytest.mark.parametrize("B", [3000, 9000])  # 9000: three sorted passes of <= 4096 samples
def test_sorted_scatter_bit_identical_and_matches_atomic(gpu, monkeypatch, B):
    """Deterministic mode (the default: sorted table scatter, split-K slices): two backward passes give the same
    bits, and equal the atomic scatter (arrival-order sums) within fp32 reassociation, hot rows and multi-pass
    batches included."""
    m, xi, xv, y = _hot_case(B)
    m = m.to(gpu).train()
    m.init_weights()
    m._sync_engine(gpu).set_deterministic(True)
    g1, _, _ = _sparse_step(m, gpu, xi, xv, y, sparse=False, bce_fused=True)
    g2, _, _ = _sparse_step(m, gpu, xi, xv, y, sparse=False, bce_fused=True)
    for k in g1:
        assert np.array_equal(g1[k], g2[k]), k
    m._sync_engine(gpu).set_deterministic(False)
    ga, _, _ = _sparse_step(m, gpu, xi, xv, y, sparse=False, bce_fused=True)
    for k in g1:
        sc = np.abs(ga[k]).max()
        assert np.abs(g1[k] - ga[k]).max() <= 2e-6 * sc + 1e-12, k


@pytest.mark.parametrize("name", ["train_deepfwfm_lw", "train_qr_mult"])
def test_fused_step_runs_are_bit_identical(gpu, name):
    """Two default FusedTrainStep instances (deterministic unless asked otherwise) from the same weights over the
    same 4 batches (dropout on, graph-replayed steps) end with bit-identical parameters and loss: the sorted scatter,
    the split-K slices of the weight-gradient GEMM and the tile-ordered reductions leave no arrival-order sum in the
    step."""
    from xsdeepfwfm_deprecated_amd.training import FusedTrainStep
    cfg, params, xi, xv, y, *_ = load_train_golden(name)
    B = 64
    bat = [tuple(torch.from_numpy(a).to(gpu) for a in b) for b in _batches(cfg, xi, xv, y, B, 3)]
    res, losses = [], []
    for _ in range(2):
        m = build(cfg, params, gpu, is_deep_dropout=True)
        torch.manual_seed(11)
        t = FusedTrainStep(m, B, lr=1e-3, weight_decay=3e-7)
        assert t.deterministic and m.deterministic
        for k in range(4):
            t.step(*bat[k % 3])
        torch.cuda.synchronize()
        losses.append(float(t.loss_sum.item()))
        res.append({n: p.detach().cpu().numpy().copy() for n, p in m.named_parameters()})
        t.close()
    for n in res[0]:
        assert np.array_equal(res[0][n], res[1][n]), n
    assert losses[0] == losses[1], losses


def test_full_size_fused_steps_bit_identical(gpu):
    """Criteo-39 sizes at the bench's batch (4096, 3x400 MLP, dropout), deterministic mode: two runs of 3 fused steps
    from the same weights give bit-identical parameters (every table, the MLP's split-K weight gradients included)."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    from xsdeepfwfm_deprecated_amd.training import FusedTrainStep
    sizes = synth.CRITEO_FEATURE_SIZES
    B = 4096
    bats = []
    for i in range(3):
        xi, xv = synth.synth_inputs(sizes, 13, B, seed=50 + i)
        bats.append((torch.from_numpy(xi).to(gpu), torch.from_numpy(xv).to(gpu),
                     torch.from_numpy((np.arange(B) % 4 == i).astype(np.float32)).to(gpu)))
    res = []
    for _ in range(2):
        torch.manual_seed(3)
        m = DeepFMs(field_size=39, feature_sizes=sizes, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1,
                    is_deep_dropout=True).to(gpu).train()
        m.init_weights()
        torch.manual_seed(21)
        t = FusedTrainStep(m, B, lr=1e-3, weight_decay=3e-7, deterministic=True)
        for b in bats:
            t.step(*b)
        torch.cuda.synchronize()
        res.append({n: p.detach().cpu().numpy().copy() for n, p in m.named_parameters()})
        t.close()
        del m
    for n in res[0]:
        assert np.array_equal(res[0][n], res[1][n]), n


def test_autograd_backward_deterministic_switch(gpu):
    """DeepFMs.deterministic reaches the autograd backward (torch.ops.dfwfm.forward's registered backward): two
    loss.backward() calls on the same batch give bit-identical gradients, at Criteo-39 table sizes."""
    m, xi, xv, y = _hot_case(4096, seed=8)
    m = m.to(gpu).train()
    m.init_weights()
    m.deterministic = True
    got = []
    for _ in range(2):
        m.zero_grad(set_to_none=True)
        out = m(torch.from_numpy(xi).to(gpu), torch.from_numpy(xv).to(gpu))
        F.binary_cross_entropy_with_logits(out, torch.from_numpy(y).to(gpu)).backward()
        torch.cuda.synchronize()
        got.append({k: p.grad.detach().cpu().numpy().copy() for k, p in m.named_parameters()})
    for k in got[0]:
        assert np.array_equal(got[0][k], got[1][k]), k


@pytest.mark.parametrize("qr,drop,B,depth", [(False, True, 4096, 3), (False, False, 4000, 3), (True, True, 1000, 3),
                                             (False, True, 512, 1), (False, True, 700, 2)])
def test_helper_wave_train_forward_bit_identical(gpu, monkeypatch, qr, drop, B, depth):
    """The training forward with helper waves (ftrain_kernel: the shallow part and the activation saves on four waves
    beside the MLP's eight) against fwd_kernel<TRAIN> (DFWFM_DIAG=ftrain=0), Criteo-39 sizes, 3x400 MLP: two deterministic
    fused steps give the same logits and the same parameters bit for bit (every saved activation feeds the
    backward), with and without deep dropout, QR tables, a ragged last tile, one and two hidden layers."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    from xsdeepfwfm_deprecated_amd.training import FusedTrainStep
    sizes = synth.CRITEO_FEATURE_SIZES
    bats = []
    for i in range(2):
        xi, xv = synth.synth_inputs(sizes, 13, B, seed=70 + i)
        bats.append((torch.from_numpy(xi).to(gpu), torch.from_numpy(xv).to(gpu),
                     torch.from_numpy((np.arange(B) % 3 == i).astype(np.float32)).to(gpu)))
    res = []
    for ft in ("0", "1"):
        monkeypatch.setenv("DFWFM_DIAG", f"ftrain={ft}")
        torch.manual_seed(5)
        kw = dict(embedding_bag=1, qr_flag=1, qr_operation="mult", qr_collisions=4, qr_threshold=200) if qr else {}
        m = DeepFMs(field_size=39, feature_sizes=sizes, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1, h_depth=depth,
                    is_deep_dropout=drop, **kw).to(gpu).train()
        m.init_weights()
        torch.manual_seed(9)
        t = FusedTrainStep(m, B, lr=1e-3, weight_decay=3e-7, deterministic=True)
        outs = []
        for b in bats:
            t.step(*b)
            outs.append(t.out.detach().cpu().numpy().copy())
        torch.cuda.synchronize()
        res.append((outs, {n: p.detach().cpu().numpy().copy() for n, p in m.named_parameters()}))
        t.close()
        del m
    for o0, o1 in zip(res[0][0], res[1][0]):
        assert np.array_equal(o0, o1)
    for n in res[0][1]:
        assert np.array_equal(res[0][1][n], res[1][1][n]), n


@pytest.mark.parametrize("det", [False, True])
def test_train_step_smaller_ragged_batch_after_larger(gpu, det):
    """the weight-gradient GEMM's split slices are sized for the workspace's batch, but a smaller
    ragged batch can round to MORE splits (39 x 10 inputs, two 320-wide layers: 36 blocks per split, cap 7; B = 1000
    rounds to 192-row splits = 6, B = 896 to 128-row splits = 7).  A step at 1000 rows then one at 896 must both run
    and match the training oracle, with the float-atomic and the deterministic split-K sums."""
    from test_gpu_parity import _sweep_case
    from xsdeepfwfm_deprecated_amd import synth
    cfg, params, _, _ = _sweep_case(39, 13, 10, 320, 2, 0, seed=11)
    xi, xv = synth.synth_inputs(cfg["feature_sizes"], 13, 1000, seed=12)
    y = (np.arange(1000) % 3 == 0).astype(np.float32)
    m = build(cfg, params, gpu, is_deep_dropout=False)
    m.deterministic = det
    hip_step(m, xi, xv, y, gpu, 1e-3, 3e-7)  # sizes the workspace for 1000 rows
    p1 = {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}
    B = 896
    out, loss, grads, newp = hip_step(m, xi[:B], xv[:B], y[:B], gpu, 1e-3, 3e-7)
    o_out, o_loss, og, onew = torch_port.train_step(cfg, p1, xi[:B], xv[:B], y[:B], 1e-3, 3e-7)
    assert logit_close(out, o_out) < 1e-5
    for k in og:
        sc = np.abs(og[k]).max()
        assert np.abs(grads[k] - og[k]).max() <= G_TOL * sc + 1e-12, k


def test_fused_step_deterministic_change_recaptures(gpu):
    """FusedTrainStep.deterministic is read at capture; changing it between steps selects another graph
    set (the key holds it), so the new mode takes effect instead of replaying the old graphs."""
    from xsdeepfwfm_deprecated_amd.training import FusedTrainStep
    cfg, params, xi, xv, y, *_ = load_train_golden("train_small_mlp")
    B = 32
    m = build(cfg, params, gpu, is_deep_dropout=False)
    t = FusedTrainStep(m, B, lr=1e-3, weight_decay=3e-7, deterministic=False)
    bats = [tuple(torch.from_numpy(a).to(gpu) for a in b) for b in _batches(cfg, xi, xv, y, B, 2)]
    t.step(*bats[0])
    k0 = t._graph_key
    t.deterministic = True
    t.step(*bats[1])
    torch.cuda.synchronize()
    assert t._graph_key != k0 and t._graph_key[2] is True
    t.close()
