"""CPU: the host kernels (libdfwfm_cpu.so, include/dfwfm_cpu.h) -- the custom op's CPU kernel and its backward, for
modules on the CPU (BASELINE configs[0]: FwFM on tiny-criteo via main_all.py, -use_cuda 0 -time_on_cuda 0) --
against the reference's golden vectors and the training oracle."""
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import (GOLDEN, REPO, golden_names, load_golden, load_train_golden, logit_close, logit_close_scaled,
                      model_kwargs, train_golden_names)
from oracle import dfwfm_oracle, torch_port

G_TOL = 2e-5


def cpu_model(cfg, params, **kw):
    from xsdeepfwfm_deprecated_amd import DeepFMs
    m = DeepFMs(**model_kwargs(cfg), **kw)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    return m


def run(m, xi, xv):
    with torch.no_grad():
        return m.eval()(torch.from_numpy(xi), torch.from_numpy(xv)).numpy()


@pytest.mark.parametrize("name", golden_names())
def test_cpu_forward_matches_reference(name):
    """Every forward golden (reference fp32 and float64 logits) at the north-star bar 1e-5 * max(1, |ref|)."""
    cfg, params, xi, xv, y, l32, l64, auc = load_golden(name)
    got = run(cpu_model(cfg, params), xi.reshape(len(xi), -1, 1), xv)
    assert got.dtype == np.float32 and got.shape == l32.shape
    assert logit_close(got, l32) < 1e-5
    assert logit_close(got, l64) < 1e-5


@pytest.mark.parametrize("name", ["tiny_fwfm_lw", "tiny_deepfwfm_lw"])
def test_cpu_auc_matches_reference(name):
    from sklearn.metrics import roc_auc_score
    cfg, params, xi, xv, y, l32, l64, auc = load_golden(name)
    got = run(cpu_model(cfg, params), xi, xv)
    assert abs(roc_auc_score(y, dfwfm_oracle.sigmoid(got)) - auc) <= 1e-4


def test_cpu_rows_independent_of_batch_and_threads():
    """A row's logit does not depend on its batch-mates, its block slot or the thread count (bit-identical)."""
    cfg, params, xi, xv, *_ = load_golden("deepfwfm_qr_mult")
    m = cpu_model(cfg, params)
    prev = torch.get_num_threads()
    try:
        torch.set_num_threads(1)
        one = run(m, xi, xv)
        torch.set_num_threads(4)
        four = run(m, xi, xv)
    finally:
        torch.set_num_threads(prev)
    assert np.array_equal(one, four)
    for B in (1, 17, 33):
        assert np.array_equal(run(m, xi[5:5 + B], xv[5:5 + B]), one[5:5 + B])
    assert run(m, xi[:0], xv[:0]).shape == (0,)


@pytest.mark.parametrize("bad", [-1, "n"])
def test_cpu_index_out_of_range_raises(bad):
    cfg, params, xi, xv, *_ = load_golden("deepfwfm_lw")
    m = cpu_model(cfg, params)
    x = xi[:8].copy()
    x[5, 3] = cfg["feature_sizes"][13 + 3] if bad == "n" else -1
    with pytest.raises(IndexError):
        run(m, x, xv[:8])
    run(m, xi[:8], xv[:8])  # the flag was cleared by the raising read


@pytest.mark.parametrize("name", train_golden_names())
def test_cpu_train_step_matches_reference(name):
    """One reference training step (train goldens: loss, every gradient, the Adam update) through autograd with
    the host backward and torch.optim.Adam (the reference's optimizer, what fit() uses on the CPU)."""
    cfg, params, xi, xv, y, loss_ref, logits_ref, ref = load_train_golden(name)
    m = cpu_model(cfg, params, is_deep_dropout=False).train()
    opt = torch.optim.Adam(m.parameters(), lr=cfg["lr"], weight_decay=cfg["l2"])
    out = m(torch.from_numpy(xi), torch.from_numpy(xv))
    loss = F.binary_cross_entropy_with_logits(out, torch.from_numpy(y))
    loss.backward()
    if cfg["use_lw"]:
        assert logit_close(out.detach().numpy(), logits_ref) < 1e-5
    else:
        assert logit_close_scaled(out.detach().numpy(), logits_ref, cfg, params, xi, xv) < 1e-5
    assert abs(loss.item() - loss_ref) <= 1e-5 * max(1.0, abs(loss_ref))
    grads = {k: p.grad.detach().numpy().copy() for k, p in m.named_parameters()}
    for k, (idx, gr, dp, gn) in ref.items():
        g = grads[k].reshape(-1).astype(np.float64)
        assert abs(np.linalg.norm(g) - gn) <= 1e-4 * gn + 1e-12, k
        gs = g[idx] if idx is not None else g
        assert np.abs(gs - gr).max() <= G_TOL * (np.abs(gr).max() + 1e-30), k
    opt.step()
    _, _, og, onew = torch_port.train_step(cfg, params, xi, xv, y, cfg["lr"], cfg["l2"])
    for k, p in m.named_parameters():
        d = (p.detach().numpy() - params[k]) / cfg["lr"]
        dr = (onew[k] - params[k]) / cfg["lr"]
        geff = np.abs(og[k] + cfg["l2"] * params[k]) > 1e-6
        assert np.abs(d - dr)[geff].max(initial=0.0) <= 2e-3, k


def test_cpu_dropout_step_matches_oracle_masks():
    """Deep-tower dropout p = 0.5: the host kernels draw the HIP kernels' counter-hash masks, which the oracle
    rebuilds; same thread-count independence."""
    cfg, params, xi, xv, y, *_ = load_train_golden("train_deepfwfm_lw")
    res = []
    prev = torch.get_num_threads()
    try:
        for threads in (1, 3):
            torch.set_num_threads(threads)
            m = cpu_model(cfg, params, is_deep_dropout=True).train()
            torch.manual_seed(99)
            seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())  # what train_forward draws next
            torch.manual_seed(99)
            out = m(torch.from_numpy(xi), torch.from_numpy(xv))
            F.binary_cross_entropy_with_logits(out, torch.from_numpy(y)).backward()
            res.append((out.detach().numpy(), {k: p.grad.numpy().copy() for k, p in m.named_parameters()}))
    finally:
        torch.set_num_threads(prev)
    assert np.array_equal(res[0][0], res[1][0])
    for k in res[0][1]:
        assert np.array_equal(res[0][1][k], res[1][1][k]), k
    widths = [cfg["field_size"] * cfg["embedding_size"]] + [cfg["deep_nodes"]] * cfg["h_depth"]
    masks = torch_port.dropout_masks(seed, 0.5, len(xi), widths)
    o_out, _, og, _ = torch_port.train_step(cfg, params, xi, xv, y, 1e-3, 0.0, masks, 0.5)
    assert logit_close(res[0][0], o_out) < 1e-5
    for k in og:
        assert np.abs(res[0][1][k] - og[k]).max() <= G_TOL * np.abs(og[k]).max() + 1e-12, k


def test_cpu_custom_op_kernel_opcheck():
    """torch.ops.dfwfm.forward's CPU kernel passes torch.library.opcheck and equals the module's forward."""
    from xsdeepfwfm_deprecated_amd import torch_ops
    cfg, params, xi, xv, *_ = load_golden("deepfwfm_lw")
    m = cpu_model(cfg, params).eval()
    xi_t, xv_t = torch.from_numpy(xi[:64]), torch.from_numpy(xv[:64])
    with torch.no_grad():
        ref = m(xi_t, xv_t)
    plist = [p for p in m.parameters() if p.requires_grad]
    mid = torch_ops.register(m)
    torch.library.opcheck(torch.ops.dfwfm.forward.default, (mid, xi_t, xv_t, plist, False, 0.0, 0),
                          test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))
    with torch.no_grad():
        out, _ = torch.ops.dfwfm.forward(mid, xi_t, xv_t, plist, False, 0.0, 0)
    assert torch.equal(out, ref)


def test_cpu_fit_learns_and_prunes():
    """fit() on the CPU (host kernels + torch.optim.Adam, the reference's -use_cuda 0 path) lowers the loss, and
    in-loop pruning (reference bisection) zeroes the requested share of the MLP weights."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = [1] * 13 + [50, 300, 7, 1000, 20, 5, 64, 9, 100, 3, 11, 17, 250, 4, 6, 30, 8, 2, 40, 12, 90, 5, 15,
                        300, 7, 60]
    xi, xv = synth.synth_inputs(sizes, 13, 2048, seed=5)
    logit = ((xi[:, 0] % 7) - 3) * 0.6 + (xv[:, 0] > 30) * 1.0 - 0.5
    y = (np.random.default_rng(1).random(2048) < 1 / (1 + np.exp(-logit))).astype(np.float32)
    m = DeepFMs(field_size=39, feature_sizes=sizes, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1, n_epochs=3,
                batch_size=256, learning_rate=1e-2, weight_decay=3e-7, h_depth=2, deep_nodes=64,
                is_deep_dropout=False, random_seed=3, warm=1, use_cuda=False)
    tr, _ = m.fit(xi.reshape(-1, 26, 1), xv, y, [], [], [], prune=1, prune_deep=1, prune_fm=1, prune_r=1)
    assert tr[-1] > tr[0] and tr[-1] > 0.7, tr
    from xsdeepfwfm_deprecated_amd.training import prune_step
    prune_step(m, 0.5, 1, 1, 1, 0.8, 1.0)  # what fit runs every 10 iterations past `warm` (reference :647-673)
    for name, p in m.named_parameters():
        z = float((p == 0).float().mean())
        if "linear" in name and "weight" in name:
            assert abs(z - 0.5) < 1e-3, (name, z)
    emb = torch.cat([p.reshape(-1) for n, p in m.named_parameters() if "fm_2nd_embeddings" in n])
    assert abs(float((emb == 0).float().mean()) - 0.4) < 1e-3
    R = m.field_cov.weight.detach()
    assert torch.equal(R == 0, (R == 0).t()) and float((R == 0).float().mean()) > 0.45


def test_main_all_cpu_fwfm_tiny_criteo_end_to_end(tmp_path):
    """BASELINE configs[0] as the reference runs it: main_all.py -dataset tiny-criteo -use_deep 0 -c FwFM
    -use_cuda 0 -time_on_cuda 0 -- ingest, fit on the host kernels, save, reload, size, and the benchmark's
    1- / 4-thread sweep plus single-sample latency (reference main_all.py:56-63, model/DeepFMs.py:982-1009)."""
    data = tmp_path / "data"
    data.mkdir()
    src = os.path.join(GOLDEN, "ingest", "tiny_train_head.csv")
    shutil.copy(src, data / "tiny_train_input.csv")
    shutil.copy(src, data / "tiny_test_input.csv")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")  # a GPU-less process
    r = subprocess.run([sys.executable, os.path.join(REPO, "main_all.py"), "-dataset", "tiny-criteo", "-n_epochs",
                        "1", "-batch_size", "256", "-data_root", str(tmp_path), "-use_deep", "0", "-c", "FwFM",
                        "-use_cuda", "0", "-time_on_cuda", "0"], cwd=str(tmp_path), capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = r.stdout
    assert "Training [1] loss" in out and "Acc:" in out
    assert "(1-Threads)" in out and "(4-Threads)" in out and "Avg forward pass time (ms)" in out
    assert any(f.startswith("FwFM_l2_") for f in os.listdir(tmp_path / "saved_models"))
