"""Training-step benchmark (BASELINE.json configs[4]: DeepFwFM training, DP over RCCL).

    python tools/bench_train.py [--gpus N] [--steps K] [--warmup W] [--batch 4096] [--first-order lw|fwlw]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_train.py

One step = the reference's fit() inner loop body (model/DeepFMs.py:619-637) on a resident synthetic
Criteo-39 batch: zero_grad, forward (train mode, deep dropout 0.5), BCE-with-logits mean, backward
(HIP), gradient all-reduce when WORLD_SIZE > 1, HIP Adam step (lr 1e-3, weight_decay 3e-7).
Prints one JSON line (samples/s over all ranks, ms/step, max over ranks).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--first-order", choices=["lw", "fwlw"], default="lw")
    ap.add_argument("--no-dropout", action="store_true")
    ap.add_argument("--deterministic", action="store_true",
                    help="fixed-order gradient sums (dfwfm_set_deterministic; the default): bit-identical runs")
    ap.add_argument("--atomic", action="store_true", help="float-atomic gradient sums (arrival order)")
    ap.add_argument("--copy-inputs", action="store_true",
                    help="copy every batch into the fused step's own input buffers (fit()'s path) instead of "
                         "reading the resident batches in place")
    ap.add_argument("--mode", choices=["fused", "autograd"], default="fused",
                    help="fused: FusedTrainStep (HIP-graph replay, what fit() runs); autograd: model() + "
                         "loss.backward() + HIP Adam")
    ap.add_argument("--exchange-world1", action="store_true",
                    help="one rank, but through the data-parallel step (a world-size-1 process group: touched-row "
                         "lists built, all-gathered and applied) -- the exchange kernels' cost without a second GPU")
    ap.add_argument("--apply-worlds", default="",
                    help="with --exchange-world1: afterwards time the apply of W ranks' lists (comma list of W; the "
                         "lists of W distinct batches built by the step itself)")
    ap.add_argument("--steps-per-graph", type=int, default=1,
                    help="fused, one rank: K > 1 replays K consecutive steps over the resident ring as one graph "
                         "(FusedTrainStep.step_many; --steps must be a multiple of K)")
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one process per GPU; started here unless "
                                                           "torchrun already set WORLD_SIZE)")
    a = ap.parse_args()
    from xsdeepfwfm_deprecated_amd.launch import spawn_ranks
    rc = spawn_ranks(a.gpus)  # before any HIP call
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or a.exchange_world1:
        import torch.distributed as dist
        backend = os.environ.get("DFWFM_BENCH_BACKEND", "nccl")  # gloo: rehearse N ranks on fewer GPUs
        if a.exchange_world1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group(backend, rank=0, world_size=1, **({"device_id": dev} if backend == "nccl" else {}))
        elif backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    from xsdeepfwfm_deprecated_amd.training import Adam, FusedTrainStep, allreduce_grads
    sizes = synth.CRITEO_FEATURE_SIZES
    fwlw = a.first_order == "fwlw"
    model = DeepFMs(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_fm=0, use_deep=1,
                    use_lw=1, use_fwlw=fwlw, numerical=13, is_deep_dropout=not a.no_dropout, use_cuda=True)
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    params = synth.synth_state(shapes, 39, 10, 400, True, True, seed=1234)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    model = model.to(dev).train()
    opt = Adam(model.parameters(), lr=1e-3, weight_decay=3e-7)
    B = a.batch
    batches = []
    for i in range(4):
        xi, xv = synth.synth_inputs(sizes, 13, B, seed=1000 * rank + i)
        y = synth.synth_labels(B, seed=1000 * rank + i)
        batches.append((torch.from_numpy(xi).to(dev), torch.from_numpy(xv).to(dev),
                        torch.from_numpy(y).float().to(dev)))

    trainer = None
    if a.mode == "fused":
        dist = torch.distributed if (world > 1 or a.exchange_world1) else None
        # the four resident batches are read in place (one captured graph set each), like a loader's ring of
        # device input buffers; --copy-inputs copies each batch into the step's own buffers first
        trainer = FusedTrainStep(model, B, lr=1e-3, weight_decay=3e-7, dist=dist, resident_inputs=not a.copy_inputs,
                                 deterministic=not a.atomic)

    def step(i):
        xi, xv, y = batches[i % 4]
        if trainer is not None:
            return trainer.step(xi, xv, y, B * world if world > 1 else None)
        opt.zero_grad()
        out = model(xi, xv)
        loss = F.binary_cross_entropy_with_logits(out, y)
        loss.backward()
        allreduce_grads(model)
        opt.step()
        return loss

    K = a.steps_per_graph if (trainer is not None and world == 1 and not a.exchange_world1) else 1
    if K > 1:
        if a.steps % K or a.warmup % K:
            raise SystemExit("--steps and --warmup must be multiples of --steps-per-graph")
        step(0)  # the first step runs eagerly (step_many needs one behind it)

        def step_k(i):
            return trainer.step_many([batches[(i + j) % 4] for j in range(K)])
    for i in range(0, a.warmup, K):
        step(i) if K == 1 else step_k(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    wall0 = time.perf_counter()
    t0.record()
    for i in range(0, a.steps, K):
        loss = step(i) if K == 1 else step_k(i)
    host = time.perf_counter() - wall0  # the host's enqueue time (ahead of the GPU if well under the step time)
    t1.record()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - wall0
    ms = t0.elapsed_time(t1)
    if world > 1:
        t = torch.tensor([ms], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        ms = float(t.item())
        torch.distributed.barrier()
    res = {"metric": "DeepFwFM training samples/sec (Criteo-39, Adam, dropout 0.5)",
           "value": round(world * B * a.steps / (ms / 1e3), 1), "unit": "samples/s", "n_gpus": world,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms / a.steps, 4), "per_gpu_batch": B,
           "first_order": a.first_order, "dropout": not a.no_dropout, "wall_s": round(wall, 3),
           "host_enqueue_us_per_step": round(host * 1e6 / a.steps, 1),
           "mode": a.mode, "deterministic": not a.atomic, "steps_per_graph": K, "inputs": "copied" if (a.copy_inputs or a.mode != "fused") else "resident (read in place)",
           "final_loss_sum": round(float(loss.item()), 4)}
    if trainer is not None and getattr(trainer, "sparse", False):
        # touched-row lists all-gathered per step (fixed capacity: sum over tables of min(batch, rows))
        res["exchange"] = {"backend": torch.distributed.get_backend(), "packed_bytes_per_rank": trainer.sp_bytes,
                           "dense_bucket_bytes": 4 * (trainer.n_bucket_a - trainer.n_tables),
                           "mlp_bucket_bytes": 4 * (trainer.grad.numel() - trainer.n_bucket_a)}
    if a.apply_worlds and trainer is not None and getattr(trainer, "sparse", False):
        res["apply"] = apply_bench(trainer, model, sizes, B, dev, [int(w) for w in a.apply_worlds.split(",")])
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1 or a.exchange_world1:
        torch.distributed.destroy_process_group()


def apply_bench(trainer, model, sizes, B, dev, worlds, reps=50):
    """The receive side of the touched-row exchange at world sizes the box cannot host: the step's own lists for
    max(worlds) distinct batches stacked as an all-gathered buffer and applied (one launch per rank and family, in
    rank order, as the step does) to a copy of the gradient buffer, graph-replayed."""
    import ctypes
    from xsdeepfwfm_deprecated_amd import _lib, synth
    L = _lib.lib()
    snaps = []
    for i in range(max(worlds)):
        xi, xv = synth.synth_inputs(sizes, 13, B, seed=7000 + i)
        y = synth.synth_labels(B, seed=7000 + i)
        trainer.step(*(torch.from_numpy(t).to(dev) for t in (xi, xv)), torch.from_numpy(y).float().to(dev))
        snaps.append(trainer.sp_send.clone())
    torch.cuda.synchronize(dev)
    counts = [[int(sn[f["o_cnt"]:f["o_cnt"] + 4].view(torch.int32).item()) for sn in snaps] for f in trainer.sp_fams]
    grad = trainer.grad.clone()
    out = {"entries_per_rank": {"width%d" % f["w"]: sum(c) / len(c) for f, c in zip(trainer.sp_fams, counts)},
           "capacity": {"width%d" % f["w"]: f["cap"] for f in trainer.sp_fams}}
    for w in worlds:
        recv = torch.stack(snaps[:w])
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)  # the capture stream
            for r in range(w):
                rb = recv[r].data_ptr()
                for f in trainer.sp_fams:
                    _lib.check(L.dfwfm_sparse_grads_apply(
                        ctypes.c_void_p(grad.data_ptr()), f["w"], ctypes.c_void_p(rb + f["o_dest"]),
                        ctypes.c_void_p(rb + f["o_rows"]), ctypes.c_void_p(rb + f["o_cnt"]), f["cap"], st), "apply")
        for _ in range(3):
            g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize(dev)
        out["world%d_us" % w] = round(e0.elapsed_time(e1) * 1e3 / reps, 2)
    return out


if __name__ == "__main__":
    main()
