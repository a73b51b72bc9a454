"""Benchmark of the hot path: DeepFwFM Criteo-39 forward, batch 4096 per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]     (N > 1: starts N ranks itself, one per GPU)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one fused forward (libdfwfm.so, a single HIP launch) over one
resident batch of 4096 synthetic Criteo-39 samples (BASELINE.json configs[1]).
Every rank processes its own batch (data-parallel shards, no collective on
the data path: "scaling": "weak").  Steps are replayed from a HIP graph
capture of the forward; K steps are timed with HIP events on the stream the
kernel runs on, bracketed by barrier + synchronize, max over ranks.

Rank 0 prints one JSON line with the throughput, the roofline of the fused
kernel (MFMA-bound: its MLP is 98.5 % of the arithmetic) and, at N = 1, the
host-CPU baseline (oracle/torch_port.py, the reference's op sequence in fp32
PyTorch-CPU) timed on this machine's cores, with the HIP logits / AUC checked
against that port on the same batch (``parity``).  ``--config qr|pruned`` runs
BASELINE.json configs[2] / [3] instead of configs[1]; ``--config fwfm`` runs configs[0]'s model (FwFM only,
no MLP: the HBM-bound gather path) at the Criteo-39 bench size.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "CTR samples/sec (forward, batch 4096, Criteo-39) at 1/2/4/8 MI355X; AUC match"
BATCH = 4096
PEAK_F32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md, dense f32 MFMA (= f32 vector peak)
PEAK_HBM_GBS = 8000.0         # MI355X_MICROARCH.md, HBM3E spec peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=600)
    ap.add_argument("--first-order", choices=["lw", "fwlw"], default="lw")
    ap.add_argument("--config", choices=["deepfwfm", "fwfm", "qr", "pruned", "fwfm_pruned"], default="deepfwfm",
                    help="BASELINE.json configs[1] (default), fwfm = configs[0]'s model (use_fwfm=1 use_deep=0: the "
                         "HBM-bound gather path) at Criteo-39 batch 4096, [2] QR embeddings (embedding_bag=1 "
                         "qr_flag=1, c=4, threshold 200, mult), [3] pruned (sparse 0.90, emb_r 0.444, prune_r 1: "
                         "the reference's magnitude masks applied on the device)")
    ap.add_argument("--settle-ms", type=float, default=400.0,
                    help="untimed back-to-back forwards for this long before the warmup steps: the chip raises its "
                         "clock over the first ~300 forwards (DESIGN.md section 7); reported in the JSON as 'settle'")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--graph-steps", type=int, default=20, help="forwards captured per hipGraph")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-per-call", action="store_true",
                    help="skip the per_call leg (one forward call per batch, sequential on one stream)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU sample per thread count")
    ap.add_argument("--inputs", choices=["uniform", "zipf"], default="uniform")
    ap.add_argument("--table-scale", type=int, default=1,
                    help="multiply every categorical table's row count by K (Criteo-39's 53 MB of second-order rows "
                         "fit the 256 MB Infinity Cache; K = 8 gives 424 MB, so the gather reads HBM)")
    ap.add_argument("--no-gate", action="store_true",
                    help="start the timed region without holding the streams until all K steps are enqueued")
    ap.add_argument("--sparse-mlp", type=float, default=None,
                    help="DeepFMs.sparse_mlp_max_density for this run (pruned config: the sparse deep tower when "
                         "the hidden layers' nonzero fraction is at most this); default: the model's")
    ap.add_argument("--pack-tables", type=int, default=1,
                    help="MLP-free configs: gather from the tables' serving copy (second + first order in one row; "
                         "0: the plain tables, A/B)")
    ap.add_argument("--pair-max", type=int, default=None,
                    help="DeepFMs.fwfm_pair_max for this run (fwfm_pruned: 0 runs the dense Gram FwFM)")
    ap.add_argument("--cu-mask", choices=["none", "even-odd", "lo-hi"], default=None,
                    help="give even-numbered streams one half of the CUs and odd-numbered streams the other (HIP CU "
                         "masks): with 32-sample workgroups a batch is 128 workgroups, one per CU of a half, so two "
                         "batches share each CU (default: even-odd with the 32-sample forward, else none)")
    ap.add_argument("--batch-set", type=int, default=32,
                    help="batches per forward launch (dfwfm_forward_batches: one grid over that many resident "
                         "batches, each batch its own inputs and logits); 1: one launch per batch (graph replay, "
                         "CU-masked stream pairs for the 32-sample forward)")
    ap.add_argument("--streams", type=int, default=None,
                    help="independent batch-4096 forwards in flight on this many HIP streams (2: a second "
                         "batch's workgroup shares each CU, hiding the gather / FwFM phases)")
    return ap.parse_args()


def _hip_runtime():
    """The HIP runtime torch already loaded (by its soname; any ROCm major), or None."""
    import ctypes
    import ctypes.util
    names = ["libamdhip64.so.7", "libamdhip64.so.6", "libamdhip64.so", ctypes.util.find_library("amdhip64")]
    for nm in names:
        if not nm:
            continue
        try:
            h = ctypes.CDLL(nm)
        except OSError:
            continue
        if all(hasattr(h, f) for f in ("hipHostMalloc", "hipHostFree", "hipStreamWaitValue32")):
            return h
    return None


class _HostGate:
    """hipStreamWaitValue32 on a coherent pinned host word: the streams wait until release() writes 1.

    The host releases the gate after at most GATE_STEPS steps are queued behind it (then keeps enqueueing while
    the GPU runs): a gate held until an unbounded number of commands is queued could fill the hardware queue,
    and the host would then block inside a launch without ever reaching release()."""

    def __init__(self):
        # allocated ahead of the warmup: the GPU idles from the warmup's end to release(), and an idle GPU lowers
        # its clock within milliseconds (a 20 ms gap cost 13 % of a 20-step region, profiles/r03/r03bm_*)
        import ctypes
        self._hip = _hip_runtime()
        if self._hip is None:
            raise OSError("HIP runtime without hipStreamWaitValue32")
        self._p = ctypes.c_void_p()
        rc = self._hip.hipHostMalloc(ctypes.byref(self._p), ctypes.c_size_t(64), ctypes.c_uint(0x40000000))
        if rc != 0:
            raise RuntimeError(f"hipHostMalloc: {rc}")
        self._word = ctypes.cast(self._p, ctypes.POINTER(ctypes.c_uint32))
        self._word[0] = 0

    def arm(self, streams):
        import ctypes
        for stream in streams:  # flags 0 = hipStreamWaitValueGte
            rc = self._hip.hipStreamWaitValue32(ctypes.c_void_p(stream.cuda_stream), self._p, ctypes.c_uint32(1),
                                                ctypes.c_uint(0), ctypes.c_uint32(0xFFFFFFFF))
            if rc != 0:
                raise RuntimeError(f"hipStreamWaitValue32: {rc}")

    def release(self):
        self._word[0] = 1
        self.released = True

    released = False

    def __del__(self):
        try:
            self._hip.hipHostFree(self._p)
        except Exception:
            pass


def r32_on(config="deepfwfm", cu_mask="even-odd", batch_set=1):
    """The library runs the 32-sample-workgroup forward (fwd32_kernel) for the bench's deep configs when the
    launch's 32-sample workgroups give every CU of its stream two (a batch set of >= 4 batches of 4096 on the whole
    chip), or one on a CU-masked stream (one batch on half of the chip); DFWFM_DIAG r32=1 forces it, r32=0 never."""
    env = diag_opt("r32")
    if config in ("fwfm", "fwfm_pruned") or env == "0":
        return False
    return env is not None or cu_mask not in (None, "none") or batch_set >= 4


def diag_opt(key):
    """The library's DFWFM_DIAG test / diagnostics option `key` (a "key=value,..." list), or None."""
    for kv in os.environ.get("DFWFM_DIAG", "").split(","):
        k, _, v = kv.partition("=")
        if k == key:
            return v
    return None


def masked_streams(dev, S, how):
    """S HIP streams (torch ExternalStream): with how = even-odd / lo-hi, even streams on one half of the CUs (even
    CU ids / the low ids) and odd streams on the other (hipExtStreamCreateWithCUMask)."""
    if how in (None, "none"):
        return [torch.cuda.Stream(dev) for _ in range(S)], None
    import ctypes
    hip = _hip_runtime()
    if hip is None or not hasattr(hip, "hipExtStreamCreateWithCUMask"):
        raise RuntimeError("hipExtStreamCreateWithCUMask unavailable")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (ncu + 31) // 32
    streams, handles = [], []
    for k in range(S):
        mask = (ctypes.c_uint32 * words)()
        for cu in range(ncu):
            side = (cu & 1) if how == "even-odd" else int(cu >= ncu // 2)
            if side == (k & 1):
                mask[cu // 32] |= 1 << (cu % 32)
        h = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
        handles.append(h)
        streams.append(torch.cuda.ExternalStream(h.value, device=dev))
    return streams, handles


def kernel_name(config="deepfwfm", cu_mask="none", batch_set=1):
    """The forward kernel instantiation the library picks for Criteo-39 / 3x400 (D, tiles per wave, K split,
    train, part, tile groups); DFWFM_DIAG ng / r32 / part3 / p3ng select the test variants."""
    if r32_on(config, cu_mask, batch_set):
        qr = 'true' if config == 'qr' else 'false'
        return f"dfwfm::fwd32_kernel<10,{qr}>"
    if config in ("fwfm", "fwfm_pruned"):
        if diag_opt("part3") == "0":
            return "dfwfm::fwd_kernel<10,1,1,false,0,4,0>"
        png = diag_opt("p3ng")
        ng = 4 if png == "4" or (png is None and batch_set > 1) else 8  # batch sets: four waves
        return f"dfwfm::fwd_kernel<10,1,1,false,3,{ng},3,false>"  # MLP-free, 3 FwFM row tiles, no QR field
    ng = 4 if diag_opt("ng") == "4" else 8
    tpw = 6 if ng == 4 else 3
    ns = 25 if ng == 8 and tpw == 3 else 0  # static 25-chunk K loop
    qr = "true" if (config == "qr" or ns != 25) else "false"  # the static form without QR fields: QR=false
    return f"dfwfm::fwd_kernel<10,{tpw},1,false,0,{ng},{ns},{qr}>"  # as rocprofv3 names it (QR argument last)


def algorithmic_counts(cfg, sizes=None):
    """Per-sample algorithmic FLOPs and HBM bytes of the fused forward."""
    F, D, N, H, num = 39, 10, 400, 3, 13
    ncat = F - num
    flops = 0
    flops += 741 * D * 2                              # FwFM pairs
    if cfg["use_deep"]:
        flops += 2 * (F * D * N + (H - 1) * N * N + N)  # MLP + fc
    flops += F * D * 2 if cfg["use_fwlw"] else 0       # fwlw
    bytes_ = ncat * 8 + num * 4 + ncat * D * 4 + 4     # Xi + Xv + gathered rows + logit
    if not cfg["use_fwlw"]:
        bytes_ += ncat * 4                             # first-order table rows
    if cfg.get("qr_flag") and sizes is not None:       # QR fields read a remainder row too
        nqr = sum(1 for n in sizes[num:] if n > cfg["qr_threshold"])
        bytes_ += nqr * (D * 4 + (0 if cfg["use_fwlw"] else 4))
    return flops, bytes_


GATE_STEPS = 640  # steps queued behind the host gate before it is released (see _HostGate)


def max_over_ranks(x, world, dev):
    """The slowest rank's value of x (the timed region's length): all-reduce MAX over the process group."""
    if world <= 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64 if dev.type == "cpu" else torch.float32, device=dev)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def aggregate_value(world, steps, ms):
    """Whole-job samples/s: every rank ran `steps` batches of BATCH in at most `ms` (the max over ranks)."""
    return world * BATCH * steps / (ms / 1e3)


RANK_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def stub_main(a, stub_ms):
    """CPU rehearsal of the N-rank path (DFWFM_BENCH_STUB_MS set; tests/test_launch.py): the same rank processes
    (spawn_ranks), rank environment, barriers around the timed region and max-over-ranks aggregation as main(),
    over gloo, with each step's forward replaced by a host sleep of stub_ms x (1 + rank / world) -- rank N-1 is the
    slowest, so the aggregate must be world x BATCH x steps over ITS region.  Never touches a GPU."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    env = {k: os.environ.get(k) for k in RANK_ENV}
    if world > 1:
        dist.init_process_group("gloo")
    per_step = stub_ms * (1.0 + rank / world) / 1e3
    for _ in range(a.warmup):
        time.sleep(per_step)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        time.sleep(per_step)
    ms_rank = (time.perf_counter() - t0) * 1e3
    if world > 1:
        dist.barrier()
    cpu = torch.device("cpu")
    ms = max_over_ranks(ms_rank, world, cpu)
    envs, times = [env], [ms_rank]
    if world > 1:
        envs, times = [None] * world, [None] * world
        dist.all_gather_object(envs, env)
        dist.all_gather_object(times, ms_rank)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(aggregate_value(world, a.steps, ms), 1),
                          "unit": "samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": round(ms / a.steps, 6), "higher_is_better": True, "scaling": "weak",
                          "stub": {"ms_per_step": stub_ms, "rank_env": envs, "rank_ms": times}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    a = parse()
    # --gpus N without torchrun: start N ranks (one process per GPU) before anything touches the GPU, and exit
    # with their status; rank 0 prints the JSON line
    from xsdeepfwfm_deprecated_amd.launch import spawn_ranks
    rc = spawn_ranks(a.gpus)
    if rc is not None:
        sys.exit(rc)
    if os.environ.get("DFWFM_BENCH_STUB_MS"):  # CPU rehearsal of the rank path (tests only)
        return stub_main(a, float(os.environ["DFWFM_BENCH_STUB_MS"]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world} (torchrun); using WORLD_SIZE", file=sys.stderr)
    # one process per GPU; the modulo only matters for rehearsing N > 1 on fewer GPUs (with
    # DFWFM_BENCH_BACKEND=gloo: RCCL refuses two ranks on one device)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("DFWFM_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    K = max(1, a.table_scale)
    sizes = synth.CRITEO_FEATURE_SIZES[:13] + [n * K for n in synth.CRITEO_FEATURE_SIZES[13:]]
    fwlw = a.first_order == "fwlw"
    qr = a.config == "qr"
    deep = int(a.config not in ("fwfm", "fwfm_pruned"))
    cfg = dict(field_size=39, numerical=13, embedding_size=10, use_fwfm=1, use_fm=0, use_logit=0, use_deep=deep,
               use_lw=1, use_fwlw=int(fwlw), h_depth=3, deep_nodes=400, embedding_bag=int(qr), qr_flag=int(qr),
               qr_operation="mult", qr_collisions=4, qr_threshold=200)
    model = DeepFMs(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_fm=0, use_deep=deep,
                    use_lw=1, use_fwlw=fwlw, numerical=13, embedding_bag=int(qr), qr_flag=int(qr),
                    qr_operation="mult", qr_collisions=4, qr_threshold=200, use_cuda=True)
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    params = synth.synth_state(shapes, 39, 10, 400, True, bool(deep), seed=1234)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    model = model.to(dev).eval()
    model.strict_index_check = False
    if a.config == "fwfm_pruned":
        model.fwfm_pair_max = 192  # the pair path (measured level with the dense Gram: DESIGN.md section 3.3)
    if a.pair_max is not None:
        model.fwfm_pair_max = a.pair_max
    model.pack_tables = bool(a.pack_tables)
    if a.config in ("pruned", "fwfm_pruned"):
        # reference :647-673 with sparse=0.90, emb_r=0.444, prune_r=1 (main_all.py flags of config 4); FwFM-only:
        # R keeps 73 of 741 pairs and the forward sums those (dfwfm_model_build_fwfm_pairs)
        from xsdeepfwfm_deprecated_amd.training import prune_step
        prune_step(model, 0.90, 1, 1, 1, 0.444, 1.0)
        torch.cuda.synchronize(dev)
        params = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}

    # batches in flight: 2 fill the CUs' register files for the deep configs (two eight-wave workgroups per
    # CU); the FwFM-only forward is latency-bound and gains from a third (three eight-wave workgroups per CU)
    # deep configs: four batches in flight on CU-masked stream pairs (even / odd CU ids): a 4096-row batch is 128
    # 32-sample workgroups, which cover a half, so the library runs fwd32_kernel and every CU holds two batches
    # (DESIGN.md section 3); DFWFM_DIAG=r32=0: the 16-sample kernel on two plain streams
    # batch sets (default): every launch is one grid over up to M resident batches on the whole chip (the
    # 32-sample forward for the deep configs: a set's workgroups cover every CU twice over); when the K steps
    # fit one set they are ONE launch, else two streams, so that the next set's workgroups take the CU slots
    # the current one frees while it drains.  --batch-set 1: one launch per batch from captured graphs; the deep
    # configs then run four batches in flight on CU-masked stream pairs
    M = max(1, a.batch_set)
    r32_default = deep and diag_opt("r32") != "0"
    cu_mask = a.cu_mask if a.cu_mask is not None else ("even-odd" if r32_default and M == 1 else "none")
    S = max(1, a.streams if a.streams is not None else
            ((1 if a.steps <= M else 2) if M > 1 else (3 if not deep else (4 if r32_default else 2))))
    # distinct resident batches, rotated: at least every batch of every launch in flight (S launches of up to M
    # batches), so no input batch is read twice inside one launch or by two concurrent launches
    n_bufs = max(8, S * M)
    batches = []
    for i in range(n_bufs):
        seed = 1000 * rank + i
        if a.inputs == "zipf":
            xi, xv = synth.zipf_inputs(sizes, 13, BATCH, seed=seed)
        else:
            xi, xv = synth.synth_inputs(sizes, 13, BATCH, seed=seed)
        batches.append((torch.from_numpy(xi).to(dev), torch.from_numpy(xv).to(dev)))
    outs = [torch.empty(BATCH, dtype=torch.float32, device=dev) for _ in range(S)]
    set_outs = [[torch.empty(BATCH, dtype=torch.float32, device=dev) for _ in range(M)] for _ in range(S)] \
        if M > 1 else None

    with torch.no_grad():
        eng = model._sync_inference(dev)  # (MLP-free configs: the tables' serving copy, built once here)
        if a.sparse_mlp is not None:
            model.sparse_mlp_max_density = a.sparse_mlp
        sparse_on = eng.sync_sparse(model.sparse_mlp_max_density) if deep else False
        streams, _stream_handles = masked_streams(dev, S, cu_mask)
        for st in streams:
            st.wait_stream(torch.cuda.current_stream(dev))

        def step(i, k):
            xi, xv = batches[(i + k) % n_bufs]
            eng.forward(xi, xv, outs[k])

        # G consecutive forwards per captured graph (launch cost amortised: a single-kernel
        # replay is host-bound at ~10-16 us); remainder graphs keep the count exact.  With S streams
        # each stream replays its own graphs (S batches in flight at once) and the K steps are split
        # over the streams: exactly K batches are timed.
        def per_stream(n):
            return [n // S + (1 if k < n % S else 0) for k in range(S)]
        G = max(1, min(a.graph_steps, max(per_stream(a.steps))))
        graphs = None
        set_pos = [0] * S
        if M > 1:
            def launch_set(k, n):
                # n batches (rotating over the resident ones) in one dfwfm_forward_batches launch on stream k
                i0 = set_pos[k] * S + k
                set_pos[k] += n
                eng.forward_batches([batches[(i0 + j * S) % n_bufs] for j in range(n)], set_outs[k][:n])
            for k in range(S):
                with torch.cuda.stream(streams[k]):
                    launch_set(k, M)  # initialise everything outside the timed region
        elif not a.no_graph:
            def capture(n, k):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=streams[k]):
                    for i in range(n):
                        step(i, k)
                return g
            for k in range(S):
                with torch.cuda.stream(streams[k]):
                    step(0, k)  # initialise everything outside the capture
            graphs = []
            for k in range(S):
                gk = {G: capture(G, k)}
                for n in per_stream(a.steps) + per_stream(a.warmup):
                    if n % G and n % G not in gk:
                        gk[n % G] = capture(n % G, k)
                graphs.append(gk)

        def run_n(n_total, progress=None):
            # enqueue round-robin over the streams (stream k's replays must not wait behind the host
            # enqueueing all of stream 0's first: the streams would start one after the other);
            # progress(steps enqueued so far) after every round
            ns = per_stream(n_total)
            done = 0
            if M > 1:
                for r in range(max(ns) // M + 1):
                    for k in range(S):
                        left = ns[k] - r * M
                        if left <= 0:
                            continue
                        with torch.cuda.stream(streams[k]):
                            launch_set(k, min(M, left))
                        done += min(M, left)
                    if progress:
                        progress(done)
                return
            if graphs is None:
                for i in range(max(ns)):
                    for k in range(S):
                        if i < ns[k]:
                            with torch.cuda.stream(streams[k]):
                                step(i, k)
                            done += 1
                    if progress:
                        progress(done)
                return
            for r in range(max(ns) // G + 1):
                for k in range(S):
                    left = ns[k] - r * G
                    if left <= 0:
                        continue
                    with torch.cuda.stream(streams[k]):
                        graphs[k][G if left >= G else left].replay()
                    done += min(G, left)
                if progress:
                    progress(done)

        # settle: untimed back-to-back forwards until the chip has run them for --settle-ms (its clock ramps
        # over the first few hundred forwards); then the W warmup steps, then the K timed steps
        settle_n, settle_t0 = 0, time.perf_counter()
        chunk = S * min(M, max(per_stream(a.steps))) if M > 1 else max(S * G, 8)  # settle launches = timed ones
        while a.settle_ms > 0:
            run_n(chunk)
            settle_n += chunk
            torch.cuda.synchronize(dev)
            if (time.perf_counter() - settle_t0) * 1e3 >= a.settle_ms:
                break
        settle_ms = (time.perf_counter() - settle_t0) * 1e3
        # per-stream events: a launch's duration while S run side by side (what rocprofv3 reports); everything
        # the timed region needs is created before the warmup, so that the GPU's idle gap between the warmup's end
        # and the region's start is only the synchronisation and the enqueue (reported as idle_before_region_us)
        s0 = [torch.cuda.Event(enable_timing=True) for _ in range(S)]
        s1 = [torch.cuda.Event(enable_timing=True) for _ in range(S)]
        wend = [torch.cuda.Event(enable_timing=True) for _ in range(S)]
        # the K steps are enqueued behind a device-side wait on a host flag (one wait per stream, one
        # flag), released once everything is queued: the timed region measures the GPU running K forwards,
        # not the host submitting graphs.  The region runs from the earliest stream's start event to the
        # latest stream's end event (each recorded on its own stream): cross-stream event waits inside the
        # region cost ~20 us each on this stack (a late second stream, a late final event)
        gate = None
        if not a.no_gate:
            try:
                gate = _HostGate()
            except (OSError, RuntimeError) as e:  # no gate on this runtime: time as --no-gate does
                print(f"bench: host gate unavailable ({e}); timing without it", file=sys.stderr)
        run_n(a.warmup)
        for k, st in enumerate(streams):
            wend[k].record(st)
        torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)
        if os.environ.get("DFWFM_BENCH_IDLE_MS"):  # diagnostics: an idle gap before the timed region
            time.sleep(float(os.environ["DFWFM_BENCH_IDLE_MS"]) / 1e3)
        wall0 = time.perf_counter()
        if gate is not None:
            gate.arm(streams)
        for k, st in enumerate(streams):
            if k and gate is None:
                st.wait_stream(streams[0])
            s0[k].record(st)

        def progress(done):
            if gate is not None and not gate.released and done >= GATE_STEPS:
                gate.release()
        run_n(a.steps, progress)
        for k, st in enumerate(streams):
            s1[k].record(st)
        if gate is not None and not gate.released:
            gate.release()
        for st in streams:
            st.synchronize()
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - wall0
        if world > 1:
            torch.distributed.barrier()
    # the timed region: the earliest stream start to the latest stream end
    first = min(range(S), key=lambda k: s0[0].elapsed_time(s0[k]))
    last = max(range(S), key=lambda k: s0[0].elapsed_time(s1[k]))
    ms = s0[first].elapsed_time(s1[last])
    idle_us = max(0.0, -max(s0[first].elapsed_time(w) for w in wend) * 1e3)  # last warmup end -> region start
    # per launch, S side by side (what rocprofv3 reports); a launch is one batch, or a set of up to M
    units = BATCH * (min(M, max(per_stream(a.steps))) if M > 1 else 1)
    n_launch = sum(-(-n // M) for n in per_stream(a.steps)) if M > 1 else a.steps
    launch_ms = sum(s0[k].elapsed_time(s1[k]) for k in range(S)) / n_launch
    # where the streams start and end inside the timed region (fill / drain of a short run)
    skew = {"start_us": [round(s0[first].elapsed_time(s0[k]) * 1e3, 2) for k in range(S)],
            "end_us": [round(s1[k].elapsed_time(s1[last]) * 1e3, 2) for k in range(S)]}
    # the graphs, then the CU-masked streams they were captured on, are released here, before the runtime's own
    # teardown (a masked stream left to process exit crashed in __cxa_finalize under rocprofv3)
    graphs = None
    torch.cuda.synchronize(dev)
    # and the torch wrappers of those streams go first: nothing may hold a handle that is about to be destroyed
    streams = st = None
    if _stream_handles:
        hip = _hip_runtime()
        for h in _stream_handles:
            hip.hipStreamDestroy(h)
    ms = max_over_ranks(ms, world, dev)

    ms_per_step = ms / a.steps
    mfma_bound = "mfma"
    value = aggregate_value(world, a.steps, ms)
    flops, bytes_ = algorithmic_counts(cfg, sizes)
    if a.config == "pruned" and sparse_on:
        # the sparse tower does the nonzero products only: 2 x nonzero hidden weights + fc, and the
        # FwFM's nonzero pairs (73 of 741 under these masks)
        nnz = sum(int(np.count_nonzero(params[f"net_1_linear_{h}.weight"])) for h in range(1, 4))
        R = params["field_cov.weight"].astype(np.float64)
        pairs = int(np.count_nonzero(np.triu(0.5 * (R + R.T), 1)))
        flops = 2 * nnz + 2 * 400 + 2 * pairs * 10
    # achieved = algorithmic FLOP of one launch / its duration, times the launches in flight (each of
    # the S concurrent launches takes ~S x the per-batch time): the aggregate rate over the timed region
    achieved_tf = flops * units * S / (launch_ms / 1e3) / 1e12
    achieved_gbs = bytes_ * units * S / (launch_ms / 1e3) / 1e9
    kname = kernel_name(a.config, cu_mask, M)
    if a.config == "pruned" and sparse_on:
        kname = "dfwfm::fwd_kernel<10,1,1,false,1,4> + dfwfm::sparse_mlp_kernel<64>"
        mfma_bound = "valu"  # the sparse MLP runs on the f32 vector FMAs (same 157.3 TF/s peak on gfx950)
    workload_id = f"{a.config}/{a.first_order}/scale{K}/{a.inputs}" + ("/set" if M > 1 else "") + \
        ("/packed" if getattr(eng, "_packed_on", False) else "")
    traffic = pmc_traffic(kname, workload_id, units // BATCH)

    result = {
        "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(ms_per_step, 6), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic Criteo-39 ({a.inputs} indices over the real field sizes, Xv integers 0..63; "
                "deterministic hash-init weights with the reference's init_weights scales)",
        "config": {"workload": (f"DeepFwFM forward, Criteo-39, emb 10, MLP 3x400, FwFM + {a.first_order}"
                                if deep else f"FwFM-only forward (use_deep=0), Criteo-39, emb 10, FwFM + {a.first_order}")
                               + {"deepfwfm": "", "fwfm": "", "qr": ", QR embeddings (c=4, mult, threshold 200)",
                                  "pruned": ", pruned (sparse 0.90, emb_r 0.444, prune_r 1)",
                                  "fwfm_pruned": ", pruned (sparse 0.90, emb_r 0.444, prune_r 1; FwFM over R's "
                                                 "nonzero pairs)"}[a.config]
                               + (f", tables x{K} ({sum(sizes[13:]) * 40 / 1e6:.0f} MB of second-order rows)"
                                  if K > 1 else "")
                               + f"; batch {BATCH} per GPU",
                   "workload_id": workload_id,
                   "global_batch": BATCH * world, "per_gpu_batch": BATCH,
                   "parallelism": f"dp{world} (independent batch shards, no collective)",
                   "launch": (f"batch sets: {units // BATCH} batches of {BATCH} per launch (dfwfm_forward_batches, "
                              f"one grid; value = the aggregate over those batches; each batch its own resident inputs "
                              f"and logits, {n_bufs} distinct resident batches, none read twice by the launches in "
                              f"flight)" if M > 1 else
                              "eager" if a.no_graph else f"hipGraph replay, {G} forwards per graph")
                             + (f", {S} streams (batches in flight)" if S > 1 else "")
                             + (f", CU masks {cu_mask} (stream pairs on chip halves)" if cu_mask != "none" else "")},
        "settle": {"forwards": settle_n, "ms": round(settle_ms, 1),
                   "what": "untimed back-to-back forwards before the warmup steps (clock ramp)"},
        "wall_s": round(wall, 4),
        "streams_in_region": skew,
        "idle_before_region_us": round(idle_us, 1),
    }
    mfma = {"bound": mfma_bound, "achieved": round(achieved_tf, 3), "peak": PEAK_F32_MFMA_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved_tf / PEAK_F32_MFMA_TFLOPS, 4), "flops_per_sample": flops}
    hbm = {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
           "frac": round(achieved_gbs / PEAK_HBM_GBS, 4), "bytes_per_sample": bytes_}
    common = {"traffic": traffic, "kernel": kname, "units_per_launch": units, "launch_us": round(launch_ms * 1e3, 3),
              "launches_in_flight": S}
    if cfg["use_deep"]:  # 98.5 % of the arithmetic is the MLP: MFMA-bound (intensity ~690 FLOP/B)
        result["roofline"] = {**mfma, **common}
    else:                # gather + FwFM only: ~12 FLOP/B, below the f32 ridge -> HBM-bound
        result["roofline"] = {**hbm, **common}
        if traffic:      # the fabric rate of the PMC-counted bytes (40-B rows fetched as 128-B lines)
            result["roofline"]["traffic_gbs"] = round(traffic * S / (launch_ms / 1e3) / 1e9, 1)
        if a.config in ("fwfm", "fwfm_pruned") and a.inputs == "uniform" and K == 1:
            # the same 26 rows x 4096 samples from the same tables and nothing else (tools/ubench_gather.hip,
            # one lane per row, three batches in flight): what the gather alone costs at this concurrency
            floor_us = 1.596
            result["roofline"]["gather_floor"] = {
                "us_per_batch": floor_us, "frac": round(floor_us / (ms_per_step * 1e3), 4),
                "source": "tools/ubench_gather.hip 3 (profiles/r02/r02q_ubench_gather_nb3.log)"}
        result["roofline_mfma"] = mfma
    if deep and not a.no_per_call and not (a.config == "pruned" and sparse_on):
        # north_star: "achieved HBM GB/s on the gather" -- the gather / shallow half as its own launch
        gl = gather_leg(eng, batches, dev, a.steps, bytes_ - 4)
        if world > 1:
            gl["us_per_batch"] = round(max_over_ranks(gl["us_per_batch"], world, dev), 3)
        result["roofline_gather"] = gl
    if not a.no_per_call and not (a.config == "pruned" and sparse_on):
        pc = per_call_leg(eng, batches, dev, a.steps, flops, bytes_, a.config)
        if world > 1:
            pc["us_per_batch"] = round(max_over_ranks(pc["us_per_batch"], world, dev), 3)
            pc["samples_per_s"] = round(world * BATCH / (pc["us_per_batch"] / 1e6), 1)
        result["per_call"] = pc
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        result["cpu_baseline"], result["parity"] = cpu_baseline(cfg, params, sizes, a.cpu_seconds, model, dev)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def per_call_leg(eng, batches, dev, steps, flops, bytes_, config, settle_ms=150.0):
    """The reference's call pattern beside the headline: one forward call per batch of 4096, the calls one after
    the other on ONE plain stream (eval_by_batch / time_forward_pass, model/DeepFMs.py:750-780, :1012-1028), each
    over its own resident batch; the library picks the kernel for a lone batch on the whole chip.  The forwards are
    replayed from captured graphs of G calls (launch cost amortised as a serving loop would), after an untimed
    settle, timed with HIP events on that stream."""
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    out = torch.empty(BATCH, dtype=torch.float32, device=dev)
    G = max(1, min(20, steps))
    n = len(batches)
    with torch.no_grad(), torch.cuda.stream(st):
        eng.forward(*batches[0], out)
        gs = []
        for j in range(max(1, min(4, n // G))):  # graphs over different batches, replayed in turn
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                for i in range(G):
                    eng.forward(*batches[(j * G + i) % n], out)
            gs.append(g)
        reps = -(-steps // G)
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < settle_ms:
            for g in gs:
                g.replay()
            st.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for r in range(reps):
            gs[r % len(gs)].replay()
        e1.record(st)
        st.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * G)
    res = {"what": "one forward call per batch, sequential on one stream (the reference's per-batch call pattern)",
           "batches": reps * G, "us_per_batch": round(us, 3), "samples_per_s": round(BATCH / (us / 1e6), 1),
           "kernel": kernel_name(config, "none", 1)}
    if config in ("fwfm", "fwfm_pruned"):
        res["hbm_frac"] = round(bytes_ * BATCH / (us / 1e6) / 1e9 / PEAK_HBM_GBS, 4)
    else:
        res["mfma_frac"] = round(flops * BATCH / (us / 1e6) / 1e12 / PEAK_F32_MFMA_TFLOPS, 4)
    return res


def gather_leg(eng, batches, dev, steps, read_bytes, settle_ms=100.0, streams=4):
    """The deep forward's gather / shallow half alone (dfwfm_forward_gather: the MLP-free kernel, fwd_kernel PART 3,
    storing deep_emb -- the per-field rows of model/DeepFMs.py:300-367 into deep_emb (:398), first + second order)
    over the resident batches, one batch of 4096 per call, replayed from captured graphs like per_call: on one
    stream (`lone`: one 16-sample tile per CU, the chain's latency) and with `streams` calls in flight (the
    headline numbers: throughput).  `achieved` = the gather's algorithmic read bytes per sample (Xi, Xv, the
    categorical rows, the first-order weights: what the fused kernel also reads) / its time; `achieved_incl_store`
    adds this launch's own deep_emb + first/second stores, which the fused kernel keeps in LDS."""
    G = max(1, min(20, steps))
    n = len(batches)

    def timed(S):
        sts = [torch.cuda.Stream(dev) for _ in range(S)]
        for st in sts:
            st.wait_stream(torch.cuda.current_stream(dev))
        gs, bufs = [], []  # every stream's graph and the output buffers its graph writes (kept alive here)
        with torch.no_grad():
            for k, st in enumerate(sts):
                with torch.cuda.stream(st):
                    E = eng.forward_gather(*batches[k % n])
                    bufs.append(E)
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=st):
                        for i in range(G):
                            eng.forward_gather(*batches[(k * G + i) % n], E[0], E[1])
                    gs.append(g)
            reps = -(-steps // G)
            t0 = time.perf_counter()
            while (time.perf_counter() - t0) * 1e3 < settle_ms:
                for k, st in enumerate(sts):
                    with torch.cuda.stream(st):
                        gs[k].replay()
                torch.cuda.synchronize(dev)
            e0 = [torch.cuda.Event(enable_timing=True) for _ in sts]
            e1 = [torch.cuda.Event(enable_timing=True) for _ in sts]
            for k, st in enumerate(sts):
                e0[k].record(st)
            for r in range(reps):
                for k, st in enumerate(sts):
                    with torch.cuda.stream(st):
                        gs[k].replay()
            for k, st in enumerate(sts):
                e1[k].record(st)
            torch.cuda.synchronize(dev)
        first = min(range(S), key=lambda k: e0[0].elapsed_time(e0[k]))
        last = max(range(S), key=lambda k: e0[0].elapsed_time(e1[k]))
        us = e0[first].elapsed_time(e1[last]) * 1e3 / (reps * G * S)
        del gs  # the graphs go before the buffers they write
        torch.cuda.synchronize(dev)
        return us, reps * G * S, bufs[0][0].shape[1] * 4 + 4

    us1, _, store = timed(1)
    us, nb, store = timed(streams)
    gbs = read_bytes * BATCH / (us / 1e6) / 1e9
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4), "bytes_per_sample": read_bytes,
            "achieved_incl_store": round((read_bytes + store) * BATCH / (us / 1e6) / 1e9, 1),
            "store_bytes_per_sample": store, "us_per_batch": round(us, 3), "batches": nb,
            "in_flight": streams,
            "lone": {"us_per_batch": round(us1, 3),
                     "achieved": round(read_bytes * BATCH / (us1 / 1e6) / 1e9, 1)},
            "kernel": "dfwfm::fwd_kernel<10,1,1,false,3,8,3,false> (dfwfm_forward_gather)",
            "what": "the deep forward's gather / shallow half as its own launch per 4096-sample batch, "
                    f"{streams} streams in flight (lone: one stream)"}


def pmc_traffic(kname, workload_id, batches=1):
    """HBM bytes per launch of kernel `kname` on workload `workload_id` from the committed PMC summary
    (tools/pmc.sh + tools/pmc_summary.py: rocprofv3 --pmc over this bench's own command): 2 x FETCH_SIZE +
    WRITE_SIZE, FETCH doubled per the gfx950 calibration; None unless that kernel was counted on that workload.
    Batch sets: the counted bytes per batch times the `batches` of this run's launches."""
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(pmc))
    except Exception:
        return None
    for e in d.get("entries", []):
        if e.get("kernel") == kname and e.get("workload") == workload_id:
            if "hbm_bytes_per_batch" in e:
                return e["hbm_bytes_per_batch"] * batches
            return e.get("hbm_bytes_per_launch")
    return None


def _time_port(torch_port, cfg, tp, xi, xv, seconds, threads):
    torch.set_num_threads(threads)
    torch_port.forward(cfg, tp, xi, xv)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        torch_port.forward(cfg, tp, xi, xv)
        n += 1
        el = time.perf_counter() - t0
        if (el >= seconds and n >= 2) or n >= 400:
            return n, el


def _cpu_quota():
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        return None


def cpu_baseline(cfg, params, sizes, seconds, model=None, dev=None):
    """oracle/torch_port.py (the reference's fp32 op sequence on PyTorch-CPU) on this host: every core of this
    process's affinity mask, and one thread; the port / reference time ratio measured in the build container
    (tools/calibrate_cpu_port.py -> profiles/cpu_calibration.json) rides along.  On the same batch, the HIP
    forward's logits and AUC against the port's (the metric's "AUC match": labels drawn from the port's
    sigmoid, AUC of both score vectors by the on-device metrics)."""
    from oracle import torch_port
    from xsdeepfwfm_deprecated_amd import synth
    # every core this process may use: the affinity mask, capped by the cgroup CPU quota (the GPU box's
    # share is 16 CPUs of a 256-core affinity mask; 256 threads under that quota ran ~100x slower, r02a)
    aff = len(os.sched_getaffinity(0))
    quota = _cpu_quota()
    cores = max(1, min(aff, int(math.ceil(quota)))) if quota else aff
    prev = torch.get_num_threads()
    tp = {k: torch.from_numpy(v) for k, v in params.items()}
    xi, xv = synth.synth_inputs(sizes, 13, BATCH, seed=99)
    xi, xv = torch.from_numpy(xi), torch.from_numpy(xv)
    torch.set_num_threads(cores)
    out_cpu = torch_port.forward(cfg, tp, xi, xv)
    n, el = _time_port(torch_port, cfg, tp, xi, xv, seconds, cores)
    n1, el1 = _time_port(torch_port, cfg, tp, xi, xv, seconds, 1)
    torch.set_num_threads(prev)
    cpu = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    base = {"value": round(n * BATCH / el, 1), "unit": "samples/s", "cores": cores, "kind": "port",
            "sample": f"{n} batches x {BATCH} rows of the same Criteo-39 workload, {el:.1f} s, "
                      f"torch {torch.__version__} CPU, {cores} threads (affinity mask {aff} cores"
                      + (f", cgroup CPU quota {quota}" if quota else "") + f"), {cpu}",
            "one_thread": {"value": round(n1 * BATCH / el1, 1), "unit": "samples/s", "cores": 1,
                           "sample": f"{n1} batches x {BATCH} rows, {el1:.1f} s"}}
    try:
        cal = json.load(open(os.path.join(REPO, "profiles", "cpu_calibration.json")))
        wl = "deepfwfm_lw" if cfg["use_deep"] else "fwfm_lw"
        ent = [e for e in cal["entries"] if e["workload"] == wl]
        if ent and not cfg.get("qr_flag") and not cfg.get("use_fwlw"):
            base["calibration"] = {
                "what": "port / reference forward time, same batch, measured beside the imported reference in the "
                        "build container (tools/calibrate_cpu_port.py); logits bit-identical",
                "host": cal.get("host"), "entries": [{k: e[k] for k in ("threads", "ref_ms_per_batch",
                                                                       "port_ms_per_batch", "port_over_ref_time")}
                                                    for e in ent]}
    except Exception:
        pass
    parity = None
    if model is not None:
        from xsdeepfwfm_deprecated_amd.metrics import DeviceMetrics
        with torch.no_grad():
            out_gpu = model(xi.to(dev), xv.to(dev))
        ref = out_cpu.detach().to(torch.float64)
        rel = ((out_gpu.cpu().to(torch.float64) - ref).abs() / ref.abs().clamp(min=1.0)).max().item()
        g = torch.Generator().manual_seed(7)
        y = (torch.rand(BATCH, generator=g, dtype=torch.float64) < torch.sigmoid(ref)).to(torch.float32)
        dm = DeviceMetrics(dev)
        auc_gpu = dm(out_gpu, y.to(dev))["auc"]
        auc_cpu = dm(out_cpu.detach().to(torch.float32).to(dev), y.to(dev))["auc"]
        parity = {"rows": BATCH, "max_rel_logit_diff_vs_cpu_port": rel, "auc_gpu": round(auc_gpu, 6),
                  "auc_cpu_port": round(auc_cpu, 6), "abs_auc_diff": abs(auc_gpu - auc_cpu),
                  "bars": "logits 1e-5 * max(1, |ref|), AUC 1e-4 (BASELINE north_star)"}
    return base, parity


if __name__ == "__main__":
    main()
