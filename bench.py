"""Benchmark: Llama-7B per-token quantized MUL_MAT set (Q4_0, batch 1) on MI355X.

BASELINE.json metric: "Q4_0 matmul GB/s + tokens/sec 7B, 1/2/4/8 MI355X vs Kotlin CPU".
Workload (SURVEY §8d, config C4 at N=1): one step = one token of Llama-7B's matmuls,
32 layers x {q, k, v, o: 4096x4096; gate, up: 11008x4096; down: 4096x11008}, Q4_0
weights (llama.kotlin block layout), F32 activations, F32 outputs — 224 computeMatMul
nodes, 3.65 GB of weights (> the 256 MiB Infinity Cache, so every step streams HBM).
Weights are random-init N(0, 0.02^2) quantized on device; activations N(0, 1); synthetic.

Schedule of the timed step ("llama7b_token_matmuls_q4_0_n1_layer_grouped"): the 7 matmuls of a
layer are treated as independent nodes, one grouped launch per layer (MulMatPlan); layer L+1 reads
layer L's outputs (h <- down, attn <- o, h2 <- v, ffn <- up), so consecutive layers are ordered by
data. A real decode also orders matrices inside a layer ({q,k,v} -> o -> {gate,up} -> down): that
schedule is the "decode_chain" line (4 launches per layer), the tokens/s a decoding user sees.
The whole step is captured once in a HIP graph and replayed (no per-launch host overhead).

Multi-GPU (one process per GPU): every weight matrix is row-sharded (rank r owns rows
[r·M/P, (r+1)·M/P)); each layer is one lk_sharded_plan of the C-ABI — the local rows computed in
place inside the full output buffers, then one RCCL group of in-place all-gathers over xGMI — and
the next layer reads the gathered outputs. Total work per step is fixed -> "scaling": "strong".
`--sharded` takes that path at one rank too (start it under `torchrun --nproc-per-node 1`): the
C-ABI communicator is built from a world-1 NCCL process group and each layer is a one-rank
lk_sharded_plan with its RCCL group of in-place gathers, captured in the HIP graph — the exact
code the 8-GPU run executes, measured on one GPU (its value should match the plain line).

Launching N ranks: under torchrun (WORLD_SIZE set) every rank is one process on GPU LOCAL_RANK and
`--gpus`, when given, must equal WORLD_SIZE. Run directly with `--gpus N > 1`, bench.py starts the N
rank processes itself before anything touches a GPU (torchrun's environment per rank, rendezvous on
127.0.0.1), relays rank 0's JSON line and exits with the worst rank's status. It refuses (exit 2) a
`--gpus` that disagrees with WORLD_SIZE or exceeds the visible GPUs (the gloo rehearsal excepted).

Exit status: the JSON line is always printed; the run exits 3 afterwards when any section reports
an error or any bounded in-launch wait gave up (sync_wait_timeouts), so a driver never takes a
partial line for a clean one.

value = whole-job algorithmic GB/s = Σ_nodes (M·K/32·18 + 4·K + 4·M) bytes per token x
tokens / wall time (max over ranks). tokens_per_s is reported beside it.
roofline = the dominant (only) kernel of the step, gemv_stream_kernel<Q4_0,3>: algorithmic
bytes per launch / average launch duration, from HIP events on the launch stream around
graph replays of the 32 layer launches.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "llama.kotlin_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

HIDDEN, FFN, LAYERS = 4096, 11008, 32
# (name, M rows, K) — LlamaConfig defaults, K/model/LlamaModel.kt:8-21; shapes :159-195, :287-304
LAYER_MATS = [("q", HIDDEN, HIDDEN), ("k", HIDDEN, HIDDEN), ("v", HIDDEN, HIDDEN), ("o", HIDDEN, HIDDEN),
              ("gate", FFN, HIDDEN), ("up", FFN, HIDDEN), ("down", HIDDEN, FFN)]
# activation each matrix reads: q,k,v share the normed hidden state, gate/up the second one
X_OF = {"q": "h", "k": "h", "v": "h", "o": "attn", "gate": "h2", "up": "h2", "down": "ffn"}
X_LEN = {"h": HIDDEN, "attn": HIDDEN, "h2": HIDDEN, "ffn": FFN}
# layer L+1 reads these outputs of layer L (the timed step's data edge between layers)
NEXT_X = {"h": "down", "attn": "o", "h2": "v", "ffn": "up"}
CHAIN = [("q", "k", "v"), ("o",), ("gate", "up"), ("down",)]
Q4_0_BLOCK = 18
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def alg_bytes(M, K, N=1):
    return M * K // 32 * Q4_0_BLOCK + 4 * K * N + 4 * M * N


def shard(M, world, rank):
    per = -(-M // world)
    r0 = min(rank * per, M)
    return r0, min(r0 + per, M)


def capture(torch, fn, stream):
    """HIP graph of fn() on `stream`; None when capture is refused (then fn runs eagerly)."""
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, stream=stream):
            fn()
    except Exception as e:  # noqa: BLE001 — reported in the JSON line, eager fallback
        print(f"[bench] graph capture failed ({type(e).__name__}: {e}); timing eager launches", file=sys.stderr)
        torch.cuda.synchronize()
        return None
    return g


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n, argv):
    """Start n rank processes of this script (torchrun's per-rank environment, rendezvous on
    127.0.0.1) before any GPU call in this process; rank 0's stdout is the caller's. Returns the
    worst exit status; when a rank fails the others are stopped (they would wait at a barrier)."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LK_BENCH_SPAWNED="1")
        out = None if r == 0 else subprocess.DEVNULL  # only rank 0 prints the line
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env, stdout=out))
    worst = 0
    while procs:
        for p in list(procs):
            rc = p.poll()
            if rc is None:
                continue
            procs.remove(p)
            if rc != 0:
                worst = worst or rc
                for q in procs:  # a failed rank leaves the others waiting for it
                    q.terminate()
        time.sleep(0.05)
    return worst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE, or 1)")
    ap.add_argument("--check-launch", action="store_true",
                    help="start the ranks, join the process group, report what each rank sees, exit (no GPU work)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--layers", type=int, default=LAYERS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-headline", action="store_true")
    ap.add_argument("--no-chain", action="store_true")
    ap.add_argument("--no-batched", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--no-multi-gpu-cost", action="store_true")
    ap.add_argument("--no-throughput", action="store_true", help="skip the multi_gpu_throughput legs")
    ap.add_argument("--cpu-sample-rows", type=int, default=6144)
    ap.add_argument("--sharded", action="store_true",
                    help="the N > 1 path (C-ABI RCCL communicator + lk_sharded_plan) at any world size")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    # LK_BENCH_BACKEND=gloo (rehearsal only, never a measurement): the N > 1 code path with
    # ranks sharing the visible GPUs and gloo collectives, to exercise it on a one-GPU box
    backend = os.environ.get("LK_BENCH_BACKEND", "nccl")
    if "WORLD_SIZE" not in os.environ:
        n = args.gpus or 1
        # (torch.cuda.device_count() does not initialise the GPU on this image: safe before the fork)
        if n > 1 and backend == "nccl" and not args.check_launch and torch.cuda.device_count() < n:
            print(f"[bench] --gpus {n}: only {torch.cuda.device_count()} GPU(s) visible", file=sys.stderr)
            sys.exit(2)
        if n > 1:
            sys.exit(spawn_ranks(n, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: refusing a line that would misstate n_gpus",
              file=sys.stderr)
        sys.exit(2)
    if args.check_launch:  # launcher check: no GPU work (CPU tests run it with the gloo backend)
        if world > 1:
            dist.init_process_group("gloo")
            seen = dist.get_world_size()
            dist.barrier()
            dist.destroy_process_group()
        else:
            seen = 1
        if rank == 0:
            print(json.dumps({"n_gpus": world, "ranks_seen": seen, "spawned": os.environ.get("LK_BENCH_SPAWNED") == "1",
                              "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}), flush=True)
        return
    if backend == "nccl" and torch.cuda.device_count() < world:
        print(f"[bench] WORLD_SIZE={world} but {torch.cuda.device_count()} GPU(s) visible", file=sys.stderr)
        sys.exit(2)
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = world > 1 or args.sharded
    if distributed:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import ggml_hip as G
    G.load_library()
    T = G.GGMLType

    # ---- device-resident operands -------------------------------------------------------
    for (_, M, _) in LAYER_MATS:
        if M % world:
            raise SystemExit(f"--gpus {world}: every matrix's rows must split evenly (M = {M})")
    gen = torch.Generator(device=dev)
    gen.manual_seed(0x5EED + rank)
    w_bytes = args.layers * sum(((M // world) * K // 32 * Q4_0_BLOCK + 15) // 16 * 16 for (_, M, K) in LAYER_MATS)
    out_per_layer = sum(M for (_, M, _) in LAYER_MATS)  # every rank holds every layer's FULL outputs
    x_per_layer = sum(X_LEN.values())
    ga = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    wbuf = ga.addBuffer(w_bytes + 256)          # this rank's Q4_0 row shards, back to back
    xbuf = ga.addBuffer(4 * x_per_layer + 256)   # layer 0's inputs
    obuf = ga.addBuffer(4 * out_per_layer * args.layers + 256)
    xs = torch.randn(x_per_layer, generator=gen, device=dev)
    ga.buffers[xbuf][: 4 * x_per_layer].copy_(xs.view(torch.uint8))
    woff = 0
    nodes_by_layer = []  # per layer: {name: (a_shard, b, dst_full)}
    local_by_layer = []  # per layer: [(a_shard, b, dst rows of this rank)] — the kernel alone
    prev = None          # previous layer's {name: dst_full}
    for layer in range(args.layers):
        ins, xo = {}, 0
        for key, n in X_LEN.items():  # layer 0 reads xbuf; layer L+1 reads layer L's outputs
            ins[key] = (G.GGMLTensor(T.F32, [1, n], bufferId=xbuf, dataOffset=4 * xo) if prev is None
                        else prev[NEXT_X[key]])
            xo += n
        nodes, outs, ooff = {}, {}, 4 * out_per_layer * layer
        for (name, M, K) in LAYER_MATS:
            rows = M // world
            a = G.GGMLTensor(T.Q4_0, [K, rows], bufferId=wbuf, dataOffset=woff, name=f"L{layer}.{name}")
            nb = rows * K // 32 * Q4_0_BLOCK
            with torch.no_grad():
                src = torch.randn(rows * K, generator=gen, device=dev, dtype=torch.float32) * 0.02
                ga.buffers[wbuf][woff:woff + nb].copy_(G.quantizeTensor(src, T.Q4_0))
                del src
            woff += (nb + 15) // 16 * 16
            d = G.GGMLTensor(T.F32, [1, M], bufferId=obuf, dataOffset=ooff)
            ooff += 4 * M
            nodes[name] = (a, ins[X_OF[name]], d)
            outs[name] = d
        nodes_by_layer.append(nodes)
        local_by_layer.append([(a, b, G.shard_view(d, world, rank)) for (a, b, d) in nodes.values()])
        prev = outs
    # timed schedule: per layer one grouped launch of its 7 matrices (independent within the layer);
    # layer L+1 reads layer L's outputs, so at N > 1 each layer's RCCL all-gather (in the C-ABI,
    # lk_sharded_plan) sits on the path between consecutive layers
    comm = None
    if distributed and backend == "nccl":
        # the C-ABI's RCCL path is the product: if it cannot be set up the run fails (no fallback)
        comm = G.Comm.from_process_group()
        if comm.rcclRanks != world:
            raise SystemExit(f"RCCL communicator holds {comm.rcclRanks} ranks, WORLD_SIZE is {world}")
        plans = [[G.ShardedMulMatPlan(comm, ga, [n[name] for (name, _, _) in LAYER_MATS])] for n in nodes_by_layer]
    elif world > 1:  # LK_BENCH_BACKEND=gloo rehearsal only: local launch + torch.distributed gather
        plans = [[G.MulMatPlan(ga, lp)] for lp in local_by_layer]
    else:
        plans = [[G.MulMatPlan(ga, [n[name] for (name, _, _) in LAYER_MATS])] for n in nodes_by_layer]
    local_plans = [[G.MulMatPlan(ga, lp)] for lp in local_by_layer]
    launches_per_step = sum(p.numLaunches for lp in local_plans for p in lp)
    torch.cuda.synchronize()

    compute = torch.cuda.Stream(device=dev)
    obuf_u8 = ga.buffers[obuf]

    def gloo_gather(layer):
        # the in-place all-gather of lk_sharded_plan, through torch.distributed (gloo rehearsal only)
        for (name, M, _) in LAYER_MATS:
            d = nodes_by_layer[layer][name][2]
            full = obuf_u8[d.dataOffset:d.dataOffset + 4 * M].view(torch.float32)
            chunk = M // world
            parts = list(full.split(chunk))
            dist.all_gather(parts, parts[rank].clone())

    def step():
        for layer, lp in enumerate(plans):
            for plan in lp:
                plan.launch(stream=compute)
            if world > 1 and comm is None:
                gloo_gather(layer)

    with torch.cuda.stream(compute):
        for _ in range(args.warmup):
            step()
    torch.cuda.synchronize()
    graph = None if (args.no_graph or (world > 1 and backend != "nccl")) else capture(torch, step, compute)
    run = graph.replay if graph is not None else step
    with torch.cuda.stream(compute):
        run()  # one untimed replay (graph upload)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    with torch.cuda.stream(compute):
        ev0.record(compute)
        for _ in range(args.steps):
            run()
        ev1.record(compute)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    token_bytes = args.layers * sum(alg_bytes(M, K) for (_, M, K) in LAYER_MATS)
    tokens = args.steps
    value_gbs = token_bytes * tokens / elapsed / 1e9
    ms_per_step = elapsed * 1e3 / args.steps

    roof = roofline(torch, local_plans, local_by_layer, compute, world)

    # the decode figure: the dependent order {q,k,v} -> o -> {gate,up} -> down (4 launches per layer;
    # at N > 1 each a sharded plan with its all-gather), timed on every rank, max over ranks
    decode = None
    if not args.no_chain and not (world > 1 and comm is None):
        try:
            if comm is not None:
                mk = lambda nodes: G.ShardedMulMatPlan(comm, ga, nodes)  # noqa: E731
            else:
                mk = lambda nodes: G.MulMatPlan(ga, nodes)  # noqa: E731
            decode = decode_chain(torch, G, ga, nodes_by_layer, compute, token_bytes, make_plan=mk,
                                  dist=dist if distributed else None, dev=dev)
        except G.HipDeviceError as e:
            decode = {"error": str(e)}

    result = {
        "metric": "Q4_0 matmul GB/s + tokens/sec 7B, 1/2/4/8 MI355X vs Kotlin CPU",
        "value": round(value_gbs, 2),
        "unit": "GB/s",
        # tokens/s of the dependent decode order (decode_chain); the timed grouped step's own rate beside it.
        # Never null: without a decode figure (--no-chain, or the section failed) it falls back
        # to the grouped step's rate, and tokens_per_s_source names which one it is
        "tokens_per_s": (decode["tokens_per_s"] if isinstance(decode, dict) and decode.get("tokens_per_s")
                         else round(tokens / elapsed, 2)),
        "tokens_per_s_source": ("decode_chain" if isinstance(decode, dict) and decode.get("tokens_per_s")
                                else "grouped_step"),
        "tokens_per_s_grouped_step": round(tokens / elapsed, 2),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "q4_0 weights x f32 activations, f32 accumulate",
        "data": "synthetic (random-init N(0,0.02^2) weights quantized on device, N(0,1) activations)",
        "config": {"workload": "llama7b_token_matmuls_q4_0_n1_layer_grouped", "layers": args.layers,
                   "matmuls_per_layer": len(LAYER_MATS), "global_batch": 1, "seq_len": 1,
                   "bytes_per_token": token_bytes,
                   "schedule": "per layer the 7 matrices as independent nodes in one grouped launch; layer L+1 "
                               "reads layer L's outputs (at N > 1 after the in-place RCCL all-gather); the "
                               "intra-layer dependent decode schedule is decode_chain",
                   "parallelism": (f"row-shard{world}+{'rccl-c-abi' if comm is not None else 'torch-' + backend}-allgather"
                                   if distributed else "single"),
                   "launches_per_step_per_rank": launches_per_step, "hip_graph": graph is not None,
                   "ranks_seen_by_rccl": comm.rcclRanks if comm is not None else None,
                   "gpu_ms_per_step": round(ev_ms / args.steps, 4)},
        "roofline": roof,
    }

    # the failure contract: a bounded in-launch wait that gave up is counted per
    # section and reported here (lk_sync_timeouts also clears the flag the next synchronous entry
    # point would raise on), so a section's result is never silently wrong and never blamed on
    # the next section
    waits = {"main": G.syncTimeouts()} if world == 1 else {}

    def section(key, fn):
        # a section whose synchronous call raised on a wait that gave up (LK_ERR_DEVICE) reports
        # the error in its place instead of ending the run; the main line above has no such waits
        try:
            result[key] = fn()
        except G.HipDeviceError as e:
            result[key] = {"error": str(e)}
        waits[key] = G.syncTimeouts()

    if decode is not None:
        result["decode_chain"] = decode
    if rank == 0 and world == 1 and not args.no_chain:
        section("persistent_chain", lambda: {
            "layer_stages": persistent_chain(torch, G, ga, nodes_by_layer, compute, token_bytes, 1),
            "decode_stages": persistent_chain(torch, G, ga, nodes_by_layer, compute, token_bytes, 4)})
    if not args.no_throughput and (comm is not None or world == 1):
        # every rank takes part (the legs' sharded plans gather over the world); world 1 without
        # --sharded uses a one-rank communicator: the same code path
        tcomm = comm if comm is not None else G.Comm.single()
        section("multi_gpu_throughput", lambda: multi_gpu_throughput(torch, G, dev, tcomm, world, rank,
                                                                      dist if distributed else None))
        if comm is None:
            tcomm.close()
    if rank == 0 and world == 1 and not args.no_headline:
        section("headline_q4_0_4096x4096_n1", lambda: headline(torch, G, dev))
    if rank == 0 and world == 1 and not args.no_batched:
        section("n1_configs", lambda: n1_configs(torch, G, dev))
        section("batched", lambda: batched(torch, G, dev))
        section("next_rows", lambda: next_rows(torch, G, dev))
    if rank == 0 and world == 1 and not args.no_multi_gpu_cost:
        section("multi_gpu_world1", lambda: multi_gpu_world1(torch, G, ga, nodes_by_layer, compute))
    if rank == 0 and world == 1 and not args.no_host_path:
        section("host_path_pcie", lambda: host_path(torch, G, dev))
    if waits:
        result["sync_wait_timeouts"] = waits
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.cpu_sample_rows, token_bytes)
    failed = [k for k, v in result.items() if isinstance(v, dict) and "error" in v]
    failed += [f"sync_wait_timeouts.{k}" for k, v in waits.items() if v]
    if failed:
        result["failed_sections"] = failed
    if rank == 0:
        print(json.dumps(result), flush=True)
    if distributed:
        dist.barrier()
        for lp in plans:
            for p in lp:
                p.close()
        if comm is not None:
            comm.close()
        dist.destroy_process_group()
    if failed:
        print(f"[bench] failed sections: {failed}", file=sys.stderr)
        sys.exit(3)


def roofline(torch, plans, local_by_layer, stream, world, reps=10):
    """Dominant kernel: the grouped launch of each layer (all 7 matrices, gemv_stream_kernel<Q4_0,3>).
    A HIP graph of the 32 layer launches (distinct weights per layer, so each launch streams HBM)
    is replayed `reps` times between two events on the launch stream; the mean launch duration is
    that time / launches. It includes the gaps between launches inside the graph, and it is measured
    un-profiled; rocprof's mean kernel duration for the same launch (profiles/rNN, a profiled run,
    which lowers the clock) is the other figure DESIGN.md reports beside it — the two differ by a few
    percent either way. achieved = algorithmic bytes per launch / mean duration."""
    def layers():
        for lp in plans:
            lp[0].launch(stream=stream)

    g = capture(torch, layers, stream)
    run = g.replay if g is not None else layers
    with torch.cuda.stream(stream):
        run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            run()
        e1.record(stream)
    torch.cuda.synchronize()
    n = reps * len(plans)
    avg_s = e0.elapsed_time(e1) / 1e3 / n
    nbytes = sum(a.ne[1] * a.ne[0] // 32 * Q4_0_BLOCK + 4 * a.ne[0] + 4 * a.ne[1] for (a, _, _) in local_by_layer[0])
    achieved = nbytes / avg_s / 1e9
    # the committed profile is of the N = 1 layer launch; a row shard is a different launch
    prof, src = pmc_traffic("gemv_stream_kernel<2, 3>") if world == 1 else (None, None)
    out = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": prof["hbm_bytes_per_launch"] if prof else None,
           "traffic_source": src,
           "kernel": "gemv_stream_kernel<Q4_0,3> (the 7 matrices of one layer in one launch)",
           "bytes_per_launch": nbytes, "avg_launch_us": round(avg_s * 1e6, 3), "launches_timed": n,
           "hip_graph": g is not None}
    if prof and prof.get("mean_us"):
        # beside the event figure: the same launch's mean kernel duration in the committed rocprof
        # kernel trace (a profiled run: lower clock, no inter-launch gaps)
        out["rocprof_mean_us"] = prof["mean_us"]
        out["rocprof_frac"] = round(nbytes / (prof["mean_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    return out


def pmc_traffic(kernel):
    """The newest committed profile of `kernel` in this bench (profiles/rNN/traffic.json, written
    by tools/prof_summary.py from tools/profile.sh's runs): HBM bytes per launch (FETCH_SIZE x 2 +
    WRITE_SIZE, separate --pmc passes) and the kernel trace's mean duration; (None, None) when absent."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")), reverse=True):
        with open(f) as fh:
            t = json.load(fh)
        if kernel in t.get("kernel", ""):
            return t, os.path.relpath(f, ROOT)
    return None, None


def decode_chain(torch, G, ga, nodes_by_layer, stream, token_bytes, reps=20, make_plan=None, dist=None, dev=None):
    """Dependent decode schedule: per layer {q,k,v} -> o -> {gate,up} -> down, 4 stream-ordered
    launches (128 per token), captured in a HIP graph. make_plan builds one group's plan (N = 1: a
    MulMatPlan; N > 1: a ShardedMulMatPlan, its in-place all-gather after the launch). With dist,
    every rank times the token and the max over ranks is reported."""
    if make_plan is None:
        make_plan = lambda nodes: G.MulMatPlan(ga, nodes)  # noqa: E731
    plans = [[make_plan([n[k] for k in grp]) for grp in CHAIN] for n in nodes_by_layer]

    def token():
        for lp in plans:
            for p in lp:
                p.launch(stream=stream)

    with torch.cuda.stream(stream):
        token()
    torch.cuda.synchronize()
    g = capture(torch, token, stream)
    run = g.replay if g is not None else token
    with torch.cuda.stream(stream):
        run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            run()
        e1.record(stream)
    torch.cuda.synchronize()
    per = e0.elapsed_time(e1) / 1e3 / reps
    if dist is not None:
        t = torch.tensor([per], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        per = float(t.item())
    for lp in plans:
        for p in lp:
            p.close()
    return {"tokens_per_s": round(1 / per, 2), "ms_per_token": round(per * 1e3, 4),
            "achieved_GBps": round(token_bytes / per / 1e9, 1), "launches_per_token": 4 * len(plans),
            "hip_graph": g is not None, "tokens_timed": reps,
            "schedule": "{q,k,v} -> o -> {gate,up} -> down per layer" + (", each group a row-sharded plan + RCCL all-gather"
                                                                        if dist is not None else "")}


def persistent_chain(torch, G, ga, nodes_by_layer, stream, token_bytes, per_layer, reps=20):
    """The same token as ONE persistent launch (lk_plan_create_chain): per_layer groups of
    dependent stages per layer (1: the 7 matrices of a layer as one stage, 32 stages; 4: the
    decode schedule {q,k,v} -> o -> {gate,up} -> down, 128 stages), a device-side grid barrier
    (agent-scope release / acquire) between consecutive stages, the next stage's weights
    streaming while it completes. Captured in a HIP graph."""
    groups = [tuple(n for (n, _, _) in LAYER_MATS)] if per_layer == 1 else CHAIN
    nodes, stages = [], []
    for layer, n in enumerate(nodes_by_layer):
        for gi, grp in enumerate(groups):
            for k in grp:
                nodes.append(n[k])
                stages.append(layer * len(groups) + gi)
    plan = G.MulMatPlan(ga, nodes, stages=stages)

    def token():
        plan.launch(stream=stream)

    with torch.cuda.stream(stream):
        token()
    torch.cuda.synchronize()
    g = capture(torch, token, stream)
    run = g.replay if g is not None else token
    with torch.cuda.stream(stream):
        run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            run()
        e1.record(stream)
    torch.cuda.synchronize()
    per = e0.elapsed_time(e1) / 1e3 / reps
    timed_out = plan.timedOut()
    return {"tokens_per_s": round(1 / per, 2), "ms_per_token": round(per * 1e3, 4),
            "achieved_GBps": round(token_bytes / per / 1e9, 1), "stages_per_token": len(groups) * len(nodes_by_layer),
            "launches_per_token": 1, "hip_graph": g is not None, "tokens_timed": reps, "barrier_timeout": timed_out}


def multi_gpu_world1(torch, G, ga, nodes_by_layer, stream, reps=5):
    """The per-layer cost of the two multi-GPU exchange designs at world size 1, eager
    (the one-shot path cannot be captured): the token's 32 layer launches enqueued behind a sleep
    kernel (so the host's enqueue rate does not show), timed between events after it, as
      plain      lk_plan per layer (no exchange);
      rccl       lk_sharded_plan per layer: the launch + one RCCL group of 7 in-place all-gathers;
      one_shot   lk_p2p_plan per layer: hipStreamWaitValue64 gate on the previous layer's signal,
                 the launch, the push kernel (no copies at world 1, only the signal).
    The differences to plain are each design's fixed per-layer cost on one GPU; xGMI transfer time
    comes on top at P > 1 (DESIGN §6b's budget)."""
    names = [n for (n, _, _) in LAYER_MATS]
    plain = [G.MulMatPlan(ga, [n[k] for k in names]) for n in nodes_by_layer]
    comm = G.Comm.single()
    rccl = [G.ShardedMulMatPlan(comm, ga, [(G.shard_view(n[k][0], 1, 0), n[k][1], n[k][2]) for k in names])
            for n in nodes_by_layer]
    group = G.P2PGroup([torch.cuda.current_device()])
    p2p = [G.P2PMulMatPlan(group, ga, [[(G.shard_view(n[k][0], 1, 0), n[k][1], n[k][2]) for k in names]])
           for n in nodes_by_layer]
    out = {}
    for key, plans, launch in (("plain", plain, lambda p: p.launch(stream=stream)),
                               ("rccl", rccl, lambda p: p.launch(stream=stream)),
                               ("one_shot", p2p, lambda p: p.launch(stream))):
        for p in plans:  # warm
            launch(p)
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                torch.cuda._sleep(20_000_000)  # ~10 ms: the host enqueues the token meanwhile
                e0.record(stream)
                for p in plans:
                    launch(p)
                e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / len(plans))
        out[key + "_us_per_layer"] = round(sorted(ts)[len(ts) // 2], 3)
    out["rccl_cost_us_per_layer"] = round(out["rccl_us_per_layer"] - out["plain_us_per_layer"], 3)
    out["one_shot_cost_us_per_layer"] = round(out["one_shot_us_per_layer"] - out["plain_us_per_layer"], 3)
    out["one_shot_signals_ok"] = all(p.signal(0) == p.numLaunches for p in p2p)
    for p in p2p + rccl:
        p.close()
    group.close(); comm.close()
    return out


# ---- the north star's "4096x4096xbatch throughput at 1/2/4/8 GPUs"  ----------------
# Every leg is a set of independent MUL_MAT calls on distinct weights, each call row-sharded over the
# world through lk_sharded_plan (local rows + one RCCL group of in-place all-gathers, the exact code the
# decode path uses), at every world size — world 1 included (a one-rank communicator). Total work per
# call is fixed, so the driver's 1 -> 8 runs read a strong-scaling curve per leg.
THROUGHPUT_LEGS = [
    # (name, node shapes (M, K) of one call, batch N)
    ("q4_0_4096x4096_n1", [(4096, 4096)], 1),
    ("q4_0_4096x4096_n32", [(4096, 4096)], 32),
    ("q4_0_4096x4096_n512", [(4096, 4096)], 512),
    ("llama7b_layer_q4_0_n32", [(M, K) for (_, M, K) in LAYER_MATS], 32),
]
MFMA_PEAK_TFS = 2500.0  # dense bf16 MFMA peak (MI355X_MICROARCH.md); the batched kernels run bf16 hi/lo MFMAs


def leg_geometry(shapes, N, world, min_rank_bytes=300e6):
    """Per-call quantities of a throughput leg at `world` ranks and how many distinct weight copies a
    timed pass rotates over, so that each rank streams >= min_rank_bytes of distinct weights per pass
    (more than the 256 MiB Infinity Cache at every world size: the weights come from HBM)."""
    for (M, _) in shapes:
        if M % world:
            raise ValueError(f"M = {M} does not split over {world} ranks")
    w_full = sum(M * K // 32 * Q4_0_BLOCK for (M, K) in shapes)
    copies = max(2, -(-int(min_rank_bytes) // max(1, w_full // world)))
    out_bytes = sum(4 * N * M for (M, _) in shapes)
    return {"copies": copies,
            "alg_bytes_per_call": sum(alg_bytes(M, K, N) for (M, K) in shapes),
            "useful_flop_per_call": sum(2 * M * N * K for (M, K) in shapes),
            "rank_alg_bytes_per_call": sum(alg_bytes(M // world, K, N) for (M, K) in shapes),
            "rank_flop_per_call": sum(2 * (M // world) * N * K for (M, K) in shapes),
            "gather_bytes_in_per_rank": out_bytes * (world - 1) // world,
            "output_bytes_per_call": out_bytes}


def throughput_leg(torch, G, dev, comm, world, rank, dist, name, shapes, N, reps=5, keep=None, min_rank_bytes=300e6):
    """One leg: `copies` calls of `shapes` at batch N (synthetic Q4_0 weights: every rank quantizes the
    same full matrices and keeps its row shard, so the gathered outputs are the single-GPU results),
    timed three ways on every rank, max over ranks:
      local     the rank's rows only (its lk_plan per call): per-rank kernel time and roofline;
      serial    lk_sharded_plan_launch per call: rows, then the RCCL group, one stream;
      overlap   lk_sharded_plan_launch_split per call: the gathers on a second stream, so call i's
                exchange overlaps call i+1's rows (the throughput schedule).
    Check (no oracle in bench.py): rank 0's gathered output of the first call against float64 dot
    products of dequantizeTensor's weights (bit-exact with the reference, tests/test_gpu_parity.py) on
    rows sampled from every rank's shard, and the same output's checksum equal on every rank."""
    T = G.GGMLType
    geo = leg_geometry(shapes, N, world, min_rank_bytes)
    copies = geo["copies"]
    K0 = shapes[0][1]
    ga = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    gen = torch.Generator(device=dev)
    gen.manual_seed(0xC0FFEE)  # the same full matrices and activations on every rank
    xs = {K: ga.addBuffer(4 * K * N + 256) for K in {k for (_, k) in shapes}}
    for K, xb in xs.items():
        ga.buffers[xb][: 4 * K * N].copy_(torch.randn(K * N, generator=gen, device=dev).view(torch.uint8))
    shard_q, full_q = [], []
    for (M, K) in shapes:
        q = G.quantizeTensor(torch.randn(M * K, generator=gen, device=dev) * 0.02, T.Q4_0)
        rb = K // 32 * Q4_0_BLOCK
        per = M // world
        full_q.append(q if len(full_q) == 0 else None)  # only the first node is checked
        shard_q.append(q[rank * per * rb:(rank + 1) * per * rb].clone())
    pitch = [(b.numel() + 255) // 256 * 256 for b in shard_q]
    wb = ga.addBuffer(copies * sum(pitch) + 256)
    db = ga.addBuffer(copies * geo["output_bytes_per_call"] + 256 * copies * len(shapes) + 256)
    sharded, local, dsts, woff, doff = [], [], [], 0, 0
    for c in range(copies):
        nodes = []
        for i, (M, K) in enumerate(shapes):
            ga.buffers[wb][woff:woff + shard_q[i].numel()].copy_(shard_q[i])
            a = G.GGMLTensor(T.Q4_0, [K, M // world], bufferId=wb, dataOffset=woff)
            d = G.GGMLTensor(T.F32, [N, M], bufferId=db, dataOffset=doff)
            nodes.append((a, G.GGMLTensor(T.F32, [N, K], bufferId=xs[K]), d))
            woff += pitch[i]
            doff += (4 * N * M + 255) // 256 * 256
        sharded.append(G.ShardedMulMatPlan(comm, ga, nodes))
        local.append(G.MulMatPlan(ga, [(a, b, G.shard_view(d, world, rank)) for (a, b, d) in nodes]))
        dsts.append([d for (_, _, d) in nodes])
    del shard_q
    compute, gather = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()

    def run_local():
        for p in local:
            p.launch(stream=compute)

    def run_serial():
        for p in sharded:
            p.launch(stream=compute)

    def run_overlap():
        for p in sharded:
            p.launchSplit(compute, gather)
        compute.wait_stream(gather)

    out = {"N": N, "nodes_per_call": len(shapes), "shapes": [list(s) for s in shapes], "weights": "Q4_0", **geo,
           "ranks_seen_by_rccl": comm.rcclRanks}
    for key, fn in (("local", run_local), ("serial", run_serial), ("overlap", run_overlap)):
        per, graphed = _graph_time(torch, fn, compute, reps)
        if dist is not None:
            t = torch.tensor([per], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            per = float(t.item())
        per /= copies
        if key == "local":
            r = {"us_per_call": round(per * 1e6, 3), "rank_GBps": round(geo["rank_alg_bytes_per_call"] / per / 1e9, 1),
                 "rank_frac_hbm": round(geo["rank_alg_bytes_per_call"] / per / 1e9 / HBM_PEAK_GBS, 4)}
            if N > 1:
                r["rank_useful_TFLOPs"] = round(geo["rank_flop_per_call"] / per / 1e12, 2)
                r["rank_frac_mfma_bf16"] = round(2 * geo["rank_flop_per_call"] / per / 1e12 / MFMA_PEAK_TFS, 4)  # hi + lo
        else:
            r = {"us_per_call": round(per * 1e6, 3), "GBps": round(geo["alg_bytes_per_call"] / per / 1e9, 1),
                 "calls_per_s": round(1 / per, 1)}
            if N > 1:
                r["useful_TFLOPs"] = round(geo["useful_flop_per_call"] / per / 1e12, 2)
        r["hip_graph"] = graphed
        out[key] = r
    best = min(out["serial"]["us_per_call"], out["overlap"]["us_per_call"])
    out["value_GBps"] = round(geo["alg_bytes_per_call"] / (best * 1e-6) / 1e9, 1)
    if N > 1:
        out["value_useful_TFLOPs"] = round(geo["useful_flop_per_call"] / (best * 1e-6) / 1e12, 2)
    # check: the first call's first node, gathered, on every rank
    torch.cuda.synchronize()
    M, K = shapes[0]
    d0 = dsts[0][0]
    got = ga.buffers[db][d0.dataOffset:d0.dataOffset + 4 * N * M].view(torch.float32).view(M, N)
    csum = torch.tensor([float(got.double().sum())], dtype=torch.float64, device=dev)
    same = True
    if dist is not None:
        lo, hi = csum.clone(), csum.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        same = bool(lo.item() == hi.item())
    rows = sorted({int(v) for v in torch.linspace(0, M - 1, 64).tolist()})
    wq = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    qb = wq.addBuffer(full_q[0].numel() + 256)
    wq.buffers[qb][: full_q[0].numel()].copy_(full_q[0])
    wf = G.dequantizeTensor(wq, G.GGMLTensor(T.Q4_0, [K, M], bufferId=qb)).view(M, K)[rows].double()
    xk = ga.buffers[xs[K]][: 4 * K * N].view(torch.float32).view(K, N).double()
    ref = wf @ xk
    err = (got[rows].double() - ref).abs()
    scale = ref.abs().max().clamp_min(1e-30)
    # the §8c bar of tests/_util.py parity_ok: 1e-3 of max(|r|, 1e-3·‖r‖∞), or the f32 accumulation
    # noise 4·√K·2⁻²⁴·Σ|w||x| (+ 2⁻¹⁷·Σ|w||x| for the batched path's bf16 hi/lo activation split)
    noise = (4.0 * K ** 0.5 * 2.0 ** -24 + (2.0 ** -17 if N > 1 else 0.0)) * (wf.abs() @ xk.abs())
    allow = torch.maximum(1e-3 * torch.maximum(ref.abs(), 1e-3 * scale), noise)
    rel = max(float((err / allow).max()) * 1e-3, float(err.max() / scale))  # <= 1e-3 passes
    if keep is not None:  # tests: the first call's operands and gathered output, on the host
        keep.update(q=full_q[0].cpu().numpy(), x=xk.float().cpu().numpy(), got=got.cpu().numpy().copy(), M=M, K=K)
    out["check"] = {"rows_checked": len(rows), "err_vs_bar": rel, "bar": 1e-3, "ok": bool(rel <= 1e-3) and same,
                    "checksum_equal_on_every_rank": same,
                    "against": "float64 dot products of dequantizeTensor's weights, rows sampled from every shard"}
    for p in sharded + local:
        p.close()
    del ga, wq
    return out


def multi_gpu_throughput(torch, G, dev, comm, world, rank, dist, legs=None):
    """Every THROUGHPUT_LEGS leg at this world size (see throughput_leg)."""
    out = {"world": world, "scaling": "strong (total work per call fixed; ranks split every matrix's rows)",
           "exchange": "in-place RCCL all-gather of each call's outputs (lk_sharded_plan)"}
    for (name, shapes, N) in (legs or THROUGHPUT_LEGS):
        try:
            out[name] = throughput_leg(torch, G, dev, comm, world, rank, dist, name, shapes, N)
        except G.HipDeviceError as e:
            out[name] = {"error": str(e)}
    return out


def headline(torch, G, dev, copies=48, reps=20):
    """North-star shape: Q4_0 4096x4096, N=1, rotating over `copies` distinct weight matrices
    (48 x 9.4 MB = 453 MB > 256 MiB Infinity Cache). Two numbers: one computeMatMul launch per
    matrix (graph-replayed, so launch-bound by the kernel itself, not the host), and the 48
    matrices as one grouped launch (MulMatPlan)."""
    T = G.GGMLType
    M = K = 4096
    nb = M * K // 32 * Q4_0_BLOCK
    g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    wb = g.addBuffer(copies * nb + 256)
    xb = g.addBuffer(4 * K + 256)
    db = g.addBuffer(4 * M * copies + 256)
    src = torch.randn(M * K, device=dev) * 0.02
    for c in range(copies):
        g.buffers[wb][c * nb:(c + 1) * nb].copy_(G.quantizeTensor(src * (1 + 0.01 * c), T.Q4_0))
    g.buffers[xb][: 4 * K].copy_(torch.randn(K, device=dev).view(torch.uint8))
    nodes = [(G.GGMLTensor(T.Q4_0, [K, M], bufferId=wb, dataOffset=c * nb), G.GGMLTensor(T.F32, [1, K], bufferId=xb),
              G.GGMLTensor(T.F32, [1, M], bufferId=db, dataOffset=4 * M * c)) for c in range(copies)]
    s = torch.cuda.Stream(device=dev)

    def singles():
        for (a, b, d) in nodes:
            G.computeMatMul(g, None, a, b, d, stream=s)

    plan = G.MulMatPlan(g, nodes)

    def timed(fn, n_launch):
        with torch.cuda.stream(s):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(reps):
                fn()
            e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 1e3 / (reps * n_launch)

    with torch.cuda.stream(s):
        singles()
    torch.cuda.synchronize()
    gr = capture(torch, singles, s)
    per = timed(gr.replay if gr is not None else singles, copies)
    per_grouped = timed(lambda: plan.launch(stream=s), 1)
    gbs = alg_bytes(M, K) / per / 1e9
    gbs_g = copies * alg_bytes(M, K) / per_grouped / 1e9
    return {"launches": reps * copies, "avg_launch_us": round(per * 1e6, 3), "achieved_GBps": round(gbs, 1),
            "frac_of_8TBps": round(gbs / HBM_PEAK_GBS, 4), "hip_graph": gr is not None,
            "rotating_weight_copies": copies,
            "grouped_48_in_one_launch": {"avg_launch_us": round(per_grouped * 1e6, 3), "achieved_GBps": round(gbs_g, 1),
                                         "frac_of_8TBps": round(gbs_g / HBM_PEAK_GBS, 4)}}


BLOCK_BYTES = {"Q4_0": 18, "Q4_1": 20, "Q8_0": 34}


def n1_configs(torch, G, dev, reps=20):
    """BASELINE.json configs at batch 1 beside the headline: C2 (Q8_0 4096x4096) and C3's FFN
    shapes (Q4_0 / Q4_1 11008x4096 and 4096x11008), one computeMatMul launch per matrix over
    rotating weight copies (> Infinity Cache), graph-replayed; algorithmic GB/s."""
    T = G.GGMLType
    out = {}
    for name, qn, M, K, copies in (("c2_q8_0_4096x4096_n1", "Q8_0", 4096, 4096, 32),
                                   ("c3_q4_0_11008x4096_n1", "Q4_0", 11008, 4096, 16),
                                   ("c3_q4_1_11008x4096_n1", "Q4_1", 11008, 4096, 16),
                                   ("c3_q4_0_4096x11008_n1", "Q4_0", 4096, 11008, 16)):
        qt = getattr(T, qn)
        nb = M * K // 32 * BLOCK_BYTES[qn]
        nb16 = (nb + 15) // 16 * 16
        g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
        wb = g.addBuffer(copies * nb16 + 256)
        xb = g.addBuffer(4 * K + 256)
        db = g.addBuffer(4 * M * copies + 256)
        src = torch.randn(M * K, device=dev) * 0.02
        for c in range(copies):
            g.buffers[wb][c * nb16:c * nb16 + nb].copy_(G.quantizeTensor(src * (1 + 0.01 * c), qt))
        g.buffers[xb][: 4 * K].copy_(torch.randn(K, device=dev).view(torch.uint8))
        nodes = [(G.GGMLTensor(qt, [K, M], bufferId=wb, dataOffset=c * nb16), G.GGMLTensor(T.F32, [1, K], bufferId=xb),
                  G.GGMLTensor(T.F32, [1, M], bufferId=db, dataOffset=4 * M * c)) for c in range(copies)]
        s = torch.cuda.Stream(device=dev)

        def run_all():
            for (a, b, d) in nodes:
                G.computeMatMul(g, None, a, b, d, stream=s)

        with torch.cuda.stream(s):
            run_all()
        torch.cuda.synchronize()
        gr = capture(torch, run_all, s)
        fn = gr.replay if gr is not None else run_all
        with torch.cuda.stream(s):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(reps):
                fn()
            e1.record(s)
        torch.cuda.synchronize()
        per = e0.elapsed_time(e1) / 1e3 / (reps * copies)
        nbytes = nb + 4 * K + 4 * M
        out[name] = {"avg_launch_us": round(per * 1e6, 3), "achieved_GBps": round(nbytes / per / 1e9, 1),
                     "frac_of_8TBps": round(nbytes / per / 1e9 / HBM_PEAK_GBS, 4), "bytes_per_launch": nbytes,
                     "rotating_weight_copies": copies, "hip_graph": gr is not None}
        del g
    return out


KQ_BLOCK = {"Q2_K": (84, 80, "f16"), "Q4_K": (144, 0, "f16"), "Q8_K": (292, 0, "f32")}  # bytes, scale offset


def _graph_time(torch, fn, s, reps):
    """Mean seconds per call of `fn` (stream-ordered launches on `s`), graph-replayed."""
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    gr = capture(torch, fn, s)
    run = gr.replay if gr is not None else fn
    with torch.cuda.stream(s):
        run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            run()
        e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps, gr is not None


def _kquant_kernel(qn, M, K, N):
    """The kernel launch_kquant (csrc/lk_hip.hip) picks for these dense, 256-B aligned operands."""
    if N == 1:
        stream = (qn == "Q4_K" or (qn == "Q2_K" and (M <= 2048 or M >= 6144) and (K // 64 * 21) % 16 == 0))
        return f"gemv_stream_kernel<{qn}> (LDS-DMA stream)" if stream and K <= 12288 else "kquant_n1_kernel"
    if qn == "Q4_K" and 16 <= N <= 32:
        return "gemm_sk_kernel<Q4_K> (wave-pair MFMA; activation split and split-K reduction in the kernel)"
    return "kquant_nc_kernel"


def next_rows(torch, G, dev, reps=20):
    """The SURVEY §8f rows beside the hot path, each at batch 1 on BASELINE shapes, one launch per
    matrix over rotating copies (> Infinity Cache), graph-replayed, algorithmic GB/s:
    K-quant dots (Q2_K / Q4_K / Q8_K x F32; Q4_K on the stream kernel; synthetic super-blocks: random
    code bytes, scale fields set to 0.01) and the device dequantizeTensor / quantizeTensor of a
    Q4_0 11008x4096 matrix (bytes = blocks in + f32 out, or f32 in + blocks out)."""
    T = G.GGMLType
    out = {}
    for name, qn, M, K, N, copies in (("q2_k_4096x4096_n1", "Q2_K", 4096, 4096, 1, 32),
                                      ("q4_k_4096x4096_n1", "Q4_K", 4096, 4096, 1, 32),
                                      ("q8_k_4096x4096_n1", "Q8_K", 4096, 4096, 1, 16),
                                      ("q4_k_11008x4096_n1", "Q4_K", 11008, 4096, 1, 16),
                                      ("q4_k_11008x4096_n32", "Q4_K", 11008, 4096, 32, 16)):
        bb, so, kind = KQ_BLOCK[qn]
        nblk = M * K // 256
        nb = nblk * bb
        g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
        wb, xb, db = g.addBuffer(copies * nb + 256), g.addBuffer(4 * K * N + 256), g.addBuffer(4 * M * N * copies + 256)
        w = g.buffers[wb][: copies * nb].view(copies * nblk, bb)
        w.copy_(torch.randint(0, 256, w.shape, dtype=torch.uint8, device=dev))
        if kind == "f16":
            w[:, so:so + 4].copy_(torch.tensor([0.01, 0.001], dtype=torch.float16).view(torch.uint8).to(dev))
        else:
            w[:, so:so + 4].copy_(torch.tensor([0.01], dtype=torch.float32).view(torch.uint8).to(dev))
        g.buffers[xb][: 4 * K * N].copy_(torch.randn(K * N, device=dev).view(torch.uint8))
        qt = getattr(T, qn)
        nodes = [(G.GGMLTensor(qt, [K, M], bufferId=wb, dataOffset=c * nb), G.GGMLTensor(T.F32, [N, K], bufferId=xb),
                  G.GGMLTensor(T.F32, [N, M], bufferId=db, dataOffset=4 * M * N * c)) for c in range(copies)]
        s = torch.cuda.Stream(device=dev)

        def run_all():
            for (a, b, d) in nodes:
                G.computeMatMul(g, None, a, b, d, stream=s)

        per, graphed = _graph_time(torch, run_all, s, reps)
        per /= copies
        nbytes = nb + 4 * K * N + 4 * M * N
        out[name] = {"avg_launch_us": round(per * 1e6, 3), "achieved_GBps": round(nbytes / per / 1e9, 1),
                     "frac_of_8TBps": round(nbytes / per / 1e9 / HBM_PEAK_GBS, 4), "bytes_per_launch": nbytes,
                     "kernel": _kquant_kernel(qn, M, K, N),
                     "rotating_weight_copies": copies, "hip_graph": graphed}
        del g
    # format kernels: dequantize / quantize of a Q4_0 11008 x 4096 matrix
    M, K, copies = 11008, 4096, 8
    n = M * K
    nb = n // 32 * BLOCK_BYTES["Q4_0"]
    g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    wb = g.addBuffer(copies * nb + 256)
    src = [torch.randn(n, device=dev) * 0.02 for _ in range(copies)]
    for c in range(copies):
        g.buffers[wb][c * nb:(c + 1) * nb].copy_(G.quantizeTensor(src[c], T.Q4_0))
    ts = [G.GGMLTensor(T.Q4_0, [K, M], bufferId=wb, dataOffset=c * nb) for c in range(copies)]
    s = torch.cuda.Stream(device=dev)
    for name, fn, nbytes in (("dequantize_q4_0_11008x4096", lambda: [G.dequantizeTensor(g, t, stream=s) for t in ts], nb + 4 * n),
                             ("quantize_q4_0_11008x4096", lambda: [G.quantizeTensor(x, T.Q4_0, stream=s) for x in src], 4 * n + nb)):
        per, graphed = _graph_time(torch, fn, s, reps)
        per /= copies
        out[name] = {"avg_launch_us": round(per * 1e6, 3), "achieved_GBps": round(nbytes / per / 1e9, 1),
                     "frac_of_8TBps": round(nbytes / per / 1e9 / HBM_PEAK_GBS, 4), "bytes_per_launch": nbytes,
                     "rotating_copies": copies, "hip_graph": graphed}
    del g
    out.update(q4_k_layers(torch, G, dev, reps))
    return out


def q4_k_layers(torch, G, dev, reps=20, layers=8):
    """A Llama-7B layer with Q4_K weights at batch 1 on the stream kernel: the 7 matrices as one
    grouped launch (MulMatPlan, as `value`'s Q4_0 layer launch) and in the dependent decode order
    (4 launches per layer, as decode_chain), over `layers` distinct layers (> Infinity Cache),
    graph-replayed. Synthetic super-blocks as above; each matrix reads a fixed activation vector."""
    T = G.GGMLType
    g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    xs = {}
    for kind, n in X_LEN.items():
        xs[kind] = G.GGMLTensor(T.F32, [1, n], bufferId=g.addBuffer(4 * n + 256))
        g.buffers[xs[kind].bufferId][: 4 * n].copy_(torch.randn(n, device=dev).view(torch.uint8))
    nodes_by_layer, wbytes = [], 0
    for _ in range(layers):
        n = {}
        for (name, M, K) in LAYER_MATS:
            nblk = M * K // 256
            wb = g.addBuffer(nblk * 144 + 256)
            w = g.buffers[wb][: nblk * 144].view(nblk, 144)
            w.copy_(torch.randint(0, 256, w.shape, dtype=torch.uint8, device=dev))
            w[:, 0:4].copy_(torch.tensor([0.01, 0.001], dtype=torch.float16).view(torch.uint8).to(dev))
            d = G.GGMLTensor(T.F32, [1, M], bufferId=g.addBuffer(4 * M + 256))
            n[name] = (G.GGMLTensor(T.Q4_K, [K, M], bufferId=wb), xs[X_OF[name]], d)
            wbytes += nblk * 144 + 4 * K + 4 * M
        nodes_by_layer.append(n)
    per_layer_bytes = wbytes / layers
    s = torch.cuda.Stream(device=dev)
    out = {}
    for name, groups in (("q4_k_layer_grouped_n1", [tuple(m for (m, _, _) in LAYER_MATS)]), ("q4_k_layer_decode_chain_n1", CHAIN)):
        plans = [[G.MulMatPlan(g, [n[k] for k in grp]) for grp in groups] for n in nodes_by_layer]

        def run_all():
            for lp in plans:
                for p in lp:
                    p.launch(stream=s)

        per, graphed = _graph_time(torch, run_all, s, reps)
        per /= layers
        out[name] = {"avg_layer_us": round(per * 1e6, 3), "launches_per_layer": len(groups),
                     "achieved_GBps": round(per_layer_bytes / per / 1e9, 1),
                     "frac_of_8TBps": round(per_layer_bytes / per / 1e9 / HBM_PEAK_GBS, 4),
                     "tokens_per_s_32_layers": round(1.0 / (32 * per), 1), "bytes_per_layer": int(per_layer_bytes),
                     "kernel": "gemv_stream_kernel<Q4_K>", "distinct_layers": layers, "hip_graph": graphed}
    del g
    return out


def batched(torch, G, dev, reps=10):
    """SURVEY §8d configs C3 (Q4_0 11008x4096, N = 32: HBM-bound) and C5 (Q4_0 4096x4096, N = 512:
    MFMA-bound) through computeMatMul (xsplit_kernel + gemm_q_lds_kernel), one call per matrix,
    rotating over distinct weight copies (> Infinity Cache), graph-replayed. Reports algorithmic
    GB/s, useful TFLOP/s (2·M·N·K) and the MFMA-issued rate (2 bf16 MFMAs per useful one:
    x = hi + lo)."""
    T = G.GGMLType
    out = {}
    for name, qn, M, K, N, copies in (("c3_q4_0_11008x4096_n32", "Q4_0", 11008, 4096, 32, 16),
                                      ("c3_q4_1_11008x4096_n32", "Q4_1", 11008, 4096, 32, 16),
                                      ("c5_q4_0_4096x4096_n512", "Q4_0", 4096, 4096, 512, 32)):
        qt = getattr(T, qn)
        nb = M * K // 32 * BLOCK_BYTES[qn]
        g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
        wb = g.addBuffer(copies * nb + 256)
        xb = g.addBuffer(4 * K * N + 256)
        db = g.addBuffer(4 * M * N * copies + 256)
        src = torch.randn(M * K, device=dev) * 0.02
        for c in range(copies):
            g.buffers[wb][c * nb:(c + 1) * nb].copy_(G.quantizeTensor(src * (1 + 0.01 * c), qt))
        g.buffers[xb][: 4 * K * N].copy_(torch.randn(K * N, device=dev).view(torch.uint8))
        nodes = [(G.GGMLTensor(qt, [K, M], bufferId=wb, dataOffset=c * nb), G.GGMLTensor(T.F32, [N, K], bufferId=xb),
                  G.GGMLTensor(T.F32, [N, M], bufferId=db, dataOffset=4 * M * N * c)) for c in range(copies)]
        s = torch.cuda.Stream(device=dev)

        def run_all():
            for (a, b, d) in nodes:
                G.computeMatMul(g, None, a, b, d, stream=s)

        with torch.cuda.stream(s):
            run_all()
        torch.cuda.synchronize()
        gr = capture(torch, run_all, s)
        fn = gr.replay if gr is not None else run_all
        with torch.cuda.stream(s):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(reps):
                fn()
            e1.record(s)
        torch.cuda.synchronize()
        per = e0.elapsed_time(e1) / 1e3 / (reps * copies)
        nbytes = nb + 4 * K * N + 4 * M * N
        tf = 2 * M * N * K / per / 1e12
        out[name] = {"avg_launch_us": round(per * 1e6, 3), "achieved_GBps": round(nbytes / per / 1e9, 1),
                     "frac_of_8TBps": round(nbytes / per / 1e9 / HBM_PEAK_GBS, 4), "useful_TFLOPs": round(tf, 2),
                     "mfma_issued_TFLOPs": round(2 * tf, 2), "frac_of_2500TF_bf16": round(2 * tf / 2500, 4),
                     "rotating_weight_copies": copies, "hip_graph": gr is not None}
        del g
    # C1 on the device: F32 512x512x512 computeMatMul (the general F32 path, A5), timed the same way
    n, copies = 512, 4
    g = G.GGMLGraphAllocator(device=str(dev), defaultBufferSize=16)
    ab = g.addBuffer(4 * n * n * copies + 256)
    xb = g.addBuffer(4 * n * n + 256)
    db = g.addBuffer(4 * n * n * copies + 256)
    g.buffers[ab][: 4 * n * n * copies].copy_(torch.randn(n * n * copies, device=dev).view(torch.uint8))
    g.buffers[xb][: 4 * n * n].copy_(torch.randn(n * n, device=dev).view(torch.uint8))
    nodes = [(G.GGMLTensor(T.F32, [n, n], bufferId=ab, dataOffset=4 * n * n * c), G.GGMLTensor(T.F32, [n, n], bufferId=xb),
              G.GGMLTensor(T.F32, [n, n], bufferId=db, dataOffset=4 * n * n * c)) for c in range(copies)]
    s = torch.cuda.Stream(device=dev)

    def run_c1():
        for (a, b, d) in nodes:
            G.computeMatMul(g, None, a, b, d, stream=s)

    with torch.cuda.stream(s):
        run_c1()
    torch.cuda.synchronize()
    gr = capture(torch, run_c1, s)
    fn = gr.replay if gr is not None else run_c1
    with torch.cuda.stream(s):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
    torch.cuda.synchronize()
    per = e0.elapsed_time(e1) / 1e3 / (reps * copies)
    out["c1_f32_512x512x512"] = {"avg_launch_us": round(per * 1e6, 3), "GFLOPs": round(2 * n ** 3 / per / 1e9, 1),
                                 "kernel": "f32_lds_kernel (general F32 path, computeMatMul :1530-1543, operands staged in LDS, on v_mfma_f32_32x32x2_f32)", "hip_graph": gr is not None}
    del g
    return out


def host_path(torch, G, dev, layers=LAYERS, reps=5):
    """The Kotlin drop-in case, PCIe included (never `value`): Llama-7B layers on HOST buffers
    (ByteArray-backed), weights pinned on the device once. Per layer the dependent schedule
    {q,k,v} -> o -> {gate,up} -> down. Three ways to run it:
      per_node  — one lk_mul_mat per node (what computeMatMulHip does): B up, dst down, sync;
      graph_all — one ResidentGraph over all nodes, every dst written back (same semantics);
      graph_out — the same graph writing back only each layer's down output.
    Reported per token (x 32 / `layers`; all 32 layers by default, 3.65 GB of host weights)."""
    import numpy as np
    T = G.GGMLType
    total = layers * sum(alg_bytes(M, K) + 64 for (_, M, K) in LAYER_MATS) + 4 * HIDDEN + 64
    ga = G.GGMLGraphAllocator(device="host", defaultBufferSize=total)  # one ByteArray, no regrowth
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    nodes, outs = [], []
    x = ga.allocateTensor(T.F32, [1, HIDDEN], bufferId=0)
    ga.setTensorBytes(x, np.random.default_rng(1).standard_normal(HIDDEN).astype(np.float32))
    act = {"h": x}
    for _ in range(layers):
        for grp in CHAIN:
            for name in grp:
                M, K = next((m, k) for (n, m, k) in LAYER_MATS if n == name)
                src = act[X_OF[name]]
                a = ga.allocateTensor(T.Q4_0, [K, M])
                w = torch.randn(M * K, generator=gen, device=dev) * 0.02
                ga.setTensorBytes(a, G.quantizeTensor(w, T.Q4_0).cpu().numpy())
                del w
                d = ga.allocateTensor(T.F32, [1, M])
                nodes.append((a, src, d))
                outs.append(name == "down")
                if name in ("q", "o", "up", "down"):  # {q,k,v} -> o -> {gate,up} -> down -> next layer
                    act[{"q": "attn", "o": "h2", "up": "ffn", "down": "h"}[name]] = d
    for a, _, _ in nodes:
        G.weightsPin(ga, a)
    lay = 32 / layers

    def per_node():
        for a, b, d in nodes:
            G.computeMatMul(ga, ga.context, a, b, d)

    res = {"layers_timed": layers, "weights_pinned": True}
    # every way is timed in its steady state: the first call of a graph builds it and the second
    # captures its HIP graph (lk_graph_compute), so two untimed calls come first
    for key, fn in (("per_node", per_node),):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        per = (time.perf_counter() - t0) / reps * lay
        res[key] = {"ms_per_token": round(per * 1e3, 3), "tokens_per_s": round(1 / per, 2)}
    for key, mask in (("graph_all", None), ("graph_out", outs)):
        g = G.ResidentGraph(ga, nodes, outputs=mask)
        g.compute()
        g.compute()
        t0 = time.perf_counter()
        for _ in range(4 * reps):
            g.compute()
        per = (time.perf_counter() - t0) / (4 * reps) * lay
        res[key] = {"ms_per_token": round(per * 1e3, 3), "tokens_per_s": round(1 / per, 2),
                    "launches_per_layer": g.numLaunches / layers,
                    "h2d_bytes_per_token": int(g.transferBytes(True) * lay),
                    "d2h_bytes_per_token": int(g.transferBytes(False) * lay)}
        g.close()
    # the plugin path (GGMLHipBackend.graphCompute, core/GGMLCpuBackend.kt:167-176 contract): the
    # whole token's MUL_MAT graph, cached as one lk_graph; results consumed only by later nodes stay
    # in HBM, the rest (k, v, gate — read by the CPU ops of a real graph — and the last down) come back
    dsts = []
    for a, b, d in nodes:
        d.op, d.src = G.GGMLOp.MUL_MAT, [a, b]
        dsts.append(d)
    be = G.GGMLHipBackend(ga, wholeGraphs=True)  # the token's whole MUL_MAT graph in one call
    cg = G.GGMLCGraph(dsts, ga)
    for _ in range(2):
        if be.graphCompute(cg) != G.GGMLStatus.SUCCESS:
            raise RuntimeError("GGMLHipBackend.graphCompute failed")
    t0 = time.perf_counter()
    for _ in range(4 * reps):
        be.graphCompute(cg)
    per = (time.perf_counter() - t0) / (4 * reps) * lay
    mask = G.backend.writeBackMask(dsts, wholeGraph=True)
    res["backend"] = {"ms_per_token": round(per * 1e3, 3), "tokens_per_s": round(1 / per, 2),
                      "d2h_bytes_per_token": int(sum(4 * d.ne[0] * d.ne[1] for d, w in zip(dsts, mask) if w) * lay),
                      "path": "GGMLHipBackend.graphCompute -> cached lk_graph (ggml_hip/backend.py)"}
    be.free()
    G.weightsEvictAll()
    return res


def cpu_baseline(sample_rows, token_bytes, min_seconds=10.0):
    """The oracle's structural restatement of computeMatMul (single thread, like the reference)
    timed on this host over a bounded sample: the first `sample_rows` rows of each of one layer's
    7 matrices. GB/s on the same algorithmic-bytes basis; tokens/s extrapolated by bytes."""
    import numpy as np
    import oracle as O
    rng = np.random.default_rng(0)
    total_b = 0
    total_t = 0.0
    passes = 0
    ops = []
    for (name, M, K) in LAYER_MATS:
        rows = min(sample_rows, M)
        q = O.quantize(O.Q4_0, (rng.standard_normal(rows * K) * 0.02).astype(np.float32))
        x = rng.standard_normal((K, 1)).astype(np.float32)
        ops.append((q, rows, K, x))
    while passes == 0 or total_t < min_seconds:  # ~10 s of single-thread work (bounded sample)
        for (q, rows, K, x) in ops:
            t0 = time.perf_counter()
            O.mat_mul_q(O.Q4_0, q, rows, K, x)
            total_t += time.perf_counter() - t0
            total_b += alg_bytes(rows, K)
        passes += 1
    gbs = total_b / total_t / 1e9
    out = {"value": round(gbs, 5), "unit": "GB/s", "cores": 1, "kind": "port",
           "tokens_per_s": round(gbs * 1e9 / token_bytes, 6),
           "sample": f"structural C restatement of computeMatMul (oracle/lk_oracle.c), Q4_0 x F32 N=1, "
                     f"first {sample_rows} rows of each of the 7 Llama-7B layer matrices, {passes} passes ({total_b} "
                     f"algorithmic bytes, {total_t:.2f} s), single thread"}
    # SURVEY §8d's other two CPU lines: the same arithmetic without the accessor overhead
    # ("tight"), on one thread and with rows split over the host's cores (OpenMP)
    threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    variants = {}
    for label, nthr, rows_cap in (("tight_1_thread", 1, 4096), (f"tight_{threads}_threads", threads, None)):
        tb, tt = 0, 0.0
        for (name, M, K) in LAYER_MATS:
            rows = M if rows_cap is None else min(rows_cap, M)
            q = O.quantize(O.Q4_0, (rng.standard_normal(rows * K) * 0.02).astype(np.float32))
            x = rng.standard_normal((K, 1)).astype(np.float32)
            reps = 0
            t0 = time.perf_counter()
            while True:  # at least 0.1 s per matrix (the all-cores line finishes a matrix in ms)
                O.mat_mul_q(O.Q4_0, q, rows, K, x, tight=True, threads=nthr)
                reps += 1
                if time.perf_counter() - t0 >= 0.1:
                    break
            tt += time.perf_counter() - t0
            tb += reps * alg_bytes(rows, K)
        g = tb / tt / 1e9
        variants[label] = {"value": round(g, 4), "unit": "GB/s", "cores": nthr, "tokens_per_s": round(g * 1e9 / token_bytes, 4),
                           "sample": f"{'all rows' if rows_cap is None else f'first {rows_cap} rows'} of each layer matrix, "
                                     f"{tb} algorithmic bytes, {tt:.2f} s"}
    # config C2's CPU side ("Kotlin CPU vecDotQ8_0"): the structural restatement on Q8_0 4096x4096
    rows = 4096
    q = O.quantize(O.Q8_0, (rng.standard_normal(rows * 4096) * 0.02).astype(np.float32))
    x = rng.standard_normal((4096, 1)).astype(np.float32)
    t0 = time.perf_counter()
    O.mat_mul_q(O.Q8_0, q, rows, 4096, x)
    tq = time.perf_counter() - t0
    qb = rows * 4096 // 32 * 34 + 4 * 4096 + 4 * rows
    variants["structural_q8_0_4096x4096"] = {"value": round(qb / tq / 1e9, 5), "unit": "GB/s", "cores": 1,
                                             "sample": f"{rows} rows of a Q8_0 4096x4096 computeMatMul, N=1, {tq:.2f} s"}
    # config C1 (BASELINE configs[0]): F32 512x512x512 computeMatMul on the CPU path, the reference's
    # own protocol (T/core/GGMLMatMulBenchmarkTest.kt:180-202: 5 warmup runs, 10 timed, mean) on
    # the shapes/values of T/core/GGMLComputeOpsDestinationTest.kt:218-265 scaled to 512^3
    # (the benchmark test's F32 generator, :51-56)
    n = 512
    a32 = ((np.arange(n * n) + 42) % 127 - 63).astype(np.float32) / np.float32(10.0)
    b32 = (((np.arange(n * n) + 84) % 127 - 63).astype(np.float32) / np.float32(10.0)).reshape(n, n)
    for _ in range(5):
        O.mat_mul_q(O.F32, a32.view(np.uint8), n, n, b32)
    t0 = time.perf_counter()
    for _ in range(10):
        O.mat_mul_q(O.F32, a32.view(np.uint8), n, n, b32)
    t1 = (time.perf_counter() - t0) / 10
    variants["c1_f32_512"] = {"value": round(t1 * 1e3, 2), "unit": "ms per computeMatMul", "cores": 1,
                              "gflops": round(2 * n ** 3 / t1 / 1e9, 4), "higher_is_better": False,
                              "sample": "structural C restatement, F32 512x512x512, 5 warmup + 10 timed runs, mean"}
    out["variants"] = variants
    out["host"] = host_cpu()
    return out


def host_cpu():
    """The CPU the baseline ran on (report the GPU box host's model and core count)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"cpu_model": model, "nproc": os.cpu_count(), "usable_cpus": usable,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


if __name__ == "__main__":
    main()
