#!/usr/bin/env python3
"""Benchmark: SpGEMM forward + SSpMM backward edges/s on Reddit (synthetic, D=256, k=16).

Metric (BASELINE.json): "SpGEMM+SSpMM edges/sec on Reddit, hidden=256, k in {8,16,32,64};
%HBM roofline". One step = one SpGEMM forward over all E edges + one SSpMM backward over
all E edges, inputs (graph, CBSR features, upstream gradient) resident in HBM;
value = 2E / step time (edges/s = 2E / (t_fwd + t_bwd)).

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)

N > 1: the rows are partitioned over the ranks (strong scaling: the Reddit graph is fixed)
and each step includes the RCCL all-gather of the CBSR records and the reduce-scatter of
grad_sp (maxk_kernels.dist). Each rank generates only its own rows of the graph (counter-based
draws: every N benchmarks the same graph). Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
sys.path.insert(0, ROOT)

# numpy, torch and maxk_kernels are imported by _imports() once the process knows it is a
# rank: a bare `bench.py --gpus N` (N > 1) parent spawns the ranks and never touches HIP
np = torch = dist = mk = graphs = RowPartition = ShardedAggregation = None


def _imports():
    global np, torch, dist, mk, graphs, RowPartition, ShardedAggregation
    import numpy as _np
    import torch as _torch
    import torch.distributed as _dist

    import maxk_kernels as _mk
    from maxk_kernels import graphs as _graphs
    from maxk_kernels.dist import RowPartition as _RP, ShardedAggregation as _SA
    np, torch, dist, mk, graphs = _np, _torch, _dist, _mk, _graphs
    RowPartition, ShardedAggregation = _RP, _SA


# BASELINE.json "metric", verbatim: the primary line is k=16 (config.workload), the other k
# of the set are the k_sweep entries
METRIC = "SpGEMM+SSpMM edges/sec on Reddit, hidden=256, k in {8,16,32,64}; %HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
# L1-miss line-request ceiling: ~1 request of 128 B per ns per CU for L2-resident gathers
# (tools/ubench_tcp.hip, profiles/r01/ubench_tcp.log), x 256 CUs
L2_REQUEST_CEILING_GBS = 256 * 128.0


def fwd_bytes(n, e, k, d):
    """Algorithmic (compulsory) bytes of one SpGEMM forward."""
    return 4 * (n + 1) + 8 * e + 5 * k * n + 4 * d * n


def bwd_bytes(n, e, k, d):
    """Algorithmic bytes of one SSpMM backward: rowptr, idx+val, G, selector, grad write."""
    return 4 * (n + 1) + 8 * e + 4 * d * n + k * n + 4 * k * n


def log(*a):
    # MAXK_BENCH_VERBOSE=1: every rank logs (multi-rank rehearsals)
    if int(os.environ.get("RANK", "0")) == 0 or os.environ.get("MAXK_BENCH_VERBOSE"):
        print(f"[rank {os.environ.get('RANK', '0')}]", *a, file=sys.stderr, flush=True)


def event_time_ms(fn, reps):
    """Average device time of fn() over reps launches, HIP events on the current stream
    (the C ABI launches on torch's current stream)."""
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def launch_percentiles_ms(fn, reps):
    """Per-launch device times (one event pair around each launch): p10 / median / p90."""
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for s, e in evs:
        s.record()
        fn()
        e.record()
    evs[-1][1].synchronize()
    t = sorted(s.elapsed_time(e) for s, e in evs)
    pick = lambda q: t[min(len(t) - 1, int(round(q * (len(t) - 1))))]  # noqa: E731
    return {"p10": pick(0.1), "median": pick(0.5), "p90": pick(0.9)}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(ptr, idx, val, sp_data, sp_index, h, g, d, sample_frac, runs, warmup, log_fn):
    """DGL-semantics dense CSR SpMM on the host cores (oracle C/OpenMP restatement of
    update_all(copy_u, sum) with edge weights), forward A @ X and backward A^T @ G, on a
    bounded sample of the destination rows, by BASELINE.md §3's protocol: `warmup` untimed
    runs, then the median of `runs` timed runs. Two inputs, as §3 lists them: (a) the dense
    MaxK output, zeros included, as DGL sees it (`value`), and (b) the ReLU of the layer
    input, the reference's ReLU baseline (`relu_value`)."""
    from oracle import oracle

    n = ptr.numel() - 1
    dev = ptr.device
    # dense MaxK output and the transposed graph, built on the GPU, copied to the host
    x = torch.zeros((n, d), dtype=torch.float32, device=dev)
    x.scatter_(1, sp_index.long(), sp_data)
    order = torch.argsort(idx.long(), stable=True)
    rows = torch.repeat_interleave(torch.arange(n, device=dev), (ptr[1:] - ptr[:-1]).long())
    idx_t = rows[order].to(torch.int32)
    val_t = val[order]
    cnt = torch.bincount(idx.long(), minlength=n)
    ptr_t = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    ptr_t[1:] = torch.cumsum(cnt, 0)
    hh = {k: v.cpu().numpy() for k, v in dict(ptr=ptr, idx=idx, val=val, x=x,
                                                relu=torch.relu(h), g=g,
                                                ptr_t=ptr_t.to(torch.int32), idx_t=idx_t,
                                                val_t=val_t).items()}
    del x, order, rows, idx_t, val_t, cnt, ptr_t
    e = int(hh["ptr"][-1])
    target = int(e * sample_frac)
    r_f = int(np.searchsorted(hh["ptr"], target))
    r_b = int(np.searchsorted(hh["ptr_t"], target))
    e_f, e_b = int(hh["ptr"][r_f]), int(hh["ptr_t"][r_b])
    y = np.zeros((n, d), np.float32)

    def one(feat):
        t0 = time.perf_counter()
        oracle.dense_spmm(hh["ptr"], hh["idx"], hh["val"], hh[feat], row_end=r_f, out=y)
        t1 = time.perf_counter()
        oracle.dense_spmm(hh["ptr_t"], hh["idx_t"], hh["val_t"], hh["g"], row_end=r_b, out=y)
        return t1 - t0, time.perf_counter() - t1

    res = {}
    for feat in ("x", "relu"):
        for _ in range(warmup):
            one(feat)
        t = [one(feat) for _ in range(runs)]
        tot = sorted(a + b for a, b in t)
        med = float(np.median(tot))
        res[feat] = {"median_s": med, "fwd_s": float(np.median([a for a, _ in t])),
                     "bwd_s": float(np.median([b for _, b in t])),
                     "min_s": tot[0], "max_s": tot[-1], "value": (e_f + e_b) / med}
        log_fn(f"cpu baseline ({feat}): median of {runs} after {warmup} warm-ups: "
               f"{med:.3f}s for fwd {e_f} + bwd {e_b} edges")
    affinity = len(os.sched_getaffinity(0))
    threads = oracle.num_threads()
    return {
        "value": res["x"]["value"],
        "unit": "edges/s",
        "cores": threads,
        "threads": threads,
        "relu_value": res["relu"]["value"],
        "median_of": runs,
        "warmup_runs": warmup,
        "cpu_model": cpu_model(),
        "host_cpus": os.cpu_count(),
        "affinity_cpus": affinity,
        "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
        "threads_reason": (
            "OpenMP threads = OMP_NUM_THREADS, the CPU share the GPU pool leases with one "
            "GPU (16 on the MI355X boxes). The affinity mask spans the whole machine "
            f"({affinity} CPUs), shared with the other leases' jobs, so more threads would "
            "time other tenants' load, not this path"
            if os.environ.get("OMP_NUM_THREADS") else
            "OpenMP default: every CPU in the affinity mask"),
        "kind": "port",
        "sample": (f"DGL-semantics dense CSR SpMM (oracle C/OpenMP, f32): forward A@X over "
                   f"rows [0,{r_f}) = {e_f} edges and backward A^T@G over rows [0,{r_b}) of "
                   f"the transposed graph = {e_b} edges ({sample_frac:.0%} of E each), "
                   f"D={d}; value: X = dense MaxK output, relu_value: X = ReLU(layer input); "
                   f"median of {runs} runs after {warmup} warm-ups (BASELINE.md §3)"),
        "fwd_s": res["x"]["fwd_s"],
        "bwd_s": res["x"]["bwd_s"],
        "runs": res,
    }


# graphs.DATASETS keys, here so the arguments parse before torch is imported (checked in run)
DATASET_NAMES = ("flickr", "ogbn-products", "ogbn-proteins", "reddit", "yelp")


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dataset", default="reddit", choices=DATASET_NAMES)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--cpu-sample", type=float, default=0.1,
                    help="fraction of E timed per direction and run for the CPU baseline")
    ap.add_argument("--cpu-runs", type=int, default=10,
                    help="timed CPU runs (the median is reported; BASELINE.md §3)")
    ap.add_argument("--cpu-warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-comparator", action="store_true")
    ap.add_argument("--k-sweep", default="8,32,64",
                    help="extra k values timed at N=1 (kernel device time; '' to skip)")
    ap.add_argument("--graph", default="auto",
                    help="'synthetic', 'auto' (the DGL cache file ~/.dgl/... when it exists, "
                         "else synthetic) or a path to a scipy save_npz adjacency")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args(argv)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv, poll_s=0.2, grace_s=10.0, straggler_s=None):
    """`bench.py --gpus N` without a launcher (no WORLD_SIZE in the environment): start N
    rank processes of this script with the torch.distributed.run environment (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT), relay rank 0's stdout
    (the JSON line), and return 0 when every rank exits 0. When a rank fails, the others
    (which may be waiting in a collective for it) are terminated by PID and the failing
    rank's exit code is returned. When some ranks exit 0 while others are still running
    ``straggler_s`` seconds later (MAXK_BENCH_STRAGGLER_S, default 300: a rank stuck in a
    collective its peers left), the rest are terminated and 124 is returned. This
    process imports neither torch nor maxk_kernels, so it never initialises HIP before the
    children start (an exec or fork after HIP init is not safe on this platform)."""
    import signal
    import subprocess
    import threading

    assert "torch" not in sys.modules, "the spawning parent must not import torch"
    if straggler_s is None:
        straggler_s = float(os.environ.get("MAXK_BENCH_STRAGGLER_S", "300"))
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    base = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                ROLE_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                MAXK_BENCH_SPAWNED="1")
    print(f"[bench] spawning {n} ranks on 127.0.0.1:{port} (parent imports no torch)",
          file=sys.stderr, flush=True)
    procs = []

    def stop(sig=None, frame=None):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.time() + grace_s
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        if sig is not None:
            sys.exit(128 + sig)

    old_term = signal.signal(signal.SIGTERM, stop)
    relay = None
    try:
        for r in range(n):
            env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                          env=env,
                                          stdout=subprocess.PIPE if r == 0 else None,
                                          text=True))

        def pump(f):
            for line in f:
                sys.stdout.write(line)
                sys.stdout.flush()

        relay = threading.Thread(target=pump, args=(procs[0].stdout,), daemon=True)
        relay.start()
        rc = 0
        first_done = None
        while True:
            codes = [p.poll() for p in procs]
            bad = [(i, c) for i, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                i, rc = bad[0]
                print(f"[bench] rank {i} exited with {rc}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                stop()
                break
            if all(c == 0 for c in codes):
                break
            if first_done is None and any(c == 0 for c in codes):
                first_done = time.time()
            if first_done is not None and time.time() - first_done > straggler_s:
                left = [i for i, c in enumerate(codes) if c is None]
                print(f"[bench] ranks {left} still running {straggler_s:.0f}s after the others "
                      f"exited; stopping them", file=sys.stderr, flush=True)
                stop()
                rc = 124
                break
            time.sleep(poll_s)
    finally:
        stop()
        if relay is not None:
            relay.join(timeout=5)
        signal.signal(signal.SIGTERM, old_term)
    return rc if rc >= 0 else 128 - rc


def rank_identity(dev_index):
    """This rank's device as the HIP runtime reports it (the driver checks these fields)."""
    import socket
    p = torch.cuda.get_device_properties(dev_index)
    return {"rank": int(os.environ.get("RANK", "0")),
            "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
            "host": socket.gethostname(), "device_index": dev_index,
            "pci_bus_id": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
            "uuid": str(p.uuid), "name": p.name, "gcn_arch": p.gcnArchName,
            "visible_devices": {v: os.environ[v] for v in ("HIP_VISIBLE_DEVICES",
                                                           "ROCR_VISIBLE_DEVICES",
                                                           "CUDA_VISIBLE_DEVICES")
                                if v in os.environ}}


def gather_topology(ident, backend, world):
    """Every rank's identity (one all_gather_object), the group's world size and backend as
    torch.distributed reports them, and the RCCL version torch is linked against."""
    ranks = [ident]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, ident)
    topo = {"world_size": dist.get_world_size() if world > 1 else 1,
            "backend": dist.get_backend() if world > 1 else None,
            "launcher_world_size": world, "requested_backend": backend, "ranks": ranks,
            "torch": torch.__version__, "hip": getattr(torch.version, "hip", None)}
    try:
        topo["rccl_version"] = ".".join(str(v) for v in torch.cuda.nccl.version())
    except Exception as exc:  # pragma: no cover - torch build without RCCL
        topo["rccl_version"] = f"unavailable: {exc!r}"[:80]
    return topo


def check_topology(topo, backend):
    """One GPU per rank under RCCL: two nccl ranks resolving to one device would time the same
    GPU twice (or share it), so every rank refuses to run (non-zero exit)."""
    if topo["world_size"] != topo["launcher_world_size"]:
        raise SystemExit(f"[bench] torch.distributed world size {topo['world_size']} != "
                         f"WORLD_SIZE {topo['launcher_world_size']}")
    if backend != "nccl":
        return
    seen = {}
    for r in topo["ranks"]:
        for key in ((r["host"], "pci", r["pci_bus_id"]), (r["host"], "uuid", r["uuid"])):
            if key in seen:
                raise SystemExit(f"[bench] ranks {seen[key]} and {r['rank']} resolve to the same "
                                 f"device ({key[1]} {key[2]} on {key[0]}): nccl needs one GPU "
                                 f"per rank")
            seen[key] = r["rank"]


def _selftest_rank(spec):
    """MAXK_BENCH_SELFTEST (tests/test_bench_spawn.py): a rank that only reports what the
    launcher handed it, without HIP. 'ok': rank 0 prints one JSON line. 'fail:R': rank R
    exits 3 and the others hang (as ranks stuck in a collective would). 'exit0:R': rank R
    exits 0 at once and the others hang (the straggler limit ends them). 'topology' /
    'topology:dup': the ranks form a gloo group, gather made-up device identities (distinct, or
    all one device) and run the nccl one-GPU-per-rank check; rank 0 prints the topology."""
    global torch, dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if spec.startswith("fail:"):
        if rank == int(spec.split(":", 1)[1]):
            time.sleep(0.5)
            sys.exit(3)
        time.sleep(600)
    if spec.startswith("exit0:"):
        if rank == int(spec.split(":", 1)[1]):
            sys.exit(0)
        time.sleep(600)
    if spec.startswith("topology"):
        import torch as _torch
        import torch.distributed as _dist
        torch, dist = _torch, _dist
        dist.init_process_group("gloo")
        q = 0 if spec == "topology:dup" else rank
        ident = {"rank": rank, "local_rank": int(os.environ["LOCAL_RANK"]), "host": "selftest",
                 "device_index": q, "pci_bus_id": f"0000:{0x05 + q:02x}:00", "uuid": f"GPU-{q}",
                 "name": "selftest", "gcn_arch": "gfx950", "visible_devices": {}}
        topo = gather_topology(ident, "gloo", world)
        check_topology(topo, "nccl")
        if rank == 0:
            print(json.dumps({"selftest": True, "topology": topo}), flush=True)
        dist.destroy_process_group()
        return
    if rank == 0:
        print(json.dumps({"selftest": True, "world": world, "rank": rank,
                          "local_rank": int(os.environ["LOCAL_RANK"]),
                          "master": f"{os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}",
                          "spawned": os.environ.get("MAXK_BENCH_SPAWNED") == "1"}), flush=True)


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if os.environ.get("MAXK_BENCH_SELFTEST"):
        _selftest_rank(os.environ["MAXK_BENCH_SELFTEST"])
        return
    _imports()
    assert set(DATASET_NAMES) == set(graphs.DATASETS), "DATASET_NAMES out of date"
    run(args)


def run(args):
    if os.environ.get("MAXK_BENCH_TRACEBACK_S"):  # where a stuck rank is (rehearsals)
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["MAXK_BENCH_TRACEBACK_S"]), repeat=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # MAXK_BENCH_BACKEND=gloo rehearses the N > 1 path with several ranks sharing the GPUs
    # a one-GPU box has (collectives staged through host memory; timings not meaningful)
    backend = os.environ.get("MAXK_BENCH_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        raise SystemExit(f"MAXK_BENCH_BACKEND={backend}: expected nccl or gloo")
    dev_index = local_rank if backend == "nccl" else local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        log(f"process group up ({backend}, world {world})")
    # what RCCL actually sees: every rank's device, checked before any work
    topology = gather_topology(rank_identity(dev_index), backend, world)
    check_topology(topology, backend)

    n, e_target = graphs.DATASETS[args.dataset]
    d, k = args.dim, args.k
    # ranks that share a device (a gloo rehearsal on a one-GPU box) take turns through the
    # setup: four processes' radix sorts at once on one GPU stalled for minutes
    shared = world > 1 and backend == "gloo" and world > torch.cuda.device_count()

    def setup_turns(fn):
        if not shared:
            return fn()
        res = None
        for q in range(world):
            if q == rank:
                res = fn()
                torch.cuda.synchronize()
            dist.barrier()
        return res

    gpath = None
    if args.graph == "auto":
        gpath = graphs.find_dgl_graph(args.dataset)
    elif args.graph != "synthetic":
        gpath = args.graph

    def build_graph():
        t0 = time.perf_counter()
        if gpath:
            ptr, idx = graphs.load_npz_csr(gpath, device=dev)
            data = (f"graph loaded from {gpath} (+ self-loops); N(0,1) features seed 97, "
                    f"upstream grad seed 98")
            part = RowPartition(ptr, world)
            e0, e1 = part.edges(ptr, rank)
            idx = idx[e0:e1].contiguous()
        else:
            ptr = graphs.synthetic_ptr(n, e_target, seed=97, device=dev)
            part = RowPartition(ptr, world)
            idx = graphs.synthetic_rows(ptr, seed=97, rows=part.rows(rank))
            data = (f"synthetic ({args.dataset}-shaped graph: lognormal degrees sigma=1.2, "
                    f"uniform columns from a counter-based stream, self-loops, seed 97; each "
                    f"rank generates its own rows; N(0,1) features seed 97, upstream grad seed 98)")
        r0, r1 = part.rows(rank)
        lptr = ptr[r0:r1 + 1]
        val = graphs.sage_mean_values(lptr, num_edges=idx.numel())   # the rank's edges
        torch.cuda.synchronize()
        log(f"graph {args.dataset}: rows [{r0}, {r1}) of N={ptr.numel() - 1}, "
            f"{idx.numel()} edges {'loaded' if gpath else 'generated'} in "
            f"{time.perf_counter() - t0:.1f}s")
        return ptr, idx, val, part, data

    ptr, idx, val, part, data = setup_turns(build_graph)
    n = ptr.numel() - 1
    e = int(part.num_edges)
    # PMC traffic in --traffic-json was collected on the synthetic graphs
    tkey = args.dataset if not gpath else args.dataset + ":file"
    r0, r1 = part.rows(rank)
    h = graphs.features(n, d, seed=97, device=dev)[r0:r1].contiguous()
    g = graphs.features(n, d, seed=98, device=dev)[r0:r1].contiguous()

    t0 = time.perf_counter()
    if world == 1:
        sp_data, sp_index = mk.maxk_forward(h, k, return_index=True)
        plan = mk.get_plan(ptr, idx, val, n, e, d, k)
        info = plan.info()
        out = torch.empty((n, d), dtype=torch.float32, device=dev)
        grad_sp = torch.empty((n, k), dtype=torch.float32, device=dev)

        def fwd():
            plan.forward(sp_data, sp_index, out)

        def bwd():
            plan.backward(g, sp_index, grad_sp)

        def step():
            fwd()
            bwd()
    else:
        def build_shard():
            sh = ShardedAggregation(part, rank, ptr, idx, val, d, k, local_edges=True)
            # the top-k lands in the shard's send records: the exchange copies nothing
            bufs = mk.maxk_forward(h, k, return_index=True, out=sh.local_buffers())
            return sh, bufs

        shard, (sp_data, sp_index) = setup_turns(build_shard)
        info = shard.plan.info()
        grad_sp = shard.grad_table
        shard.gather(sp_data, sp_index)

        def fwd():  # this rank's kernels alone, no collectives
            shard.compute_forward()

        def bwd():
            shard.compute_backward(g)

        def step():
            shard.forward(sp_data, sp_index)
            shard.backward(g)
    torch.cuda.synchronize()
    plan_s = time.perf_counter() - t0
    log(f"plan built in {plan_s:.2f}s: {info}")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    log("warm-up done")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed * 1e3 / args.steps
    value = 2.0 * e / (elapsed / args.steps)

    # per-kernel device time (HIP events on the launch stream), this rank's shard
    reps = max(5, args.steps)
    fwd_ms = event_time_ms(fwd, reps)
    bwd_ms = event_time_ms(bwd, reps)
    fwd_pct = launch_percentiles_ms(fwd, reps)
    bwd_pct = launch_percentiles_ms(bwd, reps)
    exchange = None
    if world > 1:
        # the two exchange steps alone (blocking collectives: torch's current stream waits on
        # the RCCL stream, so the events bracket them), max over ranks; bytes per rank
        def all_gather():
            shard.gather(sp_data, sp_index)

        def reduce_scatter():
            dist.reduce_scatter_tensor(shard.grad_local,
                                       grad_sp, op=dist.ReduceOp.SUM)

        dist.barrier()
        ag_ms = event_time_ms(all_gather, reps)
        dist.barrier()
        rs_ms = event_time_ms(reduce_scatter, reps)
        tx = torch.tensor([ag_ms, rs_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tx, op=dist.ReduceOp.MAX)
        ag_ms, rs_ms = (float(v) for v in tx.tolist())
        ag_bytes = shard.table_rec.numel()             # received records incl. own slice
        rs_bytes = 4 * k * part.padded_rows            # grad_sp reduced over all columns
        exchange = {"all_gather_ms": ag_ms, "reduce_scatter_ms": rs_ms,
                    "all_gather_bytes": ag_bytes, "reduce_scatter_bytes": rs_bytes,
                    "all_gather_GBps": ag_bytes / (ag_ms * 1e-3) / 1e9,
                    "reduce_scatter_GBps": rs_bytes / (rs_ms * 1e-3) / 1e9}
    # the MaxK producer of the path (exact top-k -> CBSR), this rank's rows
    topk_ms = event_time_ms(lambda: mk.maxk_forward(h, k, return_index=True), reps)
    e_loc = info["num_edges"]
    n_loc = info["num_nodes"]
    fb = fwd_bytes(n_loc, e_loc, k, d)
    bb = bwd_bytes(n_loc, e_loc, k, d)
    fwd_gbs = fb / (fwd_ms * 1e-3) / 1e9
    bwd_gbs = bb / (bwd_ms * 1e-3) / 1e9
    dom = "sspmm_bwd" if bwd_ms >= fwd_ms else "spgemm_fwd"
    achieved = bwd_gbs if dom == "sspmm_bwd" else fwd_gbs
    traffic = None
    detail = {}
    lib_sha = mk._lib.lib_sha256()
    traffic_sha = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            key = f"{tkey}:k{k}:d{d}:n{world}"
            traffic_sha = tj.get(key, {}).get("lib_sha256")
            traffic = tj.get(key, {}).get(dom)
            detail = tj.get(key, {}).get(dom + "_detail", {})
        except (OSError, ValueError):
            traffic = None
    # a figure collected on another kernel binary says nothing about this one
    traffic_stale = traffic is not None and traffic_sha != lib_sha
    if traffic_stale:
        traffic, detail = None, {}

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": data,
        "config": {
            "workload": f"{args.dataset} SpGEMM fwd + SSpMM bwd over CBSR (MaxK exact), "
                        f"D={d}, k={k}",
            "dataset": args.dataset, "num_nodes": n, "num_edges": e, "dim_origin": d,
            "dim_k": k,
            "parallelism": "single-gpu" if world == 1 else
            f"row-partition x{world} + {'RCCL' if backend == 'nccl' else 'gloo (rehearsal)'} "
            f"all-gather(CBSR records) / reduce-scatter(grad_sp)",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_stale": traffic_stale,
            "traffic_lib_sha256": traffic_sha,
            "lib_sha256": lib_sha,
            "algorithmic_bytes": bb if dom == "sspmm_bwd" else fb,
        },
        "fwd_ms": fwd_ms,
        "bwd_ms": bwd_ms,
        "exchange": exchange,
        "topk_ms": topk_ms,
        "topk_GBps": (h.numel() * 4 + 5 * h.shape[0] * k) / (topk_ms * 1e-3) / 1e9,
        "fwd_launch_ms": fwd_pct,
        "bwd_launch_ms": bwd_pct,
        # supplementary: the bound that binds an irregular gather on gfx950 is the L1-miss
        # line-request rate, not HBM bytes; from profiles/ PMC counters
        "l1_request_roofline": None if "l1_miss_requests" not in detail else {
            "kernel": dom,
            "requests_per_launch": detail["l1_miss_requests"],
            "achieved": detail["l1_miss_requests"] * 128 / ((bwd_ms if dom == "sspmm_bwd" else fwd_ms) * 1e-3) / 1e9,
            "peak": L2_REQUEST_CEILING_GBS, "unit": "GB/s",
            "frac": detail["l1_miss_requests"] * 128 / ((bwd_ms if dom == "sspmm_bwd" else fwd_ms) * 1e-3) / 1e9 / L2_REQUEST_CEILING_GBS,
            "l2_hit_rate": detail.get("l2_hit_rate"),
        },
        "fwd_edges_per_s": e_loc / (fwd_ms * 1e-3),
        "bwd_edges_per_s": e_loc / (bwd_ms * 1e-3),
        "fwd_roofline_frac": fwd_gbs / HBM_PEAK_GBS,
        "bwd_roofline_frac": bwd_gbs / HBM_PEAK_GBS,
        "plan_build_s": plan_s,
        "topology": topology,
        "cpu_baseline": None,
    }

    def sweep_traffic(ks, tf, tb):
        """PMC traffic (FETCH_SIZE x 2 + WRITE_SIZE per launch, profiles/pmc_traffic.json) of
        the k's forward and backward kernels, its rate, and its ratio to the algorithmic
        bytes (traffic well above the compulsory bytes = re-reads); null when the entry was
        collected on another kernel binary."""
        ent = {}
        try:
            ent = json.load(open(args.traffic_json)).get(f"{tkey}:k{ks}:d{d}:n1", {})
        except (OSError, ValueError):
            pass
        out = {"traffic_stale": bool(ent) and ent.get("lib_sha256") != lib_sha}
        if out["traffic_stale"]:
            ent = {}
        for dirn, kern, t, ab in (("fwd", "spgemm_fwd", tf, fwd_bytes(n, e, ks, d)),
                                  ("bwd", "sspmm_bwd", tb, bwd_bytes(n, e, ks, d))):
            tr = ent.get(kern)
            out[f"{dirn}_traffic"] = tr
            out[f"{dirn}_traffic_ratio"] = None if tr is None else tr / ab
            out[f"{dirn}_traffic_GBps"] = None if tr is None else tr / (t * 1e-3) / 1e9
        return out

    if world == 1 and args.k_sweep:
        # the metric's k in {8,16,32,64}: same graph and features, kernel device time only
        sweep = {str(k): {"fwd_ms": fwd_ms, "bwd_ms": bwd_ms,
                          "edges_per_s": 2 * e / ((fwd_ms + bwd_ms) * 1e-3),
                          "fwd_roofline_frac": fwd_gbs / HBM_PEAK_GBS,
                          "bwd_roofline_frac": bwd_gbs / HBM_PEAK_GBS}}
        sweep[str(k)].update(sweep_traffic(k, fwd_ms, bwd_ms))
        h_full = graphs.features(n, d, seed=97, device=dev)
        for ks in [int(x) for x in args.k_sweep.replace('"', "").split(",") if x.strip()]:
            if ks == k:
                continue
            sd, si = mk.maxk_forward(h_full, ks, return_index=True)
            p = mk.GraphPlan(ptr, idx, val, n, e, d, ks)
            o = torch.empty((n, d), dtype=torch.float32, device=dev)
            gr = torch.empty((n, ks), dtype=torch.float32, device=dev)
            for _ in range(2):
                p.forward(sd, si, o)
                p.backward(g, si, gr)
            tf = event_time_ms(lambda: p.forward(sd, si, o), reps)
            tb = event_time_ms(lambda: p.backward(g, si, gr), reps)
            sweep[str(ks)] = {
                "fwd_ms": tf, "bwd_ms": tb, "edges_per_s": 2 * e / ((tf + tb) * 1e-3),
                "fwd_roofline_frac": fwd_bytes(n, e, ks, d) / (tf * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "bwd_roofline_frac": bwd_bytes(n, e, ks, d) / (tb * 1e-3) / 1e9 / HBM_PEAK_GBS,
            }
            sweep[str(ks)].update(sweep_traffic(ks, tf, tb))
            log(f"k={ks}: fwd {tf:.3f} ms bwd {tb:.3f} ms")
            del p, sd, si, o, gr
        del h_full
        result["k_sweep"] = dict(sorted(sweep.items(), key=lambda kv: int(kv[0])))

    if rank == 0 and world == 1 and not args.no_comparator:
        # rocSPARSE SpMM on the dense MaxK output: the reference's cuSPARSE comparators
        # (spmm_cusparse SO@0x243a0, spmm_cusparse_coo SO@0x24700) called directly (best of
        # the CSR and COO algorithms), and the same product through torch.sparse
        from maxk_kernels import baselines
        comp = {}
        x = torch.zeros((n, d), dtype=torch.float32, device=dev)
        x.scatter_(1, sp_index.long(), sp_data)
        for alg in ("default", "csr_merge_path", "csr_row_split"):
            try:
                _, ms = baselines.spmm_rocsparse(ptr, idx, val, x, times=5, alg=alg)
                comp[f"rocsparse_spmm_{alg}_ms"] = ms
            except Exception as exc:  # pragma: no cover - library/alg availability
                comp[f"rocsparse_spmm_{alg}_error"] = repr(exc)[:160]
        rows = baselines.coo_rows(ptr)   # spmm_cusparse_coo (SO@0x24700): the COO form
        for alg in ("coo_segmented", "coo_atomic"):
            try:
                _, ms = baselines.spmm_rocsparse_coo(rows, idx, val, x, times=5, alg=alg)
                comp[f"rocsparse_spmm_{alg}_ms"] = ms
            except Exception as exc:  # pragma: no cover - library/alg availability
                comp[f"rocsparse_spmm_{alg}_error"] = repr(exc)[:160]
        del rows
        best = [v for kk, v in comp.items() if kk.endswith("_ms")]
        if best:
            comp["rocsparse_spmm_best_ms"] = min(best)
            comp["spgemm_fwd_speedup_vs_rocsparse"] = min(best) / fwd_ms
        try:
            a = torch.sparse_csr_tensor(ptr.long(), idx.long(), val, size=(n, n))
            comp["torch_sparse_mm_ms"] = event_time_ms(lambda: torch.sparse.mm(a, x), 3)
            del a
        except Exception as exc:  # pragma: no cover - depends on torch build
            comp["torch_sparse_mm_error"] = repr(exc)[:160]
        result["comparator"] = comp
        del x

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(ptr, idx, val, sp_data, sp_index, h, g, d,
                                              args.cpu_sample, args.cpu_runs, args.cpu_warmup,
                                              log)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
