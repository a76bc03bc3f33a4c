"""Benchmark: QPS @ recall@10 >= 0.95, GIST-960-shaped L2, 1M base / 1k queries (BASELINE.json).

One step = one device batch_search of the 1k-query batch at the operating-point ef: the smallest
ef reaching recall@10 >= 0.95 against exact ground truth, bracketed by the reference's sweep
{10,20,40,60,80,120,200,400,600,800} and narrowed by bisection to ~1%.  The CPU baseline runs at
the same ef.  Inputs (rows, graph, queries) are resident in HBM before the timed region.

N > 1 (one rank per GPU): under torchrun (WORLD_SIZE set, it must equal --gpus), or started as
`python bench.py --gpus N`, which launches the N ranks itself (127.0.0.1 rendezvous) before any GPU
call; rank 0 prints the JSON line.  The workload is config 4 (10k queries) unless --nq says otherwise.
  --mode shard   (default) base rows partitioned by range, one HNSW graph per shard, every rank
                 searches all queries on its shard, per-shard top-k exchanged with an RCCL
                 all_gather over xGMI and merged by (distance, global id).  Total work fixed:
                 "scaling": "strong".  --shards S (S divides N) runs S range shards x N/S query
                 groups instead (sharded.Layout); by default the shard run is followed by a
                 "layouts" leg measuring every other S (the S = 1 layout is SURVEY §8e's replica
                 mode, queries split by range), reported beside `value` with the best of them.
  --mode replica every rank holds the whole index and answers its own 1k-query batch; no
                 collective on the data path: "scaling": "weak".

Prints one JSON line on rank 0 (schema in the task contract) with a "roofline" object for the
search kernel (algorithmic bytes from the kernel's own counters / HIP-event kernel time) and a
"cpu_baseline" object (the CPU restatement of the reference's coroutine batch_search, oracle/,
timed on this host at the same ef -- test infrastructure, never the product path).
"""

from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

EF_SWEEP = (10, 20, 40, 60, 80, 120, 200, 400, 600, 800)  # adapters/annbenchmark config.yml:21
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
K = 10
R = 32

# HNSW workloads (BASELINE.json configs; generators and seeds in workloads/datasets.py)
WORKLOADS = {
    "gist-hnsw": {"gen": "gist_like", "dim": 960, "nq": 1000, "metric": 0, "sq8": False,
                  "metric_name": "QPS @ recall@10>=0.95, GIST-960 L2, {base} base / {queries} queries",
                  "config_tag": {(1_000_000, 1000): "", (1_000_000, 10000): " (config 4)"},
                  "data": "synthetic (GIST-shaped 1024-centre low-rank mixture, seeds 5/6; graph built by the "
                          "engine's HNSW builder R=32 efc=100)"},
    "sift-hnsw": {"gen": "sift_like", "dim": 128, "nq": 10000, "metric": 0, "sq8": False,
                  "metric_name": "QPS @ recall@10>=0.95, SIFT-128 L2, {base} base / {queries} queries",
                  "config_tag": {(1_000_000, 10000): " (config 3)"},
                  "data": "synthetic (SIFT-shaped 1024-centre mixture, integer-valued, seeds 3/4; graph built by "
                          "the engine's HNSW builder R=32 efc=100)"},
    "sq8-ip": {"gen": "text_like", "dim": 768, "nq": 1000, "metric": 1, "sq8": True, "n": 10_000_000,
               "metric_name": "QPS @ recall@10>=0.95, 768-d IP, SQ8 search + f32 rerank, {base} base / {queries} "
                              "queries",
               "config_tag": {(10_000_000, 1000): " (config 5)", (10_000_000, 10000): " (config 5)"},
               "data": "synthetic (text-embedding-shaped 4096-centre unit-sphere mixture, 12 latent dims, "
                       "row-normalised, seeds 7/8; graph built on f32 rows with IP, R=32 efc=100; SQ8 codes of the "
                       "same rows)"},
}


def _count(v):
    for unit, div in (("M", 1_000_000), ("k", 1000)):
        if v >= div and v % div == 0:
            return f"{v // div}{unit}"
    return str(v)


def metric_label(w, n, nq):
    """The workload's metric string for this base / query count (the BASELINE metric at its own
    shape, e.g. "QPS @ recall@10>=0.95, GIST-960 L2, 1M base / 1k queries")."""
    return w["metric_name"].format(base=_count(n), queries=_count(nq)) + w["config_tag"].get((n, nq), "")


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--n", "--n-base", dest="n", type=int, default=0,
                   help="0 = the workload's default (1M; 10M for sq8-ip); --n-base under torchrun")
    p.add_argument("--nq", type=int, default=0, help="0 = the workload's default")
    p.add_argument("--dim", type=int, default=0, help="0 = the workload's default")
    p.add_argument("--efc", type=int, default=100)
    p.add_argument("--ef", type=int, default=0, help="fixed ef (skip the recall sweep)")
    p.add_argument("--target-recall", type=float, default=0.95)
    p.add_argument("--mode", choices=("shard", "replica"), default="shard")
    p.add_argument("--shards", type=int, default=0,
                   help="N>1 shard mode: S range shards x N/S query groups (S divides N); 0 = N (every rank "
                        "its own shard, every query on every rank: the north star's layout)")
    p.add_argument("--layouts", default="auto",
                   help="N>1 shard mode: other S to measure beside the result: 'auto' (every divisor of N), "
                        "'none', or a comma list")
    p.add_argument("--no-replica-leg", action="store_true", help="alias of --layouts none")
    p.add_argument("--exchange-cus", type=int, default=-1,
                   help="CUs the pipelined shard search leaves to the exchange stream (CU-masked compute "
                        "stream); -1 = 8 on the RCCL backend with N > 1, else 0")
    p.add_argument("--build-threads", type=int, default=0)
    p.add_argument("--builder", choices=("auto", "host", "gpu"), default="auto",
                   help="graph builder: host = HNSWBuilder restated on the host (cached; multi-threaded, so "
                        "not deterministic), gpu = the device batched build (alaya_index_build_graph, "
                        "deterministic); auto = gpu")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-tail-probe", action="store_true",
                   help="skip the 4x-tiled batch beside value (profiling runs: keeps every search launch the batch's)")
    p.add_argument("--cache-dir", default=os.path.join(ROOT, "data_cache"))
    p.add_argument("--dump-counters", default="")
    p.add_argument("--workload", choices=tuple(WORKLOADS) + ("flat",), default="gist-hnsw",
                   help="gist-hnsw: the BASELINE metric (default); sift-hnsw: config 3; sq8-ip: config 5 "
                        "shape (768-d IP, SQ8 search + rerank); flat: config 2, 1M x 128 exact k-NN")
    p.add_argument("--sweep-qps", action="store_true",
                   help="also time every ef of the sweep (config 3 reports the whole QPS/recall curve)")
    a = p.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.workload in WORKLOADS:
        w = WORKLOADS[a.workload]
        # N > 1 GIST: config 4 (10k queries sharded over the GPUs); N = 1: the metric's 1k queries
        a.nq = a.nq or (10_000 if (world > 1 and a.workload == "gist-hnsw") else w["nq"])
        a.dim = a.dim or w["dim"]
        a.n = a.n or w.get("n", 1_000_000)
    else:
        a.n = a.n or 1_000_000
        a.nq = a.nq or 1000
        a.dim = a.dim or 128
    return a


def _affinity():
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:  # pragma: no cover
        return max(1, os.cpu_count() or 1)


def _cgroup_cpus():
    """CPU quota of this process's cgroup (cgroup v2 cpu.max / v1 cfs quota), or None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            return float(quota) / float(period)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            quota = float(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            period = float(f.read())
        if quota > 0:
            return quota / period
    except (OSError, ValueError):
        pass
    return None


def host_threads():
    """Every core this process may run on -- the affinity set, capped by the cgroup's CPU quota when
    there is one (a quota of 16 CPUs on a 192-thread host runs 16 threads' worth, more threads only
    add contention).  The CPU baseline uses all of them."""
    q = _cgroup_cpus()
    return max(1, min(_affinity(), int(q + 0.999))) if q else _affinity()


def host_info():
    """nproc, the affinity size and the CPU model of this host (recorded with the CPU baseline)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    q = _cgroup_cpus()
    return {"nproc": os.cpu_count(), "affinity": _affinity(), "cgroup_cpus": None if q is None else round(q, 2),
            "threads_used": host_threads(), "cpu_model": model}


def spawn_ranks(n):
    """`bench.py --gpus N` without torchrun: start N ranks of this script (RANK/LOCAL_RANK/WORLD_SIZE,
    MASTER_ADDR=127.0.0.1) as child processes -- before this process touches the GPU -- and return
    the worst exit code.  Rank 0's stdout carries the JSON line."""
    import socket
    import subprocess

    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def graph_for(native, base, efc, threads, cache_dir, tag, metric=0):
    """Build (or load a cached copy of) the HNSW graph of `base` with the engine's host builder."""
    key = hashlib.md5(base[:: max(1, base.shape[0] // 4096)].tobytes()).hexdigest()[:12]
    path = os.path.join(cache_dir, f"{tag}_n{base.shape[0]}_d{base.shape[1]}_efc{efc}_{key}.index")
    if os.path.exists(path):
        try:
            g = native.Graph.load(path, 4)
            if g.arrays()[0].shape[0] == base.shape[0]:
                log("loaded cached graph", path)
                return g, 0.0
        except Exception as exc:  # corrupt cache: rebuild
            log("cache unusable:", exc)
    t = time.time()
    g = native.Graph.build(base, metric, R, efc, threads, 100)
    dt = time.time() - t
    log(f"built graph {base.shape} in {dt:.1f}s with {threads} threads")
    try:
        os.makedirs(cache_dir, exist_ok=True)
        g.save(path + ".tmp", 4, base.shape[0])
        os.replace(path + ".tmp", path)
    except OSError as exc:
        log("could not cache graph:", exc)
    return g, dt


def exact_candidates(torch, base_dev, queries_dev, base_host, queries_host, k=K, cand=64, metric=0,
                     chunk=1_000_000):
    """Exact top-k (L2, or IP = largest inner product) with their float64 distances: fp32 GEMM
    shortlist on the device, float64 re-rank on the host (ties by id).  The base is scanned in chunks
    of `chunk` rows: one GEMM operand above 2^31 elements (e.g. 10M x 768) is outside what the BLAS
    kernels index correctly."""
    nq = queries_host.shape[0]
    n = base_dev.shape[0]
    out = np.zeros((nq, k), np.int64)
    out_d = np.zeros((nq, k), np.float64)
    for s in range(0, nq, 256):
        q = queries_dev[s:s + 256]
        best_d, best_i = None, None
        for c0 in range(0, n, chunk):
            b = base_dev[c0:c0 + chunk]
            d = (b * b).sum(1)[None, :] - 2.0 * (q @ b.T) if metric == 0 else -(q @ b.T)
            dv, di = torch.topk(d, min(cand, b.shape[0]), dim=1, largest=False)
            di = di + c0
            if best_d is None:
                best_d, best_i = dv, di
            else:
                best_d, sel = torch.topk(torch.cat([best_d, dv], 1), min(cand, best_d.shape[1] + dv.shape[1]),
                                         dim=1, largest=False)
                best_i = torch.gather(torch.cat([best_i, di], 1), 1, sel)
        idx = best_i.cpu().numpy()
        for j in range(idx.shape[0]):
            c = idx[j]
            x = base_host[c].astype(np.float64)
            y = queries_host[s + j].astype(np.float64)
            dd = ((x - y) ** 2).sum(1) if metric == 0 else -(x @ y)
            o = np.lexsort((c, dd))[:k]
            m = len(o)
            out[s + j, :m], out_d[s + j, :m] = c[o], dd[o]
            if m < k:  # fewer rows than k
                out[s + j, m:], out_d[s + j, m:] = -1, np.inf
    return out, out_d


def exact_gt(torch, base_dev, queries_dev, base_host, queries_host, k=K, cand=64, metric=0, chunk=1_000_000):
    """Exact top-k ids (exact_candidates without the distances)."""
    return exact_candidates(torch, base_dev, queries_dev, base_host, queries_host, k, cand, metric, chunk)[0]


def f64_topk(base, ys, k=K, chunk=32768):
    """Exact top-k by float64 L2 for a few queries: one chunked pass over the base,
    |b|^2 - 2 b.y + |y|^2 with float64 GEMMs (ties by id)."""
    y = np.asarray(ys, np.float64)
    yn = (y * y).sum(1)
    parts = []
    for c in range(0, base.shape[0], chunk):
        b = base[c:c + chunk].astype(np.float64)
        parts.append((b * b).sum(1)[None, :] - 2.0 * (y @ b.T) + yn[:, None])
    d = np.concatenate(parts, axis=1)
    return [np.lexsort((np.arange(d.shape[1]), d[i]))[:k] for i in range(d.shape[0])]


def exact_gt_flat(native, base, queries, device, k=K):
    """Exact top-k for L2 from the engine's own flat path (find_exact_gt's f32 metric, evaluate.hpp:29-62,
    ties by id; queries whose shortlist bound fails are recomputed exhaustively), cross-checked in
    float64 on 1% of the queries, at most 16.  Returns (ids, f64 sample agreement)."""
    fi = native.DeviceIndex(device)
    fi.set_base(base, 0)
    ids, _, redo = fi.flat_search(queries, k)
    del fi
    rng = np.random.default_rng(0)
    sample = rng.choice(queries.shape[0], min(16, max(1, queries.shape[0] // 100)), replace=False)
    ref = f64_topk(base, queries[sample], k)
    agree = sum(int(set(r.tolist()) == set(ids[qi].tolist())) for r, qi in zip(ref, sample))
    log(f"ground truth: flat path, {redo} queries recomputed, float64 top-{k} sets equal on {agree}/{len(sample)}")
    return ids.astype(np.int64), f"{agree}/{len(sample)}"


def pmc_traffic(cfg):
    """HBM traffic of the search kernel from the committed rocprofv3 PMC passes on this workload
    (tools/run_pmc.sh -> tools/pmc_summary.py -> profiles/r*/traffic.json): the profile with the same
    n / nq / dim / k and the nearest ef (the multi-threaded host build moves the operating point by a
    few ef between runs); None if absent."""
    import glob

    best = None
    # latest round first: on equal ef gaps the most recent profile of the kernel wins
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic*.json")), reverse=True):
        try:
            t = json.load(open(path))
        except (OSError, ValueError):
            continue
        if t.get("kernel", "hnsw_search_kernel") != "hnsw_search_kernel":  # flat scans: traffic_flat*.json
            continue
        c = t["config"]
        if all(c.get(k) == v for k, v in cfg.items() if k != "ef_search"):
            gap = abs(c.get("ef_search", 0) - cfg["ef_search"])
            if best is None or gap < best[2]:
                best = (path, t, gap)
    return None if best is None else best[:2]


def choose_ef(probe):
    """Smallest ef reaching the recall target: the reference's ef sweep (config.yml:21) brackets
    it, then bisection between the last failing and the first passing sweep point narrows it to
    ~1% (recall is monotone in ef up to noise; the chosen ef is one that was measured to pass)."""
    lo = 0
    for ef in EF_SWEEP:
        if probe(ef):
            hi = ef
            break
        lo = ef
    else:
        return EF_SWEEP[-1]
    if lo == 0:
        return hi
    while hi - lo > max(1, lo // 100):
        mid = (lo + hi) // 2
        if probe(mid):
            hi = mid
        else:
            lo = mid
    return hi


def recall(ids, gt):
    hits = sum(len(set(ids[i].tolist()) & set(gt[i].tolist())) for i in range(ids.shape[0]))
    return hits / float(ids.size)


def flat_scan_kernel_name(dim, contraction=None):
    """The scan kernel launch_flat_scan (csrc/flat_kernels.hip) dispatches for rows of `dim` floats:
    the slabbed wide scan past 224 columns; for the single-pass f16 contraction the single-role scan
    over the cached tile records unless ALAYA_FLAT_TILES=0; else the warp-specialised scan unless the
    f32 contraction or the diagnostics' single-role f32 scan is forced by environment."""
    if (dim + 31) // 32 * 32 > 224:
        return "flat_scan_wide_kernel"
    if (os.environ.get("ALAYA_FLAT_F32") or os.environ.get("ALAYA_FLAT_WS0")
            or os.environ.get("ALAYA_FLAT_CONTRACTION") == "f32"):
        return "flat_scan_kernel"
    if contraction == "f16" and os.environ.get("ALAYA_FLAT_TILES", "1") != "0":
        return "flat_scan_tiles_kernel"
    return "flat_scan_ws_kernel"


def run_flat(args):
    """BASELINE config 2: flat exact k-NN, 1M x 128 U[0,1) (seeds 1/2), 1k queries, k=10, MFMA."""
    import torch

    from alayalite_amd import _native
    from workloads.datasets import uniform

    native = _native._ext
    n, dim = args.n, args.dim
    if dim == 128:
        base, queries = uniform(n, args.nq, dim, 1, 2)
        data = "synthetic U[0,1) seeds 1/2"
    else:  # wide rows: the GIST-shaped mixture (uniform high-d distances concentrate, see DESIGN)
        from workloads.datasets import gist_like

        base, queries = gist_like(n, args.nq, dim)
        data = "synthetic GIST-shaped mixture (workloads.datasets.gist_like)"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    index = native.DeviceIndex(0)
    index.set_base(base, 0)
    q_dev = torch.from_numpy(queries).to(dev)
    nq = q_dev.shape[0]
    ids = torch.empty((nq, K), dtype=torch.int32, device=dev)
    dists = torch.empty((nq, K), dtype=torch.float32, device=dev)
    flags = torch.empty((nq,), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        index.flat_search_device(q_dev.data_ptr(), nq, K, ids.data_ptr(), dists.data_ptr(), flags.data_ptr(),
                                 stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    n_flag = int(flags.sum().item())
    # exactness spot check against float64 on a sample (ties aside)
    sample = np.random.default_rng(0).choice(nq, 16, replace=False)
    got = ids.cpu().numpy()
    ok = 0
    for r, qi in zip(f64_topk(base, queries[sample], K), sample):
        ok += int(set(r.tolist()) == set(got[qi].tolist()))
    flops = 2.0 * n * nq * dim
    tf = flops / (ms * 1e-3) / 1e12
    # the roofline is the issued contraction's own MFMA peak (alaya_index_flat_last_contraction):
    # the single-pass f16 (default for rows of <= 224 floats) issues one f16 product per f32 product,
    # so its ceiling is the dense f16 peak (16 x 157.3 TF); the bf16 hi/lo split issues 3 bf16
    # products per f32 product (dense bf16 peak / 3); the f32 contraction runs at the 157.3 TF f32 peak
    contraction = {0: "f32", 1: "bf16x3", 2: "f16"}[index.flat_contraction()]
    scan = flat_scan_kernel_name(dim, contraction)
    mfma_peak = {"f32": 157.3, "bf16x3": round(16 * 157.3 / 3, 1), "f16": round(16 * 157.3, 1)}[contraction]
    # HBM traffic of the scan from the committed PMC passes on this workload and kernel
    # (tools/run_pmc_flat.sh; latest round first)
    import glob

    traffic = tsrc = None
    for tpath in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic_flat*.json")), reverse=True):
        t = json.load(open(tpath))
        c = t.get("config", {})
        if ((c.get("n_base"), c.get("n_queries"), c.get("dim"), t.get("kernel"), t.get("contraction", "bf16x3"))
                == (n, nq, dim, scan, contraction)):
            traffic, tsrc = t, os.path.relpath(tpath, ROOT)
            break
    cpu = None
    if not args.no_cpu_baseline:  # find_exact_gt restated (oracle/), a bounded sample of the queries
        import oracle

        oracle.build()
        ct = args.cpu_threads or host_threads()
        _, t_probe = oracle.exact_gt(base, queries[:ct], K, ct)
        m = int(min(nq, max(ct, ct * int(20.0 / max(t_probe, 1e-6)))))
        cpu_ids, sec = oracle.exact_gt(base, queries[:m], K, ct)
        same = int(sum(set(cpu_ids[i].tolist()) == set(got[i].tolist()) for i in range(m)))
        cpu = {"value": round(m / sec, 1), "unit": "queries/s", "cores": ct, "kind": "port",
               "sample": f"{m} of {nq} queries, find_exact_gt restated (l2_sqr AVX2 order + std::sort per query), "
                         f"queries over {ct} threads; top-{K} sets equal to the device's on {same}/{m}",
               "host": host_info()}
        log("cpu baseline", cpu)
    out = {
        "metric": (f"QPS, flat exact k-NN, {n // 1000}k x {dim} L2, {nq} queries"
                   + (" (BASELINE config 2)" if (n, dim, nq) == (1_000_000, 128, 1000) else "")),
        "value": round(nq * args.steps / elapsed, 1), "unit": "queries/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": data,
        "config": {"workload": f"flat-{n // 1000}k-{dim}-l2-{nq}q", "n_base": n, "n_queries": nq, "dim": dim, "k": K,
                   "flagged_queries": n_flag, "exact_vs_f64_sample": f"{ok}/{len(sample)}"},
        "roofline": {"bound": "mfma", "achieved": round(tf, 2), "peak": mfma_peak, "unit": "TFLOP/s",
                     "frac": round(tf / mfma_peak, 4),
                     "traffic": round(traffic["traffic_bytes_per_launch"] / (ms * 1e-3) / 1e9, 1) if traffic else None,
                     "traffic_unit": f"GB/s (HBM, PMC FETCH_SIZE x2 + WRITE_SIZE of {scan})",
                     "traffic_bytes_per_launch": int(traffic["traffic_bytes_per_launch"]) if traffic else None,
                     "traffic_source": tsrc,
                     "kernel": f"{scan}+flat_merge_kernel",
                     "kernel_ms": round(ms, 4), "algorithmic_flops_per_launch": flops,
                     # achieved = algorithmic f32 products (2 n nq d) / kernel time; peak = the issued
                     # contraction's dense MFMA peak (f16: 2516.8 TF; bf16x3: 2516.8 TF / 3; f32: 157.3 TF)
                     "contraction": contraction,
                     "peak_source": {"f32": "f32 MFMA dense peak (MI355X_MICROARCH.md)",
                                     "bf16x3": "bf16 MFMA dense peak 16 x 157.3 TF / 3 bf16 products per f32 "
                                               "product (MI355X_MICROARCH.md)",
                                     "f16": "f16 MFMA dense peak 16 x 157.3 TF, one f16 product per f32 product "
                                            "(MI355X_MICROARCH.md)"}[contraction]},
        "cpu_baseline": cpu,
        "build": _native.build_provenance(),
    }
    print(json.dumps(out), flush=True)


def main():
    args = parse()
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            print(f"[bench] WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}: refusing to report "
                  f"a different GPU count", file=sys.stderr, flush=True)
            return 2
    elif args.gpus > 1:
        return spawn_ranks(args.gpus)
    if args.workload == "flat":
        return run_flat(args)
    import torch
    import torch.distributed as dist

    w = WORKLOADS[args.workload]
    metric, use_sq8 = w["metric"], w["sq8"]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # ALAYA_BENCH_REHEARSE=1: every rank on cuda:0 with gloo -- rehearses the N-GPU code path
    # (shards, exchange, merge, timing) on a one-GPU box; never used for reported numbers
    rehearse = os.environ.get("ALAYA_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from alayalite_amd import _native
    from alayalite_amd.sharded import Layout, exchange_and_merge, gather_layout_results, shard_search
    import workloads.datasets as datasets

    native = _native._ext
    threads = args.build_threads or host_threads()

    shard_mode = world > 1 and args.mode == "shard"
    lay = Layout(world, rank, args.shards or world) if shard_mode else None
    group = lay.new_groups(dist) if shard_mode else None
    t0 = time.time()
    if shard_mode and w["gen"] == "text_like":
        # each rank generates only its shard's rows (config 5: 30.7 GB of f32 per whole base)
        lo, hi = lay.rows(args.n)
        base = None
        my_base = datasets.text_like_rows(lo, hi, args.dim)
        queries = datasets.text_like_queries(args.nq, args.dim)
        log(f"data: rows [{lo}, {hi}) of {args.n} + {queries.shape} in {time.time() - t0:.1f}s")
    else:
        base, queries = getattr(datasets, w["gen"])(args.n, args.nq, args.dim)
        log(f"data {base.shape} + {queries.shape} in {time.time() - t0:.1f}s")
        if shard_mode:
            lo, hi = lay.rows(args.n)
            my_base = np.ascontiguousarray(base[lo:hi])
        else:
            lo, hi = 0, args.n
            my_base = base
    tag = (f"{w['gen']}_m{metric}_shard{lay.shard}of{lay.shards}" if shard_mode else
           f"{w['gen']}_m{metric}" if w["gen"] != "gist_like" else "gist")

    # ---- index (shard or replica) ------------------------------------------------------------
    builder = args.builder if args.builder != "auto" else "gpu"
    index = native.DeviceIndex(local)
    index.set_base(my_base, metric)
    if builder == "gpu":
        t = time.time()
        graph, bstats = index.build_graph(R, args.efc, 100, 0, 0, 2)
        build_s = time.time() - t
        log(f"device-built graph {my_base.shape} in {build_s:.1f}s ({bstats})")
    else:
        graph, build_s = graph_for(native, my_base, args.efc, threads, args.cache_dir, tag, metric)
        index.set_graph(graph)
    sq8 = None
    if use_sq8:
        # SQ8Space::fit on the shard's rows (sq8_space.hpp:116-127); reduction order of the host's
        # get_*_sq8_func choice (AVX-512 -> 2, else AVX2 -> 1), as the reference would run here.
        mn, mx = native.sq8_train(my_base)
        codes = native.sq8_encode(my_base, mn, mx, threads)
        order = native.host_sq8_order()
        index.set_sq8(codes, mn, mx, order)
        sq8 = (codes, mn, mx, order)

    q_all = torch.from_numpy(queries).to(dev)
    nq_total = q_all.shape[0]
    qa, qb = lay.queries(nq_total) if shard_mode else (0, nq_total)
    q_dev = q_all[qa:qb]  # this rank's query group (the whole batch unless --shards < N)
    nq = q_dev.shape[0]
    ids_dev = torch.empty((nq, K), dtype=torch.int32, device=dev)
    dists_dev = torch.empty((nq, K), dtype=torch.float32, device=dev)
    cnt_dev = torch.empty((nq, 4), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def launch(ef, ix=None):
        ix = index if ix is None else ix
        if shard_mode and ix is index:
            # per-shard search (SQ8: search + rerank, id-0 entries on the shard holding global row 0);
            # slots without a candidate are (0xffffffff, FLT_MAX), never a spurious hit
            shard_search(ix, lo, use_sq8, q_dev, K, ef, ids_dev, dists_dev, cnt_dev, stream.cuda_stream)
        elif use_sq8:  # SQ8 graph search + PyIndex::rerank as batch_search runs it (rerank mode 1)
            ix.search_sq8_device(q_dev.data_ptr(), 0, nq, K, ef, 1, ids_dev.data_ptr(), dists_dev.data_ptr(),
                                 cnt_dev.data_ptr(), stream.cuda_stream)
        else:
            ix.search_device(q_dev.data_ptr(), nq, K, ef, ids_dev.data_ptr(), dists_dev.data_ptr(),
                             cnt_dev.data_ptr(), stream.cuda_stream)

    def step(ef):
        launch(ef)
        if shard_mode:
            return exchange_and_merge(ids_dev, dists_dev, lo, K, group)
        return ids_dev, dists_dev

    # ---- ground truth + operating point ------------------------------------------------------
    gt_check = None
    gt = None
    if base is None:  # rows generated per rank: every rank scores its own rows, rank 0 merges
        gt = sharded_exact_gt(torch, dist, dev, my_base, lo, q_all, queries, metric, lay)
        gt_check = ("per-rank rows: each rank's fp32 GEMM shortlist of 64 with float64 re-rank, the per-shard "
                    "top-10 merged by (float64 distance, id) on rank 0")
    elif rank == 0:
        if metric == 0:
            gt, gt_check = exact_gt_flat(native, base, queries, local)
        else:  # IP (config 5): fp32 GEMM shortlist + float64 re-rank
            base_dev = torch.from_numpy(base).to(dev)
            gt = exact_gt(torch, base_dev, q_all, base, queries, metric=metric)
            del base_dev
        torch.cuda.empty_cache()

    def probe(ef):
        """recall@10 >= target at this ef (decided on rank 0, broadcast to every rank)."""
        ids, dd = step(ef)
        if shard_mode and lay.groups > 1:  # every query group's merged rows, in query order
            ids, dd = gather_layout_results(ids, dd, lay, nq_total, dist)
        torch.cuda.synchronize()
        ok = False
        if rank == 0:
            r = recall(ids.cpu().numpy(), gt)
            sweep.append({"ef": ef, "recall": round(r, 4)})
            log(f"ef={ef} recall@10={r:.4f}")
            ok = r >= args.target_recall
        if world > 1:
            flag = torch.tensor([1 if ok else 0], device=dev)
            dist.broadcast(flag, 0)
            ok = bool(flag.item())
        return ok

    sweep = []
    if args.ef:
        probe(args.ef)
        ef = args.ef
    else:
        ef = choose_ef(probe)

    def timed(ef_t, steps, warmup):
        for _ in range(warmup):
            step(ef_t)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        for i in range(steps):
            ev[i][0].record(stream)
            launch(ef_t)
            ev[i][1].record(stream)
            if shard_mode:
                # exchange + merge of the same step (the search above is the per-shard kernel)
                exchange_and_merge(ids_dev, dists_dev, lo, K, group)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t_start
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = t.item()
        return el, float(np.mean([a.elapsed_time(b) for a, b in ev]))

    # ---- the QPS/recall curve (config 3 reports the sweep) ------------------------------------
    curve = None
    if args.sweep_qps and world == 1:
        curve = []
        for pt in sorted(sweep, key=lambda x: x["ef"]):
            el, kms = timed(pt["ef"], max(3, args.steps // 4), 1)
            curve.append({"ef": pt["ef"], "recall": pt["recall"], "qps": round(nq * max(3, args.steps // 4) / el, 1),
                          "kernel_ms": round(kms, 4)})
            log("curve", curve[-1])

    # ---- timed region ------------------------------------------------------------------------
    elapsed, kernel_ms = timed(ef, args.steps, args.warmup)
    overlap = None
    if shard_mode:
        # the same K steps double-buffered (ShardPipeline: the search of step i+1 runs beside the
        # all_gather + merge of step i on a second stream); this is `value`, the synchronous loop
        # above (search, then exchange, per step) is reported beside it with the exchange alone
        sync_elapsed = elapsed
        reserve = args.exchange_cus if args.exchange_cus >= 0 else (
            8 if (world > 1 and dist.get_backend() == "nccl") else 0)
        elapsed, pipe_search_ms = timed_pipeline(torch, dist, dev, ef, args.steps, args.warmup, index, lo, use_sq8,
                                                 q_dev, nq, group, reserve)
        exch_ms = timed_exchange(torch, dist, ids_dev, dists_dev, lo, args.steps, group)
        overlap = {"ms_per_step": round(elapsed / args.steps * 1e3, 4),
                   "sync_ms_per_step": round(sync_elapsed / args.steps * 1e3, 4),
                   "search_ms": round(kernel_ms, 4), "search_ms_in_pipeline": round(pipe_search_ms, 4),
                   "exchange_ms": round(exch_ms, 4),
                   "bound_ms": round(max(pipe_search_ms, exch_ms), 4), "reserved_cus": reserve,
                   "note": "value = the overlapped steps; sync = search then exchange in one stream per step"}
        log("overlap", overlap)

    # ---- PCIe-inclusive rate (reported beside value, never value): the host-buffer API's work --
    # queries H2D from pinned host memory, the search, ids + distances D2H, each step synchronised
    pcie = None
    if world == 1:
        q_host = torch.from_numpy(queries).pin_memory()
        ids_host = torch.empty((nq, K), dtype=torch.int32).pin_memory()
        d_host = torch.empty((nq, K), dtype=torch.float32).pin_memory()

        def host_step():
            q_dev.copy_(q_host, non_blocking=True)
            launch(ef)
            ids_host.copy_(ids_dev, non_blocking=True)
            d_host.copy_(dists_dev, non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()

        for _ in range(max(1, args.warmup)):
            host_step()
        t_p = time.perf_counter()
        for _ in range(args.steps):
            host_step()
        el_p = time.perf_counter() - t_p
        pcie = {"value": round(nq * args.steps / el_p, 1), "unit": "queries/s",
                "ms_per_step": round(el_p / args.steps * 1e3, 4),
                "note": "H2D queries (pinned) + search + D2H ids and distances, synchronised per step"}
        log("pcie-inclusive", pcie)

    # ---- batch tail (reported beside value, never value): the same queries tiled 4x into one
    # launch, so the tail -- the last queries' searches running on an emptying GPU -- is amortised
    # over four batches' work ("the tail").  Kernel sustained rate vs batch rate.
    tail = None
    if world == 1 and not args.no_tail_probe:
        q4 = q_dev.repeat(4, 1).contiguous()
        i4 = torch.empty((4 * nq, K), dtype=torch.int32, device=dev)
        d4 = torch.empty((4 * nq, K), dtype=torch.float32, device=dev)
        c4 = torch.empty((4 * nq, 4), dtype=torch.int32, device=dev)

        def launch4():
            if use_sq8:
                index.search_sq8_device(q4.data_ptr(), 0, 4 * nq, K, ef, 1, i4.data_ptr(), d4.data_ptr(),
                                        c4.data_ptr(), stream.cuda_stream)
            else:
                index.search_device(q4.data_ptr(), 4 * nq, K, ef, i4.data_ptr(), d4.data_ptr(), c4.data_ptr(),
                                    stream.cuda_stream)

        launch4()
        reps = 3
        a4, b4 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a4.record(stream)
        for _ in range(reps):
            launch4()
        b4.record(stream)
        torch.cuda.synchronize()
        ms4 = a4.elapsed_time(b4) / reps
        same = bool(torch.equal(i4[:nq], ids_dev) and torch.equal(i4[3 * nq:], ids_dev))
        tail = {"tiled_x4_qps": round(4 * nq / (ms4 * 1e-3), 1), "tiled_x4_ms": round(ms4, 4),
                "ids_equal_to_batch": same,
                "note": "the batch's queries repeated 4x in one launch: the searchers' sustained rate with the "
                        "batch tail amortised; value is the single batch"}
        del q4, i4, d4, c4
        log("batch tail", tail)

    # ---- algorithmic bytes from the kernel's counters -------------------------
    cnt = cnt_dev.cpu().numpy().astype(np.int64)
    row_bytes = args.dim if use_sq8 else 4 * args.dim  # SQ8 codes are 1 B per dimension
    per_q = (row_bytes * (cnt[:, 0] + cnt[:, 2]) + 4 * R * cnt[:, 1] + 4 * R * cnt[:, 3]
             + 4 * args.dim + 8 * K)
    if use_sq8:  # the rerank reads ef ids' f32 rows (k real + ef-k zero entries -> row 0 once)
        per_q = per_q + 4 * args.dim * (K + (1 if ef > K else 0))
    bytes_launch = float(per_q.sum())
    achieved = bytes_launch / (kernel_ms * 1e-3) / 1e9
    traffic = None
    prof = pmc_traffic({"n_base": args.n, "n_queries": nq, "dim": args.dim, "k": K, "ef_search": ef})
    if prof is not None and world == 1:
        # measured HBM bytes per algorithmic byte (PMC, gfx950-corrected) of the search kernel x
        # this launch's bytes (SQ8: the search's ratio applied to search + rerank bytes)
        traffic_bytes = prof[1]["traffic_over_algorithmic"] * bytes_launch
        traffic = {"gbs": round(traffic_bytes / (kernel_ms * 1e-3) / 1e9, 1),
                   "bytes_per_launch": int(traffic_bytes),
                   "source": f"{os.path.relpath(prof[0], ROOT)} (PMC at ef={prof[1]['config']['ef_search']})"}
    if args.dump_counters and rank == 0:
        np.save(args.dump_counters, cnt)
    # measured streaming-read ceiling of this GPU (reported beside the 8 TB/s vendor figure)
    measured_peak = native.hbm_stream_read(local, 4 << 30, 5) if rank == 0 else 0.0

    units_per_step = nq_total * (world if (world > 1 and args.mode == "replica") else 1)
    value = units_per_step * args.steps / elapsed

    # ---- layouts leg (N>1 shard mode): the other S-shard x N/S-query-group layouts -------------
    layouts = None
    if shard_mode and args.layouts != "none" and not args.no_replica_leg:
        others = ([s_ for s_ in range(1, world + 1) if world % s_ == 0 and s_ != lay.shards]
                  if args.layouts == "auto" else [int(x) for x in args.layouts.split(",")])
        layouts = []
        for S in others:
            row = layout_leg(args, native, torch, dist, dev, S, base, metric, use_sq8, threads, q_all, queries,
                             rank, world, gt)
            if row is not None:
                layouts.append(row)

    # ---- CPU baseline: the reference's coroutine batch_search restated (oracle/) --------------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, graph, base, queries, ef, metric, sq8, ids_dev.cpu().numpy().astype(np.uint32))
        log("cpu baseline", cpu)

    # ---- memory per rank: the N-rank command sized against one node's host memory and HBM ----------
    import resource

    free_b, total_b = torch.cuda.mem_get_info(dev)
    mem = {"rank": rank, "host_peak_rss_gb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20, 2),
           "device_used_gb": round((total_b - free_b) / 2**30, 2)}
    mems = [mem]
    if world > 1:
        mems = [None] * world
        dist.all_gather_object(mems, mem)

    if rank == 0:
        r_at = next((s["recall"] for s in sweep if s["ef"] == ef), None)
        out = {
            "metric": metric_label(w, args.n, nq_total),
            "value": round(value, 1),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak" if (world > 1 and args.mode == "replica") else "strong",
            "vs_baseline": None,
            "dtype": "u8+f32" if use_sq8 else "f32",
            "data": w["data"] + ("; graph from the device HNSW build" if builder == "gpu" else ""),
            "config": {"workload": f"hnsw-{w['gen'].split('_')[0]}{args.dim}-{args.n // 1000}k-"
                                   f"{'ip-sq8' if use_sq8 else ('ip' if metric else 'l2')}-{nq_total}q",
                       "n_base": args.n, "n_queries": nq_total, "dim": args.dim, "k": K, "ef_search": ef,
                       "recall_at_10": r_at, "ef_sweep": sweep, "mode": args.mode if world > 1 else "single",
                       "parallelism": (f"{lay.shards}shards-x-{lay.groups}querygroups" if shard_mode else
                                       f"{args.mode}{world}" if world > 1 else "1gpu"),
                       "timed_region": ("device-resident queries and results: the search launches (plus the "
                                        "exchange when N > 1) between synchronised barriers, as the task contract "
                                        "defines value; SURVEY 8d's host-buffer region (H2D queries + search + "
                                        "D2H ids/distances) is pcie_inclusive"),
                       "graph_build_s": round(build_s, 1), "graph_builder": builder,
                       "ground_truth": (gt_check if base is None else
                                        ("engine flat path (f32 metric of find_exact_gt), float64 top-10 sets "
                                         f"equal on {gt_check} sampled queries") if gt_check else
                                        "fp32 GEMM shortlist of 64, float64 re-rank")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "measured_peak": round(measured_peak, 1),
                         "frac_measured": round(achieved / measured_peak, 4),
                         "measured_peak_source": "alaya_hbm_stream_read: best streaming read of 4 GiB (3 load "
                                                 "shapes x 2 occupancies x 5 runs), this GPU, this run",
                         "traffic": traffic["gbs"] if traffic else None,
                         "traffic_bytes_per_launch": traffic["bytes_per_launch"] if traffic else None,
                         "traffic_source": traffic["source"] if traffic else None,
                         "kernel": "hnsw_search_kernel" + ("+rerank_kernel" if use_sq8 else ""),
                         "kernel_ms": round(kernel_ms, 4),
                         "algorithmic_bytes_per_launch": int(bytes_launch),
                         "mean_n_dist": round(float(cnt[:, 0].mean()), 1),
                         "mean_n_expand": round(float(cnt[:, 1].mean()), 1)},
            "cpu_baseline": cpu,
            # which sources the loaded libalaya_hip.so was compiled from, against this tree's
            "build": _native.build_provenance(),
            "memory": {"per_rank": mems,
                       "note": "host_peak_rss_gb: the rank's peak resident set (getrusage); device_used_gb: "
                               "memory in use on the rank's GPU at the end of the run (hipMemGetInfo: every "
                               "process on that GPU, so all ranks when a rehearsal shares one GPU)"},
        }
        if curve is not None:
            out["config"]["qps_curve"] = curve
        if layouts is not None:
            out["layouts"] = layouts
            if layouts:
                best = max(layouts + [{"shards": lay.shards, "query_groups": lay.groups, "value": round(value, 1)}],
                           key=lambda x: x["value"])
                out["best_layout"] = {"shards": best["shards"], "query_groups": best["query_groups"],
                                      "value": best["value"],
                                      "note": "value stays the north star's layout; this is the fastest measured"}
        if overlap is not None:
            out["exchange_overlap"] = overlap
        if pcie is not None:
            out["pcie_inclusive"] = pcie
        if tail is not None:
            tail["tiled_over_batch"] = round(tail["tiled_x4_qps"] / value, 3)
            out["batch_tail"] = tail
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def timed_pipeline(torch, dist, dev, ef, steps, warmup, index, lo, use_sq8, q_dev, nq, group=None, reserve=0):
    """K shard steps through ShardPipeline (double-buffered: the search of step i+1 overlaps the
    exchange of step i; `reserve` CUs left to the exchange stream); barrier + synchronize on both
    sides, max over ranks.  Returns (seconds, mean search ms inside the pipeline, from a second
    untimed pass with events)."""
    from alayalite_amd.sharded import ShardPipeline, shard_search

    fn = lambda q, i, d, c, s: shard_search(index, lo, use_sq8, q, K, ef, i, d, c, s)  # noqa: E731
    pipe = ShardPipeline(fn, nq, K, lo, dev, group, reserve_cus=reserve)
    pipe.run([q_dev] * max(1, warmup))
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pipe.run([q_dev] * steps)
    torch.cuda.synchronize()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    # the search time as it runs inside the pipeline (a separate, untimed pass with events)
    tp = ShardPipeline(fn, nq, K, lo, dev, group, timing=True, reserve_cus=reserve)
    tp.run([q_dev] * steps)
    torch.cuda.synchronize()
    pipe.close()
    tp.close()
    sm = torch.tensor([tp.search_ms()], device=dev, dtype=torch.float64)
    dist.all_reduce(sm, op=dist.ReduceOp.MAX)
    return el.item(), sm.item()


def timed_exchange(torch, dist, ids_dev, dists_dev, lo, steps, group=None):
    """The exchange alone (pack, all_gather, merge sort) on resident shard results: ms per step,
    max over ranks."""
    from alayalite_amd.sharded import exchange_and_merge

    exchange_and_merge(ids_dev, dists_dev, lo, K, group)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        exchange_and_merge(ids_dev, dists_dev, lo, K, group)
    torch.cuda.synchronize()
    el = torch.tensor([(time.perf_counter() - t0) / steps * 1e3], device=ids_dev.device, dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return el.item()


# host bytes of one rank's shard rows beyond which a layouts leg is skipped (the S = 1 layout of config
# 5 would hold the whole 30.7 GB f32 base on every rank)
LAYOUT_ROWS_CAP_BYTES = 16 << 30


def layout_leg(args, native, torch, dist, dev, S, base, metric, use_sq8, threads, q_all, queries, rank, world, gt):
    """One S-shard x N/S-query-group layout (sharded.Layout) beside the main result: rank r builds
    shard r % S on the device (SQ8: its own quantizer; the shard holding global row 0 keeps the
    rerank's id-0 entries) and answers query group r // S; the group's ranks exchange inside their
    own process group.  The operating ef is chosen on rank 0 against the same ground truth.  S = 1
    is SURVEY §8e's replica mode (whole index per GPU, queries split by range, no collective).
    value = all queries x steps / step time (max over ranks): total work fixed ("strong")."""
    from alayalite_amd.sharded import Layout, exchange_and_merge, gather_layout_results, shard_search
    import workloads.datasets as datasets

    lay = Layout(world, rank, S)
    group = lay.new_groups(dist)
    lo, hi = lay.rows(args.n)
    if (hi - lo) * args.dim * 4 > LAYOUT_ROWS_CAP_BYTES:
        log(f"layout {S}x{lay.groups}: skipped ({hi - lo} rows of {args.dim} f32 per rank)")
        return None
    t = time.time()
    rows = np.ascontiguousarray(base[lo:hi]) if base is not None else datasets.text_like_rows(lo, hi, args.dim)
    ix = native.DeviceIndex(dev.index)
    ix.set_base(rows, metric)
    ix.build_graph(R, args.efc, 100, 0, 0, 2)
    if use_sq8:
        mn, mx = native.sq8_train(rows)
        ix.set_sq8(native.sq8_encode(rows, mn, mx, threads), mn, mx, native.host_sq8_order())
    del rows
    nq_total = q_all.shape[0]
    qa, qb = lay.queries(nq_total)
    q = q_all[qa:qb]
    nq = q.shape[0]
    ids = torch.empty((nq, K), dtype=torch.int32, device=dev)
    dd = torch.empty((nq, K), dtype=torch.float32, device=dev)
    cnt = torch.empty((nq, 4), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    dist.barrier()
    log(f"layout {S}x{lay.groups}: shard graphs built in {time.time() - t:.1f}s")

    def step(ef):
        shard_search(ix, lo, use_sq8, q, K, ef, ids, dd, cnt, stream.cuda_stream)
        return exchange_and_merge(ids, dd, lo, K, group)

    sweep = []

    def probe(ef):
        mi, md = step(ef)
        if lay.groups > 1:
            mi, md = gather_layout_results(mi, md, lay, nq_total, dist)
        torch.cuda.synchronize()
        ok = False
        if rank == 0:
            r = recall(mi.cpu().numpy(), gt)
            sweep.append({"ef": ef, "recall": round(r, 4)})
            ok = r >= args.target_recall
        flag = torch.tensor([1 if ok else 0], device=dev)
        dist.broadcast(flag, 0)
        return bool(flag.item())

    ef = choose_ef(probe)
    for _ in range(args.warmup):
        step(ef)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(ef)
    torch.cuda.synchronize()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = el.item()
    r_at = next((x["recall"] for x in sweep if x["ef"] == ef), None)
    out = {"shards": S, "query_groups": lay.groups, "value": round(nq_total * args.steps / el, 1),
           "unit": "queries/s", "scaling": "strong", "ms_per_step": round(el / args.steps * 1e3, 4),
           "ef_search": ef, "recall_at_10": r_at, "graph_builder": "gpu",
           "note": ("whole index per GPU, queries split by range, no collective (SURVEY 8e replica mode)" if S == 1
                    else f"{S} range shards, {lay.groups} query groups all-gathering inside their own process group")}
    log("layout", out)
    del ix
    torch.cuda.empty_cache()
    return out


def sharded_exact_gt(torch, dist, dev, rows, lo, q_all, queries, metric, lay, k=K):
    """Exact top-k when no rank holds the whole base (rows generated per rank): every rank scores its
    own rows (exact_candidates: fp32 GEMM shortlist, float64 re-rank), the per-shard (float64
    distance, global id) candidates are gathered, and rank 0 keeps the k smallest by (distance, id).
    Returns the ids on rank 0, None elsewhere."""
    base_dev = torch.from_numpy(rows).to(dev)
    ids, d64 = exact_candidates(torch, base_dev, q_all, rows, queries, k=k, metric=metric)
    del base_dev
    torch.cuda.empty_cache()
    ids = torch.from_numpy(ids + lo).to(dev)
    d64 = torch.from_numpy(d64).to(dev)
    gi = [torch.empty_like(ids) for _ in range(lay.world)]
    gd = [torch.empty_like(d64) for _ in range(lay.world)]
    if dist.get_backend() == "gloo":
        ids, d64 = ids.cpu(), d64.cpu()
        gi = [x.cpu() for x in gi]
        gd = [x.cpu() for x in gd]
    dist.all_gather(gi, ids)
    dist.all_gather(gd, d64)
    if lay.rank != 0:
        return None
    # shard r % S holds rows lay.rows(); every shard appears G times (query groups): take one copy each
    ai = np.concatenate([gi[s].cpu().numpy() for s in range(lay.shards)], 1)
    ad = np.concatenate([gd[s].cpu().numpy() for s in range(lay.shards)], 1)
    out = np.zeros((ai.shape[0], k), np.int64)
    for qi in range(ai.shape[0]):
        out[qi] = ai[qi][np.lexsort((ai[qi], ad[qi]))][:k]
    return out


def cpu_baseline(args, graph, base, queries, ef, metric, sq8, device_ids):
    """The oracle's coroutine batch driver (Scheduler/Worker restatement, AVX2 kernels) at the same
    ef on this host's cores; SQ8 adds the post-join single-thread rerank loop (index.hpp:337-345).
    Bounded sample: the whole batch when it fits ~30 s of CPU, else a prefix of the queries."""
    import oracle

    oracle.build()
    l0, levels, off, ue, ep, upper_r, _ = graph.arrays()
    view = oracle.IndexView(base, l0, levels, off, ue, upper_r, ep, metric=metric,
                            sq8=None if sq8 is None else (sq8[0], sq8[1], sq8[2], sq8[3]))
    ct = args.cpu_threads or host_threads()
    nq = queries.shape[0]

    def run(qs):
        ids, _, _, sec = view.batch_search(qs, K, ef, ct)
        if sq8 is not None:
            ids, _, rsec = view.batch_rerank(qs, ids, K, ef)
            sec += rsec
        return ids, sec

    # size the sample: time a small prefix first
    probe_n = min(nq, 100)
    _, t_probe = run(queries[:probe_n])
    per_q = t_probe / probe_n
    m = nq if per_q * nq <= 30.0 else max(probe_n, int(30.0 / max(per_q, 1e-9)))
    sample = queries[:m]
    runs, cpu_ids = [], None
    budget = time.time() + 45.0
    run(sample)  # warm-up
    while len(runs) < 5 and (time.time() < budget or not runs):
        cpu_ids, sec = run(sample)
        runs.append(sec)
    med = float(np.median(runs))
    parity = bool(np.array_equal(cpu_ids, device_ids[:m]))
    what = "search + rerank" if sq8 is not None else "search"
    qps = sorted(m / r for r in runs)
    return {"value": round(m / med, 1), "unit": "queries/s", "cores": ct, "kind": "port",
            "sample": f"{m} of {nq} queries at ef={ef} ({what}), median of {len(runs)} runs after 1 warm-up "
                      f"(Scheduler begin->join{' + rerank loop' if sq8 is not None else ''}), "
                      f"ids_equal_to_device={parity}",
            "spread": {"runs": len(runs), "min": round(qps[0], 1), "median": round(m / med, 1),
                       "max": round(qps[-1], 1), "note": "queries/s per timed run (the host is shared: "
                                                         "runs of different rounds differ up to ~2x)"},
            "host": host_info()}


if __name__ == "__main__":
    sys.exit(main() or 0)
