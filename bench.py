"""Benchmark: NetRep permutation null distributions on MI355X.

Workload (BASELINE.json configs[2], the metric's "20k genes x 50 modules"):
synthetic coexpression, 20,000 genes x 500 samples, 50 modules of
round(linspace(30, 300, 50)) genes, null = "overlap", all seven statistics.
A step = one nr_run over --perms-per-step permutations (every module of
each; kernel launches of --launch-batch permutations), nulls copied back to
host memory. The defaults time 20 x 5,120 = 102,400 permutations per GPU:
the metric's nPerm = 100k. Inputs (test corr, net, scaled data, discovery
vectors) are resident in HBM before the timed region.

A secondary record times the network-only path on the same 20k-gene
matrices (BASELINE.json configs[3], C4: the HBM-bound gather kernel) in the
same run.

Multi-GPU: one process per GPU. `--gpus N` without a torchrun environment
re-launches this script under torch.distributed.run with N processes before
any GPU call. Rank 0 builds the datasets and broadcasts the test matrices
over RCCL; every rank then evaluates its own disjoint permutation range (weak
scaling: fixed permutations per GPU), with no collective on the data path.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import netrep_amd as N  # noqa: E402
from netrep_amd import synthetic as S  # noqa: E402
from netrep_amd.distributed import broadcast_tensors, gather_nulls, perm_range  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_MFMA_PEAK_TFS = 78.6    # MI355X fp64 matrix peak (spec)


TRAFFIC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def _pmc_row(config, batch, kernel, table=False):
    """The committed rocprofv3 PMC pass (tools/collect_pmc.sh +
    tools/summarize_pmc.py, recorded by tools/pmc_to_traffic.py) of this
    config / launch size / kernel, or None. PMC counters cannot be read from
    inside the timed run, so the numbers are the ones measured on the same
    command; Gram-table passes carry "gram_table": true."""
    try:
        with open(TRAFFIC_FILE) as f:
            rows = json.load(f)
    except (OSError, ValueError):
        return None
    live = [r for r in rows if r.get("config") == config and r.get("kernel") == kernel
            and bool(r.get("gram_table", False)) == table and "superseded" not in r]
    for r in live:
        if r.get("batch") == batch:
            return r
    # a launch of a nearby size (the reference interface sizes its own
    # launches, e.g. 66 permutations at C5): the pass's per-launch bytes, flops
    # and time scaled by the launch size, marked as such
    near = [r for r in live if r.get("batch") and abs(batch / r["batch"] - 1.0) <= 0.1]
    if not near:
        return None
    r = dict(min(near, key=lambda x: abs(x["batch"] - batch)))
    f = batch / r["batch"]
    for key in ("hbm_bytes_per_launch", "fetch_size_kb_raw", "write_size_kb", "avg_ns_rocprof",
                "mfma_f64_flops_executed"):
        if key in r:
            r[key] = r[key] * f
    r["scaled_from_batch"] = r["batch"]
    return r


def traffic_fields(config, batch, kernel, avg_ms, table=False):
    """Counter traffic per launch of `kernel` from its PMC pass: `traffic` =
    FETCH_SIZE x 2 + WRITE_SIZE (the gfx950 correction MI355X_MICROARCH.md
    prescribes for wide streams), `traffic_range` = [raw FETCH_SIZE +
    WRITE_SIZE, the corrected figure] (the x2 factor is uncalibrated for narrow
    random gathers), and the pass's rocprofv3 kernel time against this run's
    HIP-event time (`traffic_time_ratio`: the pass describes this kernel when
    it is within 2% of 1)."""
    r = _pmc_row(config, batch, kernel, table)
    if r is None:
        return {"traffic": None, "traffic_source": None}
    raw = (r["fetch_size_kb_raw"] + r["write_size_kb"]) * 1024.0
    out = {"traffic": float(r["hbm_bytes_per_launch"]), "traffic_range": [raw, float(r["hbm_bytes_per_launch"])],
           "traffic_source": r.get("source"), "traffic_pass_avg_ms": r["avg_ns_rocprof"] / 1e6}
    if "scaled_from_batch" in r:
        out["traffic_scaled_from_batch"] = r["scaled_from_batch"]
    if avg_ms > 0:
        out["traffic_time_ratio"] = round(r["avg_ns_rocprof"] / 1e6 / avg_ms, 4)
        # the bytes the kernel actually moves past L2 per second, against HBM peak
        # (Infinity-Cache hits included, so this can exceed what HBM alone delivers)
        out["traffic_GBps"] = round(float(r["hbm_bytes_per_launch"]) / (avg_ms * 1e-3) / 1e9, 1)
        out["traffic_frac_of_hbm_peak"] = round(out["traffic_GBps"] / HBM_PEAK_GBS, 4)
    return out


def measured_mfma(config, batch, kernel, avg_ms, table=False):
    """Executed fp64 MFMA work of `kernel` from the same committed PMC pass
    (SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 flops per launch, tools/summarize_pmc.py),
    as TFLOP/s over this run's HIP-event launch time, and the MFMA-busy share
    (SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE / 8 x 1,024 SIMDs); None
    when no pass matches."""
    r = _pmc_row(config, batch, kernel, table)
    if r is None or "mfma_f64_flops_executed" not in r or avg_ms <= 0:
        return None
    return {"executed_TFLOPs": round(r["mfma_f64_flops_executed"] / (avg_ms * 1e-3) / 1e12, 4),
            "mfma_busy_pct": round(r.get("mfma_busy_pct", float("nan")), 2), "source": r.get("source")}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--perms-per-step", type=int, default=0,
                    help="permutations per step (0: 5,120, at least one launch)")
    ap.add_argument("--launch-batch", "--batch", type=int, default=5120, dest="batch",
                    help="permutations per kernel launch (5,120: one launch per step, 256,000 C3 items; "
                         "1,024 / 2,048 / 4,096 measured 12,237 / 12,319 / 12,340 perms/s, "
                         "profiles/r02/batch/)")
    ap.add_argument("--config", default="C3", choices=["C2", "C3", "C4", "C5"])
    ap.add_argument("--no-secondary", action="store_true", help="skip the C4 network-only record")
    ap.add_argument("--secondary-steps", type=int, default=8)
    ap.add_argument("--cpu-baseline-perms", type=int, default=0,
                    help="CPU sample size (0: sized for ~15 s on the host cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--lib", default=None,
                    help="tuning A/B only: another build of libnetrep_amd.so (make OUT=... EXTRA=-D...)")
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--c5-single", action="store_true",
                    help="C5 as one device-resident test dataset on the engine layer (round 2's C5 record) "
                         "instead of three host datasets through the reference interface")
    ap.add_argument("--stamps", action="store_true",
                    help="diagnostic run: per-phase cycle stamps in the profile kernel")
    return ap.parse_args()


def relaunch_if_needed(args):
    """`--gpus N` (N > 1) outside torchrun: start N ranks under
    torch.distributed.run as a child process -- before anything touches the
    GPU -- and exit with its code. Inside torchrun WORLD_SIZE must equal N."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != args.gpus:
            sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}\n")
            sys.exit(2)
        return
    if args.gpus <= 1:
        return
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def setup_dist(args):
    """One process per GPU. The backend is RCCL ("nccl") -- broadcasts over
    xGMI; NETREP_BENCH_BACKEND=gloo runs the same path over gloo (the -m gpu
    test of the sharded HIP path puts two ranks on one GPU that way)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("NETREP_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


scale_rows = S.scale_rows_torch


def build_case(cfg, world, rank, local, seed):
    n_nodes, n_samples, sizes, _, with_data = S.CONFIGS[cfg]
    lay = S.make_layout(n_nodes, sizes, seed)
    dev = torch.device("cuda", local)
    eng = N.Engine(local)
    mods = lay.modules
    node_off = np.concatenate([[0], np.cumsum([lay.members[m].size for m in mods])]).astype(np.int64)
    idx = np.concatenate([lay.members[m] for m in mods]).astype(np.int32)
    # -- discovery vectors (IntermediateProperties on the device), rank 0 then broadcast
    k = np.diff(node_off)
    n_cv = int((k * (k - 1) // 2).sum())
    vec = torch.empty(n_cv + 2 * int(node_off[-1]), dtype=torch.float64, device=dev)
    if rank == 0:
        dx, dc, dn = S.torch_dataset(lay, n_samples, seed + 1, device=dev)
        dxs = scale_rows(dx).contiguous()
        # torch's stream belongs to its own HIP runtime, not ordered with the
        # engine's: the inputs must be complete before the engine reads them
        torch.cuda.synchronize()
        eng.set_dataset_device(dc.data_ptr(), dn.data_ptr(), dxs.data_ptr() if with_data else 0,
                               n_nodes, n_samples)
        del dx, dc, dn, dxs
        torch.cuda.empty_cache()
        v = eng.module_vectors(node_off, idx, with_data)
        parts = [v["corr"], v["degree"], v["contribution"] if with_data else np.zeros(int(node_off[-1]))]
        vec.copy_(torch.from_numpy(np.concatenate(parts)))
    if world > 1:
        dist.broadcast(vec, src=0)
    v = vec.cpu().numpy()
    disc_cv, disc_wd, disc_nc = v[:n_cv], v[n_cv:n_cv + node_off[-1]], v[n_cv + node_off[-1]:]
    # -- test dataset: built on rank 0, broadcast over RCCL (xGMI) to every rank
    if rank == 0:
        tx, tc, tn = S.torch_dataset(lay, n_samples, seed + 2, preserve_all=False, device=dev)
        txs = scale_rows(tx).contiguous()
        del tx
    else:
        txs = torch.empty((n_nodes, n_samples), dtype=torch.float64, device=dev)
        tc = torch.empty((n_nodes, n_nodes), dtype=torch.float64, device=dev)
        tn = torch.empty((n_nodes, n_nodes), dtype=torch.float64, device=dev)
    t_bcast = 0.0
    if world > 1:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        broadcast_tensors([tc, tn, txs], src=0)   # RCCL over xGMI
        torch.cuda.synchronize()
        t_bcast = time.perf_counter() - t0
    torch.cuda.synchronize()
    eng.set_dataset_device(tc.data_ptr(), tn.data_ptr(), txs.data_ptr() if with_data else 0,
                           n_nodes, n_samples)
    eng.set_modules(len(mods), np.arange(len(mods)), node_off, idx, idx,  # null pool = all genes
                    disc_cv, disc_wd, disc_nc if with_data else None)
    eng.set_null_pool(np.arange(n_nodes, dtype=np.int32))
    # the test tensors stay alive until the secondary (network-only) engine is
    # built and, on a single rank, for the CPU baseline sample
    tensors = dict(tc=tc, tn=tn, txs=txs)
    return eng, lay, dict(node_off=node_off, idx=idx, disc_cv=disc_cv, disc_wd=disc_wd,
                          disc_nc=disc_nc, with_data=with_data, n_samples=n_samples,
                          n_nodes=n_nodes, t_bcast=t_bcast, symmetric=eng.symmetric()), tensors


def secondary_engine(local, meta, tensors):
    """Network-only engine (C4: permutationsNoData) on the same resident test
    matrices: the HBM-bound gather kernel as its own driver-timed record."""
    eng = N.Engine(local)
    tc, tn = tensors["tc"], tensors["tn"]
    eng.set_dataset_device(tc.data_ptr(), tn.data_ptr(), 0, meta["n_nodes"], 0)
    n_mod = meta["node_off"].size - 1
    eng.set_modules(n_mod, np.arange(n_mod), meta["node_off"], meta["idx"], meta["idx"],
                    meta["disc_cv"], meta["disc_wd"], None)
    eng.set_null_pool(np.arange(meta["n_nodes"], dtype=np.int32))
    return eng


def roofline_terms(sizes, n_samples, with_data):
    """Algorithmic bytes / flops per permutation, per kernel."""
    k = np.asarray(sizes, dtype=np.float64)
    net_bytes = (4 * k + 8 * k * (k - 1) / 2 + 8 * k * k).sum()
    prof_bytes = (4 * k + 8 * n_samples * k).sum() if with_data else 0.0
    prof_flops = (2 * n_samples * k * np.minimum(n_samples, k)).sum() if with_data else 0.0
    return net_bytes, prof_bytes, prof_flops


def table_bytes(sizes):
    """Algorithmic bytes per permutation of the Gram-table profile kernel:
    one 32-byte table element per pair and per diagonal entry, the column
    sums, the node indices and the discovery correlations (the data block is
    not read: the Gram comes from the table)."""
    k = np.asarray(sizes, dtype=np.float64)
    return (4 * k + 8 * k * (k - 1) / 2 + 32 * k * (k + 1) / 2 + 8 * k).sum()


# The network statistics' launches (timer 0): the column sweep (sweep.hip) --
# each test column streamed into LDS once per batch, every occurrence of the
# column reading its rows there -- so no random-gather ceiling applies; the
# roofline is SURVEY.md 8d's network bytes against HBM peak.
NET_KERNEL = "network_sweep"
# rocprofv3 names of what the engine's two timers measure (timer 0: the
# network launches, timer 1: the summary-profile launches), by path
NET_SYMBOLS = "nr::sweep_column_kernel + sweep_cols/scan/prep/finish_kernel (the column sweep, one batch)"


def profile_symbol(table, sizes, n_samples):
    """The summary-profile kernel a launch of these shapes runs (engine.hip
    plan_profile / table_wanted: one numerical path per shape)."""
    if table:
        return "nr::module_profile_table_kernel"
    if min(max(sizes), n_samples) <= 111:
        return "nr::module_profile_wave_kernel"
    return "nr::module_profile_big_kernel + nr::module_profile_packed4_kernel (the summary-profile launches)"
NET_UNITS = ("achieved = SURVEY.md 8d network bytes 4k + 8k(k-1)/2 + 8k^2 per module-permutation x the "
             "launch's items / HIP-event time of the sweep's five kernels (sweep.hip)")


def time_steps(eng, world, rank, steps, warmup, perms_per_step, seed, base_warm):
    """W untimed warm-up steps, then K steps bracketed by barrier + device
    synchronisation; returns (max-over-ranks seconds, local null chunks, base)."""
    for s_ in range(warmup):
        p0 = base_warm + s_ * perms_per_step
        eng.run(p0, p0 + perms_per_step, seed)
    eng.synchronize()
    eng.set_timing(True)
    eng.reset_timing()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    total = world * steps * perms_per_step
    base, _ = perm_range(rank, world, total)   # this rank's contiguous chunk
    chunks = []
    for s_ in range(steps):
        p0 = base + s_ * perms_per_step
        chunks.append(eng.run(p0, p0 + perms_per_step, seed))
    eng.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, chunks, total


def host_cores():
    """The host CPU as this process sees it: the machine's logical CPUs
    (nproc), the ones this process may run on (affinity), the CPU model, and
    the GPU lease's share of them (OMP_NUM_THREADS, 16 per GPU on the box)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, affinity)
    return {"nproc": os.cpu_count() or 1, "affinity": affinity, "lease_share": share, "model": model}


def cpu_baseline(lay, meta, host, n_perm, seed):
    """The C++ CPU restatement of the reference's path (oracle/netrep_ref.cpp:
    per-thread contiguous permutation chunks as src/permutations.cpp:338-373,
    one null-pool shuffle per permutation, LAPACK dgesvd per module) on a
    bounded sample of the same workload, on every host core of this GPU's
    lease (the box gives a one-GPU command its share of the machine:
    OMP_NUM_THREADS; nproc shows the whole machine)."""
    from oracle import ref_cpp
    hc = host_cores()
    threads = max(1, min(hc["lease_share"], hc["affinity"]))
    tc = host["tc"].cpu().numpy()
    tn = host["tn"].cpu().numpy()
    tx = host["txs"].cpu().numpy().T if meta["with_data"] else None   # S x N view, column-major
    no = meta["node_off"]
    args = dict(n_rows=len(lay.modules), row_of=np.arange(len(lay.modules)), node_off=no,
                test_idx=meta["idx"], null_pos=meta["idx"], null_idx=np.arange(meta["n_nodes"]),
                disc_cv=meta["disc_cv"], disc_wd=meta["disc_wd"],
                disc_nc=meta["disc_nc"] if meta["with_data"] else None, seed=seed, n_threads=threads,
                want_observed=False)
    if n_perm <= 0:   # size the sample for ~15 s of CPU work
        t0 = time.perf_counter()
        ref_cpp.permutation_procedure(tx, tc, tn, n_perm=threads, **args)
        rate = threads / max(time.perf_counter() - t0, 1e-9)      # permutations/s, all threads
        n_perm = int(max(threads, min(100000, 15.0 * rate)))
    t0 = time.perf_counter()
    ref_cpp.permutation_procedure(tx, tc, tn, n_perm=n_perm, **args)
    dt = time.perf_counter() - t0
    return n_perm / dt, dt, n_perm, threads, hc


def run_c5(args, world, rank, local):
    """BASELINE.json configs[4] as stated: 40,000 genes x 1,000 samples,
    modules of geomspace(30, 2000, 40) genes, THREE test datasets,
    null = "all" -- through the reference interface, as modulePreservation
    drives it (one PermutationProcedure per test dataset,
    R/modulePreservation.R:553-635). The discovery modules cover 30,000 of
    the genes; each test dataset holds all 40,000 in its own column order, so
    the "all" pool (the test colnames, src/permutations.cpp:317-323) is larger
    than the module nodes. The test matrices start in host memory (as R holds
    them): dataset t+1 is uploaded by netrep_PrefetchTestDataset while
    dataset t's permutations run. A step = --perms-per-step permutations of
    each of the three datasets; value = permutations / wall time of the
    pipelined loop. Upload alone and compute alone are timed separately."""
    if world != 1:
        raise SystemExit("--config C5 (three test datasets through the reference interface) is a one-GPU run")
    from netrep_amd.api import RMatrix
    n, s, sizes, _, _ = S.CONFIGS["C5"]
    seed = args.seed
    n_disc = 30_000
    rng = np.random.default_rng(seed)
    all_names = [f"G{i}" for i in range(n)]
    disc_pos = np.sort(rng.choice(n, n_disc, replace=False))
    lay_d = S.make_layout(n_disc, sizes, seed)
    d_names = [all_names[i] for i in disc_pos]
    ma = dict(zip(d_names, lay_d.labels))
    modules = lay_d.modules
    dev = torch.device("cuda", local)
    t_setup = time.perf_counter()
    dx, dc, dn = S.torch_dataset(lay_d, s, seed + 1, device=dev)
    dxs = scale_rows(dx).contiguous()
    del dx
    torch.cuda.synchronize()
    eng = N.Engine(local)
    eng.set_dataset_device(dc.data_ptr(), dn.data_ptr(), dxs.data_ptr(), n_disc, s)
    node_off, idx = S.csr_of(lay_d)
    v = eng.module_vectors(node_off, idx, True)
    eng.close()
    del dxs, dc, dn
    torch.cuda.empty_cache()
    disc = {"degree": {}, "corr": {}, "contribution": {}}
    o = ocv = 0
    for m in modules:
        k = lay_d.members[m].size
        disc["degree"][m] = v["degree"][o:o + k]
        disc["contribution"][m] = v["contribution"][o:o + k]
        disc["corr"][m] = v["corr"][ocv:ocv + k * (k - 1) // 2]
        o += k
        ocv += k * (k - 1) // 2
    datasets = []
    for t in range(3):
        order = np.random.default_rng(seed + 10 + t).permutation(n)
        t_names = [all_names[i] for i in order]
        pos_of = {nm: j for j, nm in enumerate(t_names)}
        lay_t = S.Layout(n, sizes, t_names, ["0"] * n, modules,
                         {m: np.sort(np.array([pos_of[d_names[i]] for i in lay_d.members[m]])) for m in modules})
        tx, tc, tn = S.torch_dataset(lay_t, s, seed + 20 + t, preserve_all=(t == 0), device=dev)
        txs = scale_rows(tx)
        del tx
        # host copies, column-major (the matrices are symmetric: the transposed
        # view of the row-major copy is the column-major matrix)
        tcn, tnn = tc.cpu().numpy().T, tn.cpu().numpy().T
        txn = np.asfortranarray(txs.cpu().numpy().T)
        del tc, tn, txs
        torch.cuda.empty_cache()
        datasets.append((RMatrix(txn, None, t_names), RMatrix(tcn, t_names, t_names), RMatrix(tnn, t_names, t_names)))
    t_setup = time.perf_counter() - t_setup
    P = args.perms_per_step or 256
    K, W = args.steps, args.warmup
    n_cores = host_cores()["lease_share"]   # nThreads: the lease's host cores stage the uploads
    N._lib.load().nr_set_host_threads(n_cores)

    # modulePreservation's loop over (step, test dataset), pipelined: the next
    # dataset's upload is started before the current one's permutations
    order = [(k_, t) for k_ in range(-W, K) for t in range(3)]
    N.PrefetchTestDataset(*datasets[0])
    call_s = []
    t0 = None
    for i, (k_, t) in enumerate(order):
        if k_ == 0 and t == 0:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        if i + 1 < len(order):
            N.PrefetchTestDataset(*datasets[order[i + 1][1]])   # uploads while dataset t runs
        tc_ = time.perf_counter()
        last = N.PermutationProcedure(disc, *datasets[t], ma, modules, P, nCores=n_cores, nullHypothesis="all",
                                      seed=seed + 1000 * k_ + t)
        if k_ >= 0:
            call_s.append(round(time.perf_counter() - tc_, 4))
    elapsed = time.perf_counter() - t0
    finite = float(np.isfinite(last["nulls"]).mean())
    # upload alone (pinned double-buffered chunks, 25.9 GB per dataset) and
    # compute alone (dataset resident) on one dataset, engine layer
    x, c, nt = datasets[0]
    e2 = N.Engine(local)
    t1 = time.perf_counter()
    e2.set_dataset(c.f, nt.f, x.f)
    upload_s = time.perf_counter() - t1
    names0 = list(nt.colnames)
    pos0 = {nm: j for j, nm in enumerate(names0)}
    idx_t = np.concatenate([[pos0[d_names[i]] for i in lay_d.members[m]] for m in modules]).astype(np.int32)
    e2.set_modules(len(modules), np.arange(len(modules)), node_off, idx_t, idx_t, v["corr"], v["degree"],
                   v["contribution"])
    e2.set_null_pool(np.arange(n, dtype=np.int32))
    e2.run(0, 8, seed)
    e2.synchronize()
    e2.set_timing(True)
    e2.reset_timing()
    t1 = time.perf_counter()
    e2.run(0, P, seed)
    e2.synchronize()
    compute_s = time.perf_counter() - t1
    ms0, l0, _ = e2.timing(0)
    ms1, l1, _ = e2.timing(1)
    diag = e2.diagnostics()
    e2.close()
    _, prof_b, prof_f = roofline_terms(sizes, s, True)
    total = 3 * P * K
    line = {
        "metric": f"permutations/sec (whole node), {n // 1000}k genes x {len(sizes)} modules, 3 test datasets",
        "value": total / elapsed, "unit": "permutations/sec", "n_gpus": 1, "steps": K, "warmup": W,
        "ms_per_step": elapsed / K * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic coexpression (SURVEY.md 8d generator), random module layout",
        "config": {"workload": f"C5: {n} genes x {s} samples, {len(sizes)} modules ({min(sizes)}-{max(sizes)} genes, "
                               f"discovery over {n_disc} genes), 3 test datasets of {n} genes each in host memory, "
                               f"null=all (pool = the {n} test genes), 7 statistics, "
                               f"netrep_PermutationProcedure per dataset with netrep_PrefetchTestDataset",
                   "perms_per_step": 3 * P, "perms_per_dataset_per_step": P, "parallelism": "perm-shard x1"},
        "upload_s_per_dataset": upload_s,
        "upload_GBps": (2 * n * n + s * n) * 8 / upload_s / 1e9,
        "compute_s_per_dataset": compute_s,
        "compute_perms_per_sec": P / compute_s,
        "pipelined_s_per_dataset": elapsed / (3 * K),
        "call_s": call_s,
        "kernels": {NET_KERNEL: {"avg_ms": ms0 / max(l0, 1), "launches": l0},
                    "module_profile_kernel": {"avg_ms": ms1 / max(l1, 1), "launches": l1,
                                              "achieved": prof_f * P / (ms1 * 1e-3) / 1e12 if ms1 > 0 else None,
                                              "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s"}},
        "finite_fraction": finite, "setup_s": t_setup, "eigen_diagnostics": diag,
    }
    mk = line["kernels"]["module_profile_kernel"]
    if mk["achieved"] is not None:
        mk["frac"] = mk["achieved"] / mk["peak"]
    # the dominant kernel (the summary-profile launches of one batch: the
    # large modules' Gram executes on the matrix cores)
    b_launch = int(round(P / max(l1, 1)))
    if mk["achieved"] is not None:
        avg1 = ms1 / max(l1, 1)
        line["roofline"] = {"kernel": profile_symbol(False, sizes, s), "timer": "module_profile_kernel",
                            "bound": "mfma", "achieved": round(mk["achieved"], 4),
                            "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s", "frac": round(mk["frac"], 6),
                            "avg_ms": avg1, "algorithmic_bytes": round(prof_b * b_launch),
                            "launch_permutations": b_launch,
                            "units_note": "achieved = SURVEY.md 8d Gram flops F(k) = 2 S k min(S,k) per "
                                          "module-permutation x the launch's items / HIP-event launch time"}
        line["roofline"].update(traffic_fields("C5", b_launch, "module_profile_kernel", avg1))
        line["roofline"]["traffic_unit"] = ("L2-miss bytes/launch incl. Infinity Cache hits (rocprofv3 FETCH_SIZE "
                                            "x2 + WRITE_SIZE; traffic_range = [raw, x2]; profiles/pmc_traffic.json)")
        line["roofline"]["executed"] = measured_mfma("C5", b_launch, "module_profile_kernel", avg1)
    cpu = None
    if not args.no_cpu_baseline:
        # the C++ restatement on the same resident-dataset index sets (dataset 0,
        # null = "all": the pool is every test gene), one permutation per thread
        from oracle import ref_cpp
        hc = host_cores()
        threads = max(1, min(hc["lease_share"], hc["affinity"]))
        n_cpu = args.cpu_baseline_perms or threads
        t1 = time.perf_counter()
        ref_cpp.permutation_procedure(x.f, c.f, nt.f, len(modules), np.arange(len(modules)), node_off, idx_t, idx_t,
                                      np.arange(n), v["corr"], v["degree"], v["contribution"], n_cpu, seed=seed,
                                      n_threads=threads, want_observed=False)
        dt = time.perf_counter() - t1
        cpu = {"value": n_cpu / dt, "unit": "permutations/sec", "cores": threads, "kind": "port",
               "per_core": n_cpu / dt / threads,
               "host": {"cpu_model": hc["model"], "nproc": hc["nproc"], "affinity": hc["affinity"],
                        "lease_share": hc["lease_share"], "whole_host_estimate": n_cpu / dt / threads * hc["nproc"]},
               "sample": f"{n_cpu} permutations x {len(modules)} modules of test dataset 0 in {dt:.1f} s: C++ "
                         f"restatement of src/permutations.cpp (std::thread chunks, LAPACK SVD), {threads} threads"}
    line["cpu_baseline"] = cpu
    print(json.dumps(line))


def main():
    args = parse()
    if args.lib:
        N._lib.LIB_PATH = os.path.abspath(args.lib)
    relaunch_if_needed(args)
    world, rank, local = setup_dist(args)
    if args.config == "C5" and not args.c5_single:
        run_c5(args, world, rank, local)
        return
    eng, lay, meta, tensors = build_case(args.config, world, rank, local, args.seed)
    B, K, W = args.batch, args.steps, args.warmup
    P = args.perms_per_step or max(5120, B)
    eng.set_batch(B)
    net_b, prof_b, prof_f = roofline_terms(lay.module_sizes, meta["n_samples"], meta["with_data"])
    n_cfg, s_cfg, sizes_cfg, _, _ = S.CONFIGS[args.config]

    eng2 = None
    if not args.no_secondary and meta["with_data"] and args.config == "C3":
        eng2 = secondary_engine(local, meta, tensors)
    host = tensors if (rank == 0 and world == 1) else None
    if host is None:
        del tensors
    torch.cuda.empty_cache()

    if args.stamps:
        eng.set_stamps(True)
    elapsed, chunks, total_perms = time_steps(eng, world, rank, K, W, P, args.seed, 10**12 + rank * W * P)
    ms0, l0, _ = eng.timing(0)
    ms1, l1, _ = eng.timing(1)
    diag = eng.diagnostics()
    if args.stamps:
        diag["stamps_cycles"] = eng.stamps()
    local_cube = np.concatenate(chunks, axis=2)
    del chunks
    cube = gather_nulls(local_cube, rank, world, total_perms) if world > 1 else local_cube
    finite = float(np.isfinite(cube).mean()) if rank == 0 else None
    del cube, local_cube

    # -- secondary record: network-only (C4) on the same matrices ---------------
    secondary = None
    if eng2 is not None:
        # C4's own launch size (5,120 permutations: the committed PMC pass of
        # the sweep, profiles/pmc_traffic.json, is of this launch)
        B2 = 5120
        P2 = 4 * B2
        eng2.set_batch(B2)
        el2, ch2, tot2 = time_steps(eng2, world, rank, args.secondary_steps, 1, P2, args.seed + 1,
                                    2 * 10**12 + rank * P2)
        ms2, l2, _ = eng2.timing(0)
        fin2 = float(np.isfinite(np.concatenate(ch2, axis=2)).mean())
        del ch2
        if rank == 0:
            t2 = ms2 / max(l2, 1) / 1e3
            secondary = {
                "metric": "permutations/sec (whole node), network-only path (permutationsNoData), "
                          f"{n_cfg // 1000}k nodes x {len(lay.modules)} modules",
                "config": "C4 (BASELINE.json configs[3]) on the same resident 20k-gene matrices",
                "value": tot2 / el2, "unit": "permutations/sec", "steps": args.secondary_steps,
                "perms_per_step": P2, "launch_batch": B2, "ms_per_step": el2 / args.secondary_steps * 1e3,
                "finite_fraction": fin2,
                "roofline": {"kernel": NET_SYMBOLS, "timer": NET_KERNEL, "bound": "hbm", "avg_ms": ms2 / max(l2, 1),
                             "achieved": net_b * B2 / t2 / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": net_b * B2 / t2 / 1e9 / HBM_PEAK_GBS,
                             "algorithmic_bytes": round(net_b * B2), "units_note": NET_UNITS},
            }
            secondary["roofline"].update(traffic_fields("C4", B2, NET_KERNEL, ms2 / max(l2, 1)))
        eng2.close()

    if rank == 0:
        value = total_perms / elapsed
        # dominant kernel + roofline (per launch = one batch of B permutations)
        kernels = {}
        fused = meta["with_data"] and l0 == 0   # network statistics computed inside the profile kernel
        if l0 > 0:
            t0 = ms0 / l0 / 1e3
            kernels[NET_KERNEL] = {
                "bound": "hbm", "avg_ms": ms0 / l0, "launches": l0,
                "achieved": net_b * B / t0 / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "algorithmic_bytes": round(net_b * B), "units_note": NET_UNITS}
        table = meta["with_data"] and eng.gram_table()
        if table:
            # Gram table: every statistic of a module-permutation in this one
            # launch -- network values and the packed Gram from one 32-byte
            # table gather per pair, then the Lanczos eigenpair. The kernel
            # executes no MFMA (its Gram comes from the per-dataset table), so
            # it is a memory kernel: the primary figure is SURVEY.md 8d's
            # algorithmic bytes B(k) per launch against HBM peak; the Gram
            # flops F(k) the table serves stay as a secondary figure.
            t1 = ms1 / max(l1, 1) / 1e3
            tab_b = table_bytes(lay.module_sizes)
            kernels["module_profile_kernel"] = {
                "bound": "hbm", "avg_ms": ms1 / max(l1, 1), "launches": l1,
                "achieved": (net_b + prof_b) * B / t1 / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "algorithmic_bytes": round((net_b + prof_b) * B),
                "units_note": "achieved = SURVEY.md 8d algorithmic bytes B(k) = 4k + 8k(k-1)/2 + 8k^2 + 8Sk per "
                              "module-permutation x the launch's items / HIP-event launch time",
                "gram_table": True, "fused_network_statistics": fused,
                "f_units": {"achieved": prof_f * B / t1 / 1e12, "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                            "frac": prof_f * B / t1 / 1e12 / FP64_MFMA_PEAK_TFS,
                            "note": "secondary: SURVEY.md 8d Gram flops F(k) = 2 S k min(S,k) per module-permutation "
                                    "/ launch time; served by the dataset's Gram table (2 S n^2 flops once per "
                                    "dataset), not executed per item (executed MFMA: roofline.executed)"},
                "table_gather_bytes": {"achieved": tab_b * B / t1 / 1e9, "unit": "GB/s",
                                       "note": "32-byte table element per pair and diagonal entry + indices + "
                                               "discovery vectors, the bytes this kernel's gathers need"},
                "table_build_ms": eng.gram_table_ms(),
                "table_build_note": "one-off per test dataset, in the first (warm-up) run: X^T X on the "
                                    "matrix cores + the widened {corr, net, gram, net^T} layout; outside "
                                    "the timed steps like the dataset upload (it is "
                                    f"{eng.gram_table_ms() / (elapsed * 1e3) * 100:.2f}% of this run's timed region)"}
        elif meta["with_data"]:
            t1 = ms1 / max(l1, 1) / 1e3
            kernels["module_profile_kernel"] = {
                "bound": "mfma", "avg_ms": ms1 / max(l1, 1), "launches": l1,
                "achieved": prof_f * B / t1 / 1e12, "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                "fused_network_statistics": fused,
                "units_note": "achieved = SURVEY.md 8d Gram flops F(k) = 2 S k min(S,k) per module-permutation "
                              "x the launch's items / HIP-event launch time (executed on the matrix cores)",
                "algorithmic_bytes": round(((net_b if fused else 0.0) + prof_b) * B),
                "hbm_achieved_GBps": ((net_b if fused else 0.0) + prof_b) * B / t1 / 1e9}
        for kv in kernels.values():
            kv["frac"] = kv["achieved"] / kv["peak"]
        dom_name = max(kernels, key=lambda n: kernels[n]["avg_ms"])
        dom = kernels[dom_name]
        symbol = (NET_SYMBOLS if dom_name == NET_KERNEL
                  else profile_symbol(bool(table), lay.module_sizes, meta["n_samples"]))
        roofline = {"kernel": symbol, "timer": dom_name, "bound": dom["bound"], "achieved": round(dom["achieved"], 4),
                    "peak": dom["peak"], "unit": dom["unit"], "frac": round(dom["frac"], 6),
                    "avg_ms": dom["avg_ms"], "algorithmic_bytes": dom["algorithmic_bytes"],
                    "units_note": dom.get("units_note")}
        roofline.update(traffic_fields(args.config, B, dom_name, dom["avg_ms"], bool(table)))
        roofline["traffic_unit"] = ("L2-miss bytes/launch incl. Infinity Cache hits (rocprofv3 FETCH_SIZE x2 + "
                                    "WRITE_SIZE; traffic_range = [raw, x2]; profiles/pmc_traffic.json)")
        if table and dom_name == "module_profile_kernel":
            for key in ("gram_table", "f_units", "table_build_ms"):
                roofline[key] = dom[key]
        roofline["executed"] = measured_mfma(args.config, B, dom_name, dom["avg_ms"], bool(table))
        cpu = None
        if world == 1 and not args.no_cpu_baseline and host is not None:
            rate, dt, n_cpu, threads, hc = cpu_baseline(lay, meta, host, args.cpu_baseline_perms, args.seed)
            cpu = {"value": rate, "unit": "permutations/sec", "cores": threads, "kind": "port",
                   "per_core": rate / threads,
                   "host": {"cpu_model": hc["model"], "nproc": hc["nproc"], "affinity": hc["affinity"],
                            "lease_share": hc["lease_share"],
                            "whole_host_estimate": rate / threads * hc["nproc"],
                            "whole_host_estimate_note": "per-core rate x nproc (linear; the reference's "
                                                        "threads are independent, src/permutations.cpp:338-373)"},
                   "sample": f"{n_cpu} permutations x {len(lay.modules)} modules of the same workload in "
                             f"{dt:.1f} s: C++ restatement of src/permutations.cpp (std::thread chunks, "
                             f"LAPACK SVD), {threads} threads = every core of this GPU's lease "
                             f"({hc['nproc']}-CPU host: {hc['model']})"}
        null_desc = "all" if args.config == "C5" else "overlap"
        line = {
            "metric": f"permutations/sec (whole node), {n_cfg // 1000}k genes x {len(sizes_cfg)} modules"
                      + ("" if meta["with_data"] else " (network only)"),
            "value": value,
            "unit": "permutations/sec",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic coexpression (SURVEY.md 8d generator), random module layout",
            "config": {"workload": f"{args.config}: {meta['n_nodes']} genes x {meta['n_samples']} samples, "
                                   f"{len(lay.modules)} modules ({min(lay.module_sizes)}-{max(lay.module_sizes)} genes), "
                                   f"null={null_desc} (pool = every gene), "
                                   f"{'7' if meta['with_data'] else '4'} statistics",
                       "perms_per_step": P, "launch_batch": B, "global_perms": total_perms,
                       "parallelism": f"perm-shard x{world}"},
            "module_perms_per_sec": value * len(lay.modules),
            # the Gram table's one-off build (first, untimed run) charged to
            # this run's timed region: what `value` would be with it inside
            "value_incl_table_build": (total_perms / (elapsed + eng.gram_table_ms() / 1e3)
                                       if table else None),
            "algorithmic_GBps": value * (net_b + prof_b) / 1e9,
            "roofline": roofline,
            "kernels": kernels,
            "cpu_baseline": cpu,
            "secondary": secondary,
            "finite_fraction": finite,
            "broadcast_s": meta["t_bcast"],
            "symmetric_matrices": meta["symmetric"],
            "eigen_diagnostics": diag,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
