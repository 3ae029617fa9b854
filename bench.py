"""Benchmark of the hot path: per-layer pairwise distance + Vietoris-Rips
persistence H0-H2 (BASELINE.json metric "layers/sec ... at 1/2/4/8 MI355X").

A step = one pass of the hot path over one 32-layer sweep, diagrams returned
to the host:
  * primary (``value``, SURVEY 8(d) as written): ``sweep48_host`` -- the
    reference's 32-layer sweep (debug_tda_pipeline.py:92-150) of 48-point
    clouds, configs[1] per layer (48 points, D=3, H0-H2), host numpy array in,
    every layer's ``dgms`` list materialised on the host; each step submits a
    DIFFERENT sweep (8 noise seeds of the generator, rotated);
  * ``workloads`` (N=1 only): the same sweep HBM-resident (``sweep48``),
    configs[4] grid144, configs[3] torus1024, the top of the N range, the
    drop-in ``ripser()`` call itself at the reference's N = 36 and the
    adversarial N = 324 (``ripser36`` / ``ripser324``), each with its own
    roofline and CPU baseline.
Multi-GPU: one process per GPU (torchrun).  ``--scaling weak`` (default):
every rank runs its own 32-layer sweeps; ``strong``: the 32 layers are sharded
(configs[2]: 4 layers/GPU at 8 GPUs).  Either way a step ends with the one
gather of per-layer records to rank 0 (distributed.sharded_sweep_step); at
N > 1 a strong-scaling record is added next to the weak one, the CPU baseline
is measured by the launching process before any rank touches a GPU, and rank 0
runs the stage pass that gives the line its roofline.

CPU baseline: the oracle (oracle/rips_oracle.c, a C restatement of the
ripser semantics; "kind": "port") on the same inputs, 1 core and P worker
processes (the host CPUs this job may use: 16 per GPU, the whole host at
8 GPUs), on bounded samples.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import glob
import importlib
import json
import math
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
FP64_MFMA_PEAK_TFS = 78.6  # MI355X FP64 matrix peak (vendor spec; v_mfma_f64_16x16x4_f64)
METRIC = "layers/sec (pairwise-dist + VR persistence H0-H2) at 1/2/4/8 MI355X"

WORKLOADS = {
    # name: (layers, maxdim, description, default steps, default warmup)
    "sweep48": (32, 2, "qwen-vl 32-layer sweep x 48 points (configs[1] per layer), D=3, H0-H2", 400, 5),
    "grid144": (32, 2, "12x12 torus grid x 32 layers (configs[4]), N=144, D=3, H0-H2", 30, 2),
    "torus1024": (1, 1, "S1xS1 torus N=1024 (configs[3]), D=3, H0-H1", 5, 2),
    # configs[3]'s cloud as a sweep: 32 tori (seeds 0..31) per call, like the reference's 32-layer loop --
    # the GPU's layers in flight against the CPU baseline's layers in flight (one per worker process)
    "torus1024x32": (32, 1, "32 S1xS1 tori N=1024 (configs[3]'s cloud, seeds 0-31) per call, D=3, H0-H1", 3, 1),
    # four sweeps per call (128 layers): the same per-layer work, a larger batch -- the
    # latency-bound 32-layer step leaves most CUs idle (throughput capacity, not the headline)
    "sweep48x4": (128, 2, "4 x the qwen-vl 32-layer sweep x 48 points in one call (128 layers), D=3, H0-H2", 50, 5),
    # SURVEY 8(d) as written: host numpy array in, every layer's dgms list materialised on the host in the timed loop
    "sweep48_host": (32, 2, "qwen-vl 32-layer sweep x 48 points, D=3, H0-H2: numpy (32, 48, 3) in, per-layer dgms lists out "
                            "(host-array-in -> diagrams-on-host-out, debug_tda_pipeline.py:104-110)", 400, 5),
    # configs[2]'s per-GPU share: 4 of the 32 layers in one call (8 GPUs, strong scaling)
    "sweep48_L4": (4, 2, "4 layers x 48 points per call (configs[2]'s per-GPU share at 8 GPUs), D=3, H0-H2", 100, 10),
    # configs[1] as written: one 48-point layer per call, H0-H2, one call at a time (per-call latency)
    "sweep48_L1": (1, 2, "1 layer x 48 points per call (configs[1]), D=3, H0-H2, one call at a time", 200, 10),
    # the top of north_star's N range (N = 48-2048): one layer per call, as configs[3] at N = 1024
    "torus2048": (1, 1, "S1xS1 torus N=2048 (top of the north_star N range), D=3, H0-H1, one layer per call", 3, 1),
    # ... and at maxdim 2 with ripser's thresh (tests/golden/large_h2_2048.npz, torus2048_t12)
    "torus2048_h2": (1, 2, "S1xS1 torus N=2048, D=3, H0-H2 at thresh=1.2 (ripser's thresh argument; "
                           "tests/golden/large_h2_2048.npz torus2048_t12), one layer per call", 3, 1),
    # raw hidden states (no UMAP): distance on the FP64 matrix cores + TwoNN + H0
    "raw4096": (32, 0, "32 layers x 144 tokens x 4096 raw hidden-state features: distance (FP64 MFMA) + H0 + TwoNN "
                       "intrinsic dimension (metrics.py:113-208)", 100, 3),
    # the drop-in itself at the reference's own call: ripser(cloud, maxdim=1) once per layer, numpy (N, 3) f32 in,
    # the full ripser.py dict out (dgms, num_edges, dperm2all, ...), one call at a time (debug_tda_pipeline.py:109-110)
    "ripser36": (32, 1, "ripser(cloud, maxdim=1) per layer on the reference's 32 committed UMAP clouds (N=36, D=3), "
                        "one call per layer, full dict out (debug_tda_pipeline.py:109-110)", 10, 2),
    # ... and at the adversarial experiment's N = 324 (analyze_adversarial_tda.py:100)
    "ripser324": (32, 1, "ripser(cloud, maxdim=1) per layer on 32 UMAP clouds of 324 prompts (N=324, D=3; "
                         "analyze_adversarial_tda.py:100), one call per layer, full dict out", 5, 1),
}
DATA = {
    "sweep48": "synthetic: reference UMAP clouds (tda-output/point_clouds_3d) resampled to 48 points + noise",
    "sweep48_host": "synthetic: reference UMAP clouds (tda-output/point_clouds_3d) resampled to 48 points + noise",
    "sweep48_L4": "synthetic: reference UMAP clouds (tda-output/point_clouds_3d) resampled to 48 points + noise",
    "sweep48x4": "synthetic: reference UMAP clouds (tda-output/point_clouds_3d) resampled to 48 points + noise",
    "grid144": "synthetic: 12x12 grid on the torus + N(0, 0.02^2) + random rotation per layer",
    "torus1024": "synthetic: uniform angles on S1 x S1 (R=2, r=1), seed 0",
    "torus1024x32": "synthetic: uniform angles on S1 x S1 (R=2, r=1), seeds 0-31",
    "sweep48_L1": "synthetic: reference UMAP clouds (tda-output/point_clouds_3d) resampled to 48 points + noise",
    "torus2048": "synthetic: uniform angles on S1 x S1 (R=2, r=1), seed 3",
    "torus2048_h2": "synthetic: uniform angles on S1 x S1 (R=2, r=1), seed 3",
    "raw4096": "synthetic: activation-like f32 clouds (heavy-tailed feature scales, offsets, outlier features)",
    "ripser36": "the reference's own 32 UMAP clouds (tda-output/point_clouds_3d, tests/golden/reference_clouds.npz)",
    "ripser324": "synthetic: this build's umap_batch (cosine, n_neighbors 6, 3 components) of 18 x 18 two-factor activation "
                 "clouds (tests/golden/adv_clouds.npz, tools/make_adv_clouds.py)",
}
NPOINTS = {"torus1024x32": 1024, "sweep48": 48, "sweep48x4": 48, "sweep48_host": 48, "sweep48_L4": 48, "sweep48_L1": 48,
           "grid144": 144, "torus1024": 1024, "raw4096": 144, "torus2048": 2048, "torus2048_h2": 2048, "ripser36": 36,
           "ripser324": 324}
DIMS = {w: (4096 if w == "raw4096" else 3) for w in WORKLOADS}  # point dimension D of each workload (make_workload)
CALL_KW = {"raw4096": {"twonn": True}, "torus2048_h2": {"thresh": 1.2}}
# dynamic batching of consecutive steps (ripser.SweepPipeline): every step submits one 32-layer sweep;
# up to `coalesce` queued sweeps run as one call over their concatenated layers and `depth` calls are in
# flight on separate workspace slots, one stream (hardware queue) each.  The dense N <= 64 path is a
# chain of latency-bound kernels that leaves most of the 256 CUs idle; wider calls and several calls in
# flight fill them (r04, tools/ab_coalesce.sh: 148 K layers/s one call at a time -> 217 K coalescing 4,
# 305 K with 2 in flight, 455 K with 4; after the r04 kernel changes 4 x 4: 445-488 K, 4 x 8: 580 K,
# 6 x 4: 578 K).  Every record also carries the one-call-at-a-time figure
# (pipeline.sequential).  sweep48_L4 stays one call at a time: it is the per-call latency record.
# grid144 (parallel reducer) and raw4096 (distance + H0 + TwoNN) gain from calls in flight but not from wider
# calls (r04: grid144 5.60 K -> 7.54 K layers/s with 3 in flight, 7.87 K with 4; raw4096 120 K -> 148 K with 4).
# r06, after the host side moved to C (_hostviews): sweep48_host at 400 steps, 15 interleaved repeats
# (tools/short_run.py, profiles/r06_steady_shapes_b.txt): 4 x 8 581 K, 5 x 8 579 K, 6 x 6 617 K, 8 x 8 655 K,
# 6 x 8 667 K; at the driver's 20 steps 6 x 4 and 4 x 5 tie (414 / 409 K, profiles/r06_short_run_20steps.txt).
PIPE = {"sweep48": (6, 8), "sweep48_host": (6, 8), "sweep48_L4": (1, 1), "sweep48_L1": (1, 1), "grid144": (4, 1),
        "raw4096": (4, 1), "torus1024x32": (1, 1)}  # workload -> (depth, coalesce); (1, 1): one call at a time (env A/B only)
def pipe_shape(name: str, steps: int) -> tuple:
    """(depth, coalesce) of a workload's timed loop: its PIPE row, with fewer
    sweeps per call when the run is short -- the K timed steps include the
    pipeline's fill and drain, so a short run puts all its steps into one wave
    of `depth` calls (r04, sweep48 at --steps 20, tools/ab_k20.sh: 4 x 8
    305-324 K layers/s; 4 x 4 mean 354 K over 5 runs; 4 x 5 mean 378 K).
    TDA_BENCH_DEPTH / TDA_BENCH_COALESCE override (A/B runs)."""
    if name not in PIPE:
        return 1, 1
    depth, coalesce = PIPE[name]
    if steps < 32 * depth:
        coalesce = min(coalesce, max(1, -(-steps // depth)))
    return int(os.environ.get("TDA_BENCH_DEPTH", depth)), int(os.environ.get("TDA_BENCH_COALESCE", coalesce))


# workloads whose layers are the same clouds as another's: one CPU baseline serves both
CPU_SAME = {"sweep48": "sweep48_host", "sweep48_L4": "sweep48_host", "sweep48x4": "sweep48_host", "sweep48_L1": "sweep48_host"}
# distinct sweeps per step: step i runs sweep i % K -- K noise seeds of the same generator
# (synthetic.sweep48 / sweep144 `variant`), so no step resubmits the previous step's array.  K = 8 keeps a
# slot's captured graphs (one per device input address without parts) well under its limit of 16.
ROTATE = {w: 8 for w in ("sweep48", "sweep48_host", "sweep48_L4", "sweep48_L1", "sweep48x4", "grid144")}


def algo_bytes_per_layer(n: int, d: int, maxdim: int) -> int:
    """B = 4ND + 4C(N,2) + sum_{k=1..maxdim} 12 C(N,k+1)."""
    return 4 * n * d + 4 * math.comb(n, 2) + sum(12 * math.comb(n, k + 1) for k in range(1, maxdim + 1))


def mfma_executed(n: int, d: int, L: int, ms: float) -> dict:
    """The FP64 Gram kernels execute only the 16x16 output blocks on or above
    the block diagonal (nb (nb + 1) / 2 of nb^2, nb = ceil(N / 16)): the
    matrix-core utilisation on the flops actually issued, next to the
    algorithmic 2 N^2 D figure (PMC SQ_INSTS_VALU_MFMA_F64 x 2048 agrees,
    profiles/r03_pmc_mfma.json)."""
    nb = -(-n // 16)
    ex = nb * (nb + 1) // 2 * 16 * 16 * 2 * d
    tf = ex * L / (ms * 1e-3) / 1e12
    return {"executed_flops_per_layer": ex, "achieved_executed": tf, "frac_executed": tf / FP64_MFMA_PEAK_TFS}


# The >= 20x bar of north_star, one stated CPU comparison per workload: a
# single-layer call (configs[3], C4) against one CPU core running that layer
# (the reference runs one ripser call per layer and ripser is single-threaded);
# a sweep (many independent layers per step) against the CPU running its
# layers in parallel, one per worker process (P processes, the box's CPU share).
BAR_BASIS = {"torus1024": "one_core", "torus2048": "one_core", "torus2048_h2": "one_core", "sweep48_L1": "one_core",
             "ripser36": "one_core", "ripser324": "one_core"}


def speedups(value: float, cb: dict, name: str) -> dict:
    basis = BAR_BASIS.get(name, "all_cores")
    sp = {"all_cores": value / cb["value"], "one_core": value / cb["value_1core"],
          "all_cores_extrapolated": value / cb["value_all_cores_extrapolated"]}
    sp["bar_20x"] = {"basis": basis, "basis_note": ("one GPU call on one layer vs one CPU core on that layer"
                                                    if basis == "one_core" else
                                                    f"the GPU sweep vs the CPU running {cb['cores']} layers at once "
                                                    f"({cb['cores']} worker processes)"),
                     "ratio": sp[basis], "met": sp[basis] >= 20.0}
    return sp


def make_workload(name: str, layers: int | None = None, variant: int = 0):
    syn = importlib.import_module("tda-multimodal_amd.synthetic")
    L = layers or WORKLOADS[name][0]
    if name in ("sweep48", "sweep48x4", "sweep48_host", "sweep48_L4", "sweep48_L1"):
        return syn.sweep48(L, variant)
    if name == "grid144":
        return syn.sweep144(L, variant)
    if name == "ripser36":
        return syn.reference_clouds()[:L]
    if name == "ripser324":
        z = np.load(os.path.join(ROOT, "tests", "golden", "adv_clouds.npz"))
        return z["n324"][:L].astype(np.float32)
    if name == "torus1024":
        return syn.torus(1024)[None].repeat(L, 0)
    if name == "torus1024x32":
        return np.stack([syn.torus(1024, seed=s) for s in range(L)])
    if name in ("torus2048", "torus2048_h2"):
        return syn.torus(2048, seed=3)[None].repeat(L, 0)
    if name == "raw4096":
        return syn.activations(L, 144, 4096)
    raise ValueError(name)


def workload_sweeps(name: str, layers: int | None = None) -> list:
    """The sweeps a workload's steps rotate through (ROTATE; one otherwise)."""
    return [make_workload(name, layers, v) for v in range(ROTATE.get(name, 1))]


def workload_layers(name: str, layers: int | None = None) -> np.ndarray:
    """Every layer the workload's steps run, concatenated (the CPU baseline's inputs)."""
    return np.concatenate(workload_sweeps(name, layers))


# ---------------------------------------------------------------- CPU baseline
_WORKER_CACHE: dict = {}


def _cpu_layers(task):
    """Worker process: the oracle on layers [lo, hi) of a workload."""
    name, lo, hi, maxdim = task
    from oracle import oracle

    if name not in _WORKER_CACHE:
        _WORKER_CACHE[name] = workload_layers(name)
    X = _WORKER_CACHE[name]
    oracle.lib()
    if hi > lo:
        if CALL_KW.get(name, {}).get("twonn"):  # distances + TwoNN restatement (H0 is negligible next to them)
            from oracle import twonn

            for x in X[lo:hi]:
                twonn.twonn_from_dist(oracle.distances(x))
        else:
            oracle.rips_batch_f32(X[lo:hi], maxdim, thresh=CALL_KW.get(name, {}).get("thresh", np.inf))
    return hi - lo


def cpu_info() -> dict:
    model = ""
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {"nproc": os.cpu_count(), "affinity": aff, "cpu_model": model}


def cpu_workers() -> int:
    """CPUs this job may use: the affinity set, at most 16 (a one-GPU box's share)."""
    if os.environ.get("TDA_CPU_WORKERS"):
        return max(1, int(os.environ["TDA_CPU_WORKERS"]))
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(aff, 16))


def cpu_baseline(pool, P: int, name: str, X, maxdim: int, seconds: float) -> dict:
    """The oracle on the workload's layers: 1 core in this process, then P
    worker processes with one layer per task, each for about `seconds`."""
    from oracle import oracle

    oracle.lib()
    L = X.shape[0]
    _WORKER_CACHE[name] = X
    done, t1 = 0, 0.0
    t0 = time.perf_counter()
    while t1 < seconds and done < 100000:
        _cpu_layers((name, done % L, done % L + 1, maxdim))
        done += 1
        t1 = time.perf_counter() - t0
    one = done / t1
    n_tasks = max(P, int(seconds * P * one))  # ~`seconds` of work per worker
    tasks = [(name, i % L, i % L + 1, maxdim) for i in range(n_tasks)]
    t0 = time.perf_counter()
    got = sum(pool.imap_unordered(_cpu_layers, tasks, chunksize=max(1, n_tasks // (8 * P))))
    tp = time.perf_counter() - t0
    nproc = os.cpu_count() or P
    # SURVEY 8(d) asks for P = os.cpu_count() worker processes.  On the GPU box that is the whole
    # machine (256 CPUs shared by 8 GPU jobs; this job's share is 16), so P = 16 is measured and the
    # all-CPU figure is the measured per-process rate scaled linearly to nproc -- an upper bound
    # (no memory-bandwidth or SMT contention), labelled as an extrapolation.
    return {"value": got / tp, "unit": "layers/s", "cores": P, "kind": "port", "value_1core": one,
            "value_all_cores_extrapolated": got / tp * nproc / P, "nproc": nproc,
            "sample": f"{got} layers on {P} worker processes ({tp:.1f} s) and {done} layers on 1 core ({t1:.1f} s): "
                      f"oracle/rips_oracle.c (C restatement of the ripser semantics, -O3), same inputs ({name}); "
                      f"value_all_cores_extrapolated = the {P}-process rate x {nproc}/{P} (not measured)"}


# ---------------------------------------------------------------- GPU measurement
def _timed_steps(pkg, torch, Xs, maxdim, kw, steps, warmup, depth, host_in, dev_index, coalesce=1):
    """K steps (sequential, or through ripser.SweepPipeline: `depth` calls in flight on separate
    workspace slots, each call covering up to `coalesce` consecutive steps' sweeps) between two
    syncs; step i runs sweep Xs[i % len(Xs)].  Returns (elapsed s, device ms per step)."""
    import collections

    dev_ms = []
    K = len(Xs)

    def done(res, info):
        if host_in:  # debug_tda_pipeline.py:110: dgms = result['dgms'] for every layer
            for r in res:
                r.dgms
        dev_ms.append(info["device_ms"] / info.get("coalesced", 1))

    if depth <= 1 and coalesce <= 1:
        for i in range(max(warmup, K)):  # every input address once (a device input's graph is keyed by it)
            pkg.ripser_batch(Xs[i % K], maxdim=maxdim, **kw)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            done(*pkg.ripser_batch(Xs[i % K], maxdim=maxdim, return_time=True, **kw))
        torch.cuda.synchronize()
        return time.perf_counter() - t0, dev_ms
    inflight = depth * coalesce  # steps submitted and not yet waited on
    with pkg.SweepPipeline(depth=depth, device=dev_index, coalesce=coalesce, maxdim=maxdim, return_time=True, **kw) as pipe:
        n_warm = max(max(warmup, 1) * inflight, K * depth)  # every slot captures its graphs (and sees every input)
        for f in [pipe.submit(Xs[i % K]) for i in range(n_warm)]:
            f.result()
        torch.cuda.synchronize()
        dev_ms.clear()
        t0 = time.perf_counter()
        q = collections.deque()
        for i in range(steps):
            if len(q) == inflight:
                done(*q.popleft().result())
            q.append(pipe.submit(Xs[i % K]))
        while q:
            done(*q.popleft().result())
        torch.cuda.synchronize()
        return time.perf_counter() - t0, dev_ms


def stage_roofline(run, name: str, X, Lk: int, n: int, d: int, maxdim: int, kw: dict, calls: int) -> dict:
    """Per-kernel durations of one batch (`Lk` layers): HIP events around every kernel with all
    stages on ONE stream (each interval brackets exactly one kernel), median over `calls` calls;
    the dominant kernel (largest median) against its roofline.  `run` is ripser_batch (or a
    multi-rank rehearsal's stand-in with the same interface)."""
    acc: dict = {}
    run(X, maxdim=maxdim, stage_times=True, stage_serial=True, **kw)  # untimed: first use of this schedule
    for _ in range(max(1, calls)):
        _, info = run(X, maxdim=maxdim, return_time=True, stage_times=True, stage_serial=True, **kw)
        for k, ms in info["stages"]:
            acc.setdefault(k, []).append(ms)
    stages = {k: float(np.median(v)) for k, v in acc.items()}  # median: one slow outlier (a profiler hiccup) no longer sets it
    kern = {k: v for k, v in stages.items() if k.startswith("k_")}
    dom = max(kern, key=kern.get)
    # an event pair around a kernel also measures the events themselves: the stage pass's empty
    # interval (two events, nothing between) is subtracted, so the short dense-path kernels match
    # rocprof's kernel-only durations of the same launches (r05: k_h2_phase1 79.6 us by events,
    # 74.7 us by rocprof; the event gap ~5 us)
    gap = stages.get("event_gap", 0.0)
    k_raw, k_mean_raw = kern[dom], float(np.mean(acc[dom]))
    kern[dom] = max(k_raw - gap, 0.5 * k_raw)
    dom_mean = max(k_mean_raw - gap, 0.5 * k_mean_raw)  # rocprof's --stats average is a mean over the same launches
    bpl = algo_bytes_per_layer(n, d, maxdim)
    achieved = bpl * Lk / (kern[dom] * 1e-3) / 1e9
    bound, peak, unit, per_layer = "hbm", HBM_PEAK_GBS, "GB/s", {"algo_bytes_per_layer": bpl}
    if dom in ("k_distance_mfma", "k_gram_layer"):  # 2 N^2 D FP64 FLOPs per layer (Gram) against the FP64 MFMA peak
        fpl = 2 * n * n * d
        achieved = fpl * Lk / (kern[dom] * 1e-3) / 1e12
        bound, peak, unit, per_layer = "mfma", FP64_MFMA_PEAK_TFS, "TFLOP/s", {"algo_flops_per_layer": fpl,
                                                                              **mfma_executed(n, d, Lk, kern[dom])}
    traffic = None
    pmc = {}
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_{name}.json")
    pmc_scale = 1.0
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pj = json.load(f)
        pmc = pj.get("kernels", {})
        # counters of a run whose launches covered another batch: per-layer bytes x this batch
        # (every kernel works on its layers independently)
        pmc_scale = Lk / pj["layers_per_launch"] if pj.get("layers_per_launch") else 1.0
        traffic = pmc.get(dom, {}).get("hbm_bytes_per_launch")
        traffic = traffic * pmc_scale if traffic is not None else None
    # what actually bounds the latency-bound small-N kernels: resident waves per CU and the LDS-array
    # busy fraction of the same launch shape (tools/pmc_lds.py, the newest profiles/*_pmc_lds_<wl>.json)
    lds_occ = None
    lds_files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_lds_{name}.json")))
    if lds_files:
        with open(lds_files[-1]) as f:
            lj = json.load(f)
        kk = lj.get("kernels", {}).get(dom)
        if kk:
            lds_occ = {k: kk[k] for k in ("resident_waves_per_cu", "lds_busy_frac", "lds_bank_conflict_share",
                                          "lds_insts_per_wave")}
            lds_occ.update(source=os.path.relpath(lds_files[-1], ROOT), layers_per_launch=lj.get("layers_per_launch"),
                           note="the kernel's bound: one- or two-wave workgroups with ~46 KB of LDS each (occupancy) "
                                "and dependent LDS chains; the HBM fraction above is small by construction")
    gram = next((k for k in ("k_gram_layer", "k_distance_mfma") if k in kern), None)
    mfma_roof = None
    if gram and gram != dom:  # the FP64 Gram kernel when another kernel dominates (e.g. raw4096: H0)
        fpl = 2 * n * n * d
        kern[gram] = max(kern[gram] - gap, 0.5 * kern[gram])  # less the empty event interval, as the dominant kernel
        a_tf = fpl * Lk / (kern[gram] * 1e-3) / 1e12
        mfma_roof = {"bound": "mfma", "kernel": gram, "achieved": a_tf, "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                     "frac": a_tf / FP64_MFMA_PEAK_TFS,
                     "traffic": (pmc[gram]["hbm_bytes_per_launch"] * pmc_scale) if gram in pmc else None,
                     "algo_flops_per_layer": fpl, "layers_per_launch": Lk, "kernel_avg_ms": kern[gram],
                     **mfma_executed(n, d, Lk, kern[gram])}
    return {
        "roofline": {"bound": bound, "kernel": dom, "achieved": achieved, "peak": peak, "unit": unit,
                     "frac": achieved / peak, "traffic": traffic, **per_layer, "lds_occupancy": lds_occ,
                     "layers_per_launch": Lk, "kernel_avg_ms": kern[dom], "kernel_mean_ms": dom_mean,
                     "kernel_avg_ms_events": k_raw, "event_gap_ms": gap,
                     "kernel_timing": "HIP events around each kernel on its stream, all stages serialised on one "
                                      "stream, after the timed region (same batch); median (kernel_avg_ms) and mean "
                                      "(kernel_mean_ms) of the stage pass's calls, less the median empty event "
                                      "interval (event_gap_ms; kernel_avg_ms_events is the raw median).  The same "
                                      "launches alone under rocprofv3: profiles/<round>_kernel_stats_<workload>_stage.csv"},
        "roofline_mfma": mfma_roof,
        "stages_ms": {k: round(v, 5) for k, v in stages.items()},
    }


def measure(pkg, torch, dev, name: str, steps: int, warmup: int, layers: int | None = None) -> dict:
    L, maxdim, desc, _, _ = WORKLOADS[name]
    L = layers or L
    if name.startswith("ripser"):
        return measure_dropin(pkg, torch, name, steps, warmup, L)
    sweeps = workload_sweeps(name, L)
    X_host = sweeps[0]
    n, d = X_host.shape[1], X_host.shape[2]
    host_in = name.endswith("_host")
    # resident in HBM before the timed region -- except the host-in record, which passes numpy arrays
    Xs = sweeps if host_in else [torch.from_numpy(x).to(dev) for x in sweeps]
    torch.cuda.synchronize()
    kw = dict(CALL_KW.get(name, {}))
    if os.environ.get("TDA_BENCH_READY", "1") == "1" and not host_in:
        # Xs were synchronised above (resident in HBM before the timed region): no per-call event on
        # torch's stream, whose hardware queue a pipeline slot may share (TDA_BENCH_READY=0: with it)
        kw["input_ready"] = True
    depth, coalesce = pipe_shape(name, steps)
    kw_pipe = dict(kw)
    if os.environ.get("TDA_BENCH_ONE_STREAM") in ("0", "1"):  # else SweepPipeline's default (one stream when depth > 1)
        kw_pipe["one_stream"] = os.environ["TDA_BENCH_ONE_STREAM"] == "1"
    dev_index = dev.index if dev.index is not None else 0
    seq = None
    piped = depth > 1 or coalesce > 1
    # TDA_BENCH_STAGE_ONLY=1 (profiling): only the stage pass below runs, so a rocprof trace of the
    # command holds exactly the launches the roofline's kernel_avg_ms is taken from (profiles/*_stage.csv)
    stage_only = os.environ.get("TDA_BENCH_STAGE_ONLY") == "1"
    if piped and os.environ.get("TDA_BENCH_NO_SEQ") != "1" and not stage_only:  # the one-call-at-a-time figure next to the pipelined one
        # (TDA_BENCH_NO_SEQ=1: profiling runs, so every launch in the trace is the pipeline's batch)
        el_s, dm_s = _timed_steps(pkg, torch, Xs, maxdim, kw, steps, warmup, 1, host_in, dev_index)
        seq = {"value": L * steps / el_s, "ms_per_step": el_s / steps * 1e3, "device_ms_per_step": sum(dm_s) / len(dm_s)}
    if stage_only:
        el, dev_ms = float("nan"), [float("nan")]
    else:
        el, dev_ms = _timed_steps(pkg, torch, Xs, maxdim, kw_pipe if piped else kw, steps, warmup, depth, host_in, dev_index,
                                  coalesce)
    # per-kernel durations after the timed region, same batch (a coalesced pipeline launches every
    # kernel over `coalesce` sweeps: the stage pass runs that batch too)
    Xst, Lk = ([Xs[i % len(Xs)] for i in range(coalesce)], L * coalesce) if coalesce > 1 else (Xs[0], L)
    sr = stage_roofline(pkg.ripser_batch, name, Xst, Lk, n, d, maxdim, kw, max(1, min(steps, 10)))
    return {
        "value": L * steps / el, "unit": "layers/s", "ms_per_step": el / steps * 1e3, "steps": steps, "warmup": warmup,
        "device_ms_per_step": sum(dev_ms) / len(dev_ms), "X_host": np.concatenate(sweeps), "maxdim": maxdim,
        "config": {"workload": desc, "layers_per_gpu_step": L, "n_points": int(n), "dim": int(d), "maxdim": maxdim,
                   "distinct_sweeps": len(sweeps)},
        **sr,
        "pipeline": {"depth": depth, "coalesce": coalesce, "one_stream": kw_pipe.get("one_stream", depth > 1), "sequential": seq,
                     "note": "value: every step submits one sweep to ripser.SweepPipeline; up to `coalesce` consecutive "
                             "sweeps run as one call over their concatenated layers (each step's future returns its own "
                             "sweep), `depth` calls in flight on separate workspace slots; sequential: one "
                             "ripser_batch call per step, one at a time"} if piped else None,
    }


def measure_dropin(pkg, torch, name: str, steps: int, warmup: int, L: int) -> dict:
    """The drop-in at the reference's own call: a step is the reference's
    layer loop -- ``result = ripser(cloud, maxdim=1); dgms = result['dgms']`` for each of the L
    layers, one call per layer (debug_tda_pipeline.py:109-110; analyze_adversarial_tda.py:100):
    host numpy (N, 3) f32 in, ripser.py's full dict out (dgms, num_edges, the (N, N) dperm2all
    distance matrix, ...).  One call at a time, so the rate is the per-call latency floor."""
    _, maxdim, desc, _, _ = WORKLOADS[name]
    X = make_workload(name, L)
    n, d = X.shape[1], X.shape[2]
    for i in range(max(warmup, 1) * L):
        pkg.ripser(X[i % L], maxdim=maxdim)["dgms"]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        for l in range(L):
            dgms = pkg.ripser(X[l], maxdim=maxdim)["dgms"]  # noqa: F841  (the reference reads result['dgms'])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    sr = stage_roofline(pkg.ripser_batch, name, X[:1], 1, n, d, maxdim, {}, 10)
    return {
        "value": L * steps / el, "unit": "layers/s", "ms_per_step": el / steps * 1e3, "steps": steps, "warmup": warmup,
        "ms_per_call": el / (steps * L) * 1e3, "device_ms_per_step": None, "X_host": X, "maxdim": maxdim,
        "config": {"workload": desc, "layers_per_gpu_step": L, "n_points": int(n), "dim": int(d), "maxdim": maxdim,
                   "calls_per_step": L},
        **sr, "pipeline": None,
        "note": "one ripser() call per layer, one at a time: the rate is set by the per-call latency (host wrapper, "
                "input copy, the captured graph's launch and its device time, result copy incl. dperm2all), not by "
                "throughput -- ripser_batch / SweepPipeline are the throughput entries",
    }


UMAP_DESC = ("UMAP before ripser (debug_tda_pipeline.py:96-104): 32 layers x 36 prompts x 4096 features, "
             "n_neighbors 6, 3 components, min_dist 0.1, cosine, 500 epochs")


def measure_umap(pkg, torch, dev, steps: int = 10, warmup: int = 2) -> dict:
    """SURVEY 8(f) row 3 (outside the headline metric): the reference's UMAP
    step for a 32-layer sweep on the GPU.  No CPU baseline: umap-learn is
    absent here and the oracle restates only its fuzzy graph."""
    X = torch.from_numpy(pkg.synthetic.activations(32, 36, 4096)).to(dev)
    kw = dict(n_neighbors=6, n_components=3, min_dist=0.1, metric="cosine", random_state=42)
    for _ in range(warmup):
        pkg.umap_batch(X, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        pkg.umap_batch(X, **kw)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"value": 32 * steps / el, "unit": "layers/s", "ms_per_step": el / steps * 1e3, "steps": steps, "warmup": warmup,
            "config": {"workload": UMAP_DESC, "layers_per_gpu_step": 32, "n_points": 36, "dim": 4096},
            "data": DATA["raw4096"], "roofline": None,
            "cpu_baseline": None, "note": "umap-learn is not installed here (no CPU reference to time); layout parity unpinned"}


def _free_port() -> int:
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int, argv: list) -> int:
    """``bench.py --gpus N`` started without torchrun: start N ranks (one
    process per GPU) as ``python -m torch.distributed.run --nproc-per-node N
    bench.py ...`` in a CHILD process -- before this process touches the GPU
    -- and return its exit code (BASELINE.json: "at 1/2/4/8 MI355X")."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    return subprocess.call(cmd)


def _standin():
    """TDA_BENCH_STANDIN=module:function -- a CPU rehearsal of the multi-rank
    loop (tests only): the per-shard batch call is that function (same
    result interface as ripser_batch), no GPU is touched, gloo carries the
    collectives.  bench.py itself never imports a stand-in otherwise."""
    spec = os.environ.get("TDA_BENCH_STANDIN")
    if not spec:
        return None
    mod, fn = spec.split(":")
    return getattr(importlib.import_module(mod), fn)


def summary(out: dict) -> dict:
    """One short row per record, emitted LAST on the line (the driver keeps the
    line's tail): rate, CPU speed-ups and the 20x bar, roofline fraction."""
    rows = {}
    recs = [(out["config"]["workload_name"], out)] + list(out.get("workloads", {}).items())
    for name, r in recs:
        sp = r.get("speedup_vs_cpu") or {}
        rf = r.get("roofline") or {}
        bar = sp.get("bar_20x") or {}
        rows[name] = {"value": round(r["value"], 3), "x_1core": round(sp["one_core"], 2) if "one_core" in sp else None,
                      f"x_{(r.get('cpu_baseline') or {}).get('cores', 'P')}proc": round(sp["all_cores"], 2) if "all_cores" in sp else None,
                      "bar_20x": bar.get("met"), "bar_basis": bar.get("basis"),
                      "roofline": (rf.get("kernel"), rf.get("bound"), rf.get("frac")) if rf else None}
        seq = (r.get("pipeline") or {}).get("sequential")
        if seq:
            rows[name]["one_call_at_a_time"] = round(seq["value"], 3)
    return rows


def parent_cpu_baseline(args) -> str | None:
    """``--gpus N`` without torchrun: the launching process measures the
    CPU baseline BEFORE any rank touches a GPU -- 1 core and P = 16 x N worker processes (the
    job's host share, 16 per GPU), the whole host (os.cpu_count()) at N >= 8 -- and hands it to
    rank 0 through a file.  Returns the file path (None with --no-cpu)."""
    if args.no_cpu:
        return None
    import multiprocessing as mp
    import tempfile

    nproc = os.cpu_count() or 1
    P = int(os.environ.get("TDA_CPU_WORKERS", 0)) or (nproc if args.gpus >= 8 else min(nproc, 16 * args.gpus))
    L, maxdim = args.layers or WORKLOADS[args.workload][0], WORKLOADS[args.workload][1]
    X = workload_layers(args.workload, L)
    with mp.get_context("spawn").Pool(P) as pool:
        pool.map(_cpu_layers, [(args.workload, 0, 0, 0)] * P)  # warm: imports, oracle load
        cb = cpu_baseline(pool, P, args.workload, X, maxdim, args.cpu_seconds)
    cb.update(cpu_info())
    cb["measured_by"] = f"the launching process, before the {args.gpus} ranks started (P = {P} worker processes measured)"
    fd, path = tempfile.mkstemp(prefix="tda_bench_cpu_", suffix=".json")
    with os.fdopen(fd, "w") as f:
        json.dump(cb, f)
    return path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default: the workload's own (WORKLOADS)")
    ap.add_argument("--warmup", type=int, default=None, help="default: the workload's own (WORKLOADS)")
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--workload", default="sweep48_host", choices=list(WORKLOADS))
    ap.add_argument("--extra", default="sweep48,sweep48_L1,sweep48_L4,grid144,torus1024,torus1024x32,torus2048,torus2048_h2,"
                                       "raw4096,umap36,sweep48x4,ripser36,ripser324",
                    help="secondary workloads measured at N=1 (comma list, '' for none)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: every rank runs its own L-layer batch; strong: the L layers are sharded over ranks")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = WORKLOADS[args.workload][3]
    if args.warmup is None:
        args.warmup = WORKLOADS[args.workload][4]

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        cpu_file = parent_cpu_baseline(args)  # before any process touches the GPU
        try:
            env_argv = sys.argv[1:]
            if cpu_file:
                os.environ["TDA_BENCH_CPU_FILE"] = cpu_file
            sys.exit(launch_ranks(args.gpus, env_argv))  # the ranks print the JSON line (rank 0)
        finally:
            if cpu_file and os.path.exists(cpu_file):
                os.unlink(cpu_file)

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    standin = _standin()
    backend = os.environ.get("TDA_DIST_BACKEND", "gloo" if standin else "nccl")  # nccl = RCCL over xGMI
    if standin and (world < 2 or backend != "gloo"):
        raise SystemExit("TDA_BENCH_STANDIN is a multi-rank CPU rehearsal: it needs WORLD_SIZE > 1 and gloo")
    do_cpu = rank == 0 and world == 1 and not args.no_cpu
    pool, P = None, 0
    if do_cpu:  # worker processes start before this process touches the GPU
        import multiprocessing as mp

        P = cpu_workers()
        pool = mp.get_context("spawn").Pool(P)
        pool.map(_cpu_layers, [(args.workload, 0, 0, 0)] * P)  # warm: imports, oracle load

    import torch

    n_dev = 0 if standin else torch.cuda.device_count()
    if standin:
        dev = torch.device("cpu")
    else:
        # one GPU per rank; more ranks than GPUs only in a gloo rehearsal (TDA_DIST_BACKEND=gloo on a 1-GPU box)
        if local >= n_dev and backend != "gloo":
            raise RuntimeError(f"rank {rank} (local {local}) has no GPU of its own: {n_dev} visible; "
                               "wrapping ranks onto shared GPUs is a rehearsal only (TDA_DIST_BACKEND=gloo)")
        local = local % max(1, n_dev)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    # distinct devices the job runs on (local ranks 0..world-1 on one node, wrapped only in a rehearsal)
    n_gpus = min(world, n_dev)
    dist = None
    coll_dev = dev if backend == "nccl" else None         # gloo: collectives on host tensors
    if world > 1:
        import torch.distributed as dist

        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    pkg = importlib.import_module("tda-multimodal_amd")
    if not standin and pkg.lib().tda_device_ok(local) != 1:
        raise RuntimeError("no gfx950 device")

    L, maxdim, desc, _, _ = WORKLOADS[args.workload]
    L = args.layers or L
    prim, strong, multi_roof = None, None, None
    if world == 1:
        prim = measure(pkg, torch, dev, args.workload, args.steps, args.warmup, args.layers)
        value, el_ms = prim["value"], prim["ms_per_step"]
    else:
        host_in = args.workload.endswith("_host")
        sweeps = workload_sweeps(args.workload, L)
        Xs = sweeps if (standin or host_in) else [torch.from_numpy(x).to(dev) for x in sweeps]
        # the same dynamic batching as the one-GPU record (bench PIPE): each rank's steps through a SweepPipeline
        slots, coalesce = pipe_shape(args.workload, args.steps)
        sync = (lambda: None) if standin else torch.cuda.synchronize
        gpu_ix = None if standin else local
        K = len(Xs)

        def run_multi(shard: bool):
            sync()
            for i in range(args.warmup):
                pkg.distributed.sharded_sweep_step(Xs[i % K], maxdim, rank, world, device=coll_dev, shard=shard, run=standin,
                                                   gpu=gpu_ix)
            if slots > 1 or coalesce > 1:  # every slot captures its graphs before the timed region
                warm = pkg.distributed.PipelinedSweep(Xs[0], maxdim, rank, world, device=coll_dev, shard=shard, slots=slots,
                                                      coalesce=coalesce, run=standin, gpu=gpu_ix)
                for i in range(max(max(args.warmup, 1) * slots * coalesce, K * slots)):
                    warm.step(Xs[i % K])
                warm.close()
            dist.barrier()
            sync()
            t0 = time.perf_counter()
            # every step's records are exchanged; the exchange of step i overlaps the GPU work of later steps
            pipe = pkg.distributed.PipelinedSweep(Xs[0], maxdim, rank, world, device=coll_dev, shard=shard, slots=slots,
                                                  coalesce=coalesce, run=standin, gpu=gpu_ix)
            for i in range(args.steps):
                pipe.step(Xs[i % K])
            pipe.close()
            sync()
            dist.barrier()
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)  # max over ranks
            return float(t.item())

        el = run_multi(args.scaling == "strong")
        value = (L if args.scaling == "strong" else L * world) * args.steps / el
        el_ms = el / args.steps * 1e3
        el_s = run_multi(True) if args.scaling == "weak" else el
        strong = {"value": L * args.steps / el_s, "unit": "layers/s", "ms_per_step": el_s / args.steps * 1e3,
                  "scaling": "strong", "layers_total": L, "layers_per_gpu": -(-L // world)}
        if rank == 0:
            # the line's roofline: rank 0's own GPU, the weak step's per-rank batch (the same stage pass as the
            # one-GPU record), after every rank's timed region
            Lk = L * coalesce if coalesce > 1 else L
            Xst = [Xs[i % K] for i in range(coalesce)] if coalesce > 1 else Xs[0]
            run = standin or pkg.ripser_batch
            kw = dict(CALL_KW.get(args.workload, {}))
            if not standin:
                kw["device"] = local
            multi_roof = stage_roofline(run, args.workload, Xst, Lk, int(sweeps[0].shape[1]), int(sweeps[0].shape[2]), maxdim,
                                        kw, max(1, min(args.steps, 10)))
        dist.barrier()

    out = None
    if rank == 0:
        out = {
            "metric": METRIC, "value": value, "unit": "layers/s", "n_gpus": n_gpus, "ranks": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el_ms, "higher_is_better": True, "scaling": args.scaling,
            "vs_baseline": None, "dtype": "f32", "data": DATA[args.workload],
            "config": {"workload": desc, "workload_name": args.workload,
                       "layers_per_gpu_step": L if args.scaling == "weak" else -(-L // world),
                       "n_points": NPOINTS[args.workload], "dim": DIMS[args.workload], "maxdim": maxdim,
                       "distinct_sweeps": ROTATE.get(args.workload, 1),
                       "parallelism": f"layers sharded ({args.scaling}), {world} process(es) on {n_gpus} GPU(s), "
                                      f"{'RCCL' if backend == 'nccl' else backend} gather of per-layer records "
                                      f"(overlapped with the next step's GPU work)"},
            "roofline": prim["roofline"] if prim else (multi_roof or {}).get("roofline"),
            "cpu_baseline": None,
        }
        if standin:
            out["rehearsal"] = {"kind": "cpu stand-in (no GPU)", "standin": os.environ["TDA_BENCH_STANDIN"],
                                "note": "multi-rank launch + gloo collectives rehearsed on the CPU; not a GPU measurement "
                                        "(the roofline's stages are the stand-in's)"}
        elif world > n_gpus:
            out["rehearsal"] = {"kind": f"{world} ranks on {n_gpus} GPU(s) over gloo", "note": "not a multi-GPU measurement"}
        if prim:
            if prim.get("roofline_mfma"):
                out["roofline_mfma"] = prim["roofline_mfma"]
            out["device_ms_per_step"] = prim["device_ms_per_step"]
            out["stages_ms"] = prim["stages_ms"]
            out["pipeline"] = prim["pipeline"]
        elif multi_roof:
            out["stages_ms"] = multi_roof["stages_ms"]
            if multi_roof.get("roofline_mfma"):
                out["roofline_mfma"] = multi_roof["roofline_mfma"]
        if strong:
            out["strong"] = strong
        if world > 1 and (slots > 1 or coalesce > 1):
            out["pipeline"] = {"depth": slots, "coalesce": coalesce, "note": "each rank's steps through ripser.SweepPipeline "
                               "(as the one-GPU record); the records of every `coalesce` steps exchanged in one "
                               "all-reduce + gather, in step order"}
        cpu_file = os.environ.get("TDA_BENCH_CPU_FILE")
        if world > 1 and cpu_file and os.path.exists(cpu_file):  # measured by the launching process
            with open(cpu_file) as f:
                cb = json.load(f)
            out["cpu_baseline"] = cb
            out["speedup_vs_cpu"] = speedups(value, cb, args.workload)
            if strong:
                strong["speedup_vs_cpu"] = speedups(strong["value"], cb, args.workload)
    if rank == 0 and world == 1:
        cpu_done = {}
        if do_cpu:
            cb = cpu_baseline(pool, P, args.workload, prim["X_host"], prim["maxdim"], args.cpu_seconds)
            cb.update(cpu_info())
            out["cpu_baseline"] = cb
            cpu_done[args.workload] = cb
            out["speedup_vs_cpu"] = speedups(value, cb, args.workload)
        out["workloads"] = {}
        for w in [w for w in args.extra.split(",") if w and w != args.workload]:
            if w == "umap36":
                out["workloads"][w] = measure_umap(pkg, torch, dev)
                continue
            if w == "ripser324" and not os.path.exists(os.path.join(ROOT, "tests", "golden", "adv_clouds.npz")):
                continue
            _, _, _, st, wu = WORKLOADS[w]
            m = measure(pkg, torch, dev, w, st, wu)
            rec = {k: m[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup", "device_ms_per_step",
                                     "config", "roofline", "roofline_mfma", "stages_ms", "pipeline", "ms_per_call", "note")
                   if k in m}
            if rec.get("roofline_mfma") is None:
                rec.pop("roofline_mfma", None)
            rec["data"] = DATA[w]
            if do_cpu:
                same = CPU_SAME.get(w)
                if same in cpu_done:  # the same layers' oracle rate (per-layer work is identical)
                    rec["cpu_baseline"] = dict(cpu_done[same], sample=cpu_done[same]["sample"] + f"; shared with {w}")
                else:
                    rec["cpu_baseline"] = cpu_baseline(pool, P, w, m["X_host"], m["maxdim"], args.cpu_seconds)
                    cpu_done[w] = rec["cpu_baseline"]
                cbw = rec["cpu_baseline"]
                rec["speedup_vs_cpu"] = speedups(m["value"], cbw, w)
            out["workloads"][w] = rec
    if pool is not None:
        pool.close()
        pool.join()
    if rank == 0:
        if world == 1:
            out["summary"] = summary(out)  # last key: the driver keeps the tail of the line
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
