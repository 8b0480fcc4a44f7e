#!/usr/bin/env python3
"""bench.py -- rows/s per training iteration on MI355X (BASELINE.json metric).

A default run times all four BASELINE workloads, one after the other, each
with its own data resident in HBM and freed before the next:
  kmeans       (headline, BASELINE configs[1], the config the metric is
               quoted on) KMeans k=1024 on synthetic dense fp64 10M x 256, one
               Lloyd iteration per step (KMeans.scala:275-334: statistics,
               findClosest for every row, per-cluster sums/weights/cost,
               merge, centroid update)
  gramian      RowMatrix.computeGramianMatrix pass (configs[2]: 100M x 1024)
  pca          RowMatrix.computeCovariance, the PCA variant of configs[2], on
               the same rows (mean pass, isSparseMatrix, centred syrk)
  lr_multi     multinomial LR, 100 classes, 512 dense features (configs[3]:
               50M rows); one RDDLossFunction.calculate per step
  lr_sparse    binomial LR on CSR, 1M features, 64 nnz/row (configs[4]: 200M
               rows, tiles layout); one RDDLossFunction.calculate per step
The headline JSON line is KMeans's; the other three ride along under
"workloads", each with its own value, roofline and cpu_baseline.
--workload NAME times one of them alone.

Rows per GPU (--scaling auto): KMeans config 2 is a one-GPU config, so each
GPU holds 10M rows (weak scaling); configs 3-5 are totals split over the N
GPUs by contiguous row ranges (strong scaling, parallel.shard_bounds), capped
at the largest shard one GPU holds resident (Gramian: 30M rows = 246 GB, so
100M rows need N >= 4 to be whole).  --scaling weak|strong forces one mode
for every workload; --rows overrides the rows per GPU.
With --gpus N (one process per GPU via torch.distributed.run) the merge is
one RCCL all-reduce per iteration over libcyclone's communicator (cyc_comm,
the only RCCL communicator per GPU); torch.distributed runs on gloo for the
rendezvous, the RCCL id and the host barriers.

Prints ONE JSON line on rank 0.  `roofline` is for the workload's dominant
kernel (the priced kernel with the most time per step), timed with HIP
events on the stream it runs on inside the timed region (cyc_profile_*),
lists every priced kernel's fraction under `priced_kernels`, and carries
`step_frac`: the workload's algorithmic work per step (`step_work`) over
`ms_per_step`, against the same kind of peak; `cpu_baseline` is the CPU
restatement (oracle/, a C port of the reference loops) on a bounded sample of
the same data, one partition per available host core.  On one GPU a `blas`
leg follows: the per-call netlib layer (libcyclone_blas.so) at
BLASBenchmark's shapes against its published rates.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6   # MI355X fp64 (vector = matrix) spec, BASELINE.md section 2
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
I8_PEAK_TOPS = 5000.0     # dense i8 MFMA: 2x the ~2.5 PF dense bf16 rate (MI355X_MICROARCH.md)
# (bound, unit, peak, unit scale) of a priced kernel
HBM = ("hbm", "GB/s", HBM_PEAK_GBS, 1e9)
FP64 = ("mfma", "TFLOP/s", FP64_PEAK_TFLOPS, 1e12)
I8 = ("mfma", "TOPS", I8_PEAK_TOPS, 1e12)

DIST_BACKEND = "gloo"     # torch.distributed's group: host only, no second RCCL communicator
ORDER = ("kmeans", "gramian", "pca", "lr_multi", "lr_sparse")
# BASELINE configs: rows of the whole problem, and whether it is per GPU
# (pca: the PCA variant of configs[2], on the same rows as gramian)
CONFIG_ROWS = {"kmeans": 10_000_000, "gramian": 100_000_000, "pca": 100_000_000,
               "lr_multi": 50_000_000, "lr_sparse": 200_000_000}
PER_GPU_CONFIG = {"kmeans": True, "gramian": False, "pca": False, "lr_multi": False,
                  "lr_sparse": False}
# the largest shard one MI355X holds resident (288 GB HBM)
MAX_RESIDENT_ROWS = {"kmeans": 10_000_000, "gramian": 30_000_000, "pca": 30_000_000,
                     "lr_multi": 50_000_000, "lr_sparse": 200_000_000}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="all", choices=("all",) + ORDER + ("blas",))
    ap.add_argument("--scaling", default="auto", choices=("auto", "weak", "strong"))
    ap.add_argument("--rows", type=int, default=0, help="rows per GPU (0 = from --scaling)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target CPU time of each cpu_baseline sample (0 disables)")
    return ap.parse_args(argv)


def rows_per_gpu(workload, scaling, world, rank, override=0):
    """(rows this rank holds, scaling mode, rows of the whole job) for a
    workload: weak = the config's per-GPU rows on every GPU; strong = the
    config's total split by parallel.shard_bounds, each shard capped at
    MAX_RESIDENT_ROWS."""
    from cycloneml_amd.parallel import shard_bounds
    mode = scaling
    if mode == "auto":
        mode = "weak" if PER_GPU_CONFIG[workload] else "strong"
    if override:
        return override, mode, override * world
    if mode == "weak":
        n = min(CONFIG_ROWS[workload], MAX_RESIDENT_ROWS[workload])
        return n, mode, n * world
    s, e = shard_bounds(CONFIG_ROWS[workload], rank, world)
    cap = MAX_RESIDENT_ROWS[workload]
    total = sum(min(b - a, cap) for a, b in
                (shard_bounds(CONFIG_ROWS[workload], r, world) for r in range(world)))
    return min(e - s, cap), mode, total


def pmc_traffic(workload, kernel, rows):
    """HBM bytes per timed launch of `kernel`, from the latest committed
    rocprofv3 --pmc summary of this workload
    (profiles/r<NN>_<workload>_pmc.json, tools/pmc_summary.py: separate
    FETCH_SIZE / WRITE_SIZE passes, gfx950 corrections applied there): the
    summary's bytes PER DISPATCH (not per step: a profiled run may dispatch
    a kernel outside its steps too), scaled by this run's rows over the
    profiled run's `_rows` (the same launch shape per step at equal rows);
    (None, None) when there is none."""
    import glob
    import re

    def tag(f):   # r06ak after r06z after r06y: round, then suffix length, then suffix
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{workload}_pmc.json")), key=tag)
    for f in reversed(files):
        try:
            d = json.load(open(f))
            if kernel not in d:
                continue
            return d[kernel]["hbm_bytes_per_dispatch"] * rows / d["_rows"], os.path.basename(f)
        except Exception:
            continue
    return None, None


def _cgroup_cpus():
    """CPUs the cgroup quota allows (cpu.max / cfs quota), None if unlimited."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(int(q) / int(p)))
    except Exception:
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, q // p)
    except Exception:
        pass
    return None


def host_cores():
    """The host cores this process can use -- Spark's local[N] with N = all
    of them (LocalSchedulerBackend.scala:87-93): the CPUs in
    its affinity mask, capped by a cgroup CPU quota when one is set.  Every
    cpu_baseline runs one partition per such core and records the counts."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = _cgroup_cpus()
    n = min(aff, quota) if quota else aff
    return max(1, n), {"os_cpu_count": os.cpu_count(), "affinity_cpus": aff,
                       "cgroup_quota_cpus": quota}


def cpu_threads():
    return host_cores()[0]


def _cores_info():
    return host_cores()[1]


def timed_parallel(fn, parts, threads):
    from concurrent.futures import ThreadPoolExecutor
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        out = list(ex.map(fn, parts))
    return time.perf_counter() - t0, out


# ------------------------------------------------------------ synthetic data
# Shared with the parity tests that check the timed data itself
# (tests/test_kmeans_gpu.py::test_full_config_all_rows,
# tests/test_logistic_gpu.py::test_sparse_config5_full_size).

def kmeans_data(n, dev, rank=0, d=256, k=1024):
    """BASELINE config 2 / SURVEY 8d: k true centers ~ N(0, 4^2) per dim plus
    point noise N(0, 1), fp64 row-major n x d; torch Philox on the device,
    the centers seeded 1234, the rows 1000 + rank in 1M-row chunks."""
    import torch
    g = torch.Generator(device=dev).manual_seed(1234)
    true_c = torch.randn(k, d, generator=g, device=dev, dtype=torch.float64) * 4.0
    gr = torch.Generator(device=dev).manual_seed(1000 + rank)
    X = torch.empty(n, d, dtype=torch.float64, device=dev)
    for s in range(0, n, 1 << 20):
        e = min(n, s + (1 << 20))
        lab = torch.randint(0, k, (e - s,), generator=gr, device=dev)
        X[s:e] = true_c[lab] + torch.randn(e - s, d, generator=gr, device=dev,
                                           dtype=torch.float64)
    return X


def gramian_data(n, dev, rank=0, p=1024):
    """BASELINE config 3 / SURVEY 8d rows: U[0, 1) fp64 n x p, torch Philox
    seeded 77 + rank, 1M-row chunks (tests/test_gramian_gpu.py checks the
    Gramian and the covariance on these rows)."""
    import torch
    g = torch.Generator(device=dev).manual_seed(77 + rank)
    X = torch.empty(n, p, dtype=torch.float64, device=dev)
    for s in range(0, n, 1 << 20):
        e = min(n, s + (1 << 20))
        X[s:e] = torch.rand(e - s, p, generator=g, device=dev, dtype=torch.float64)
    return X


def lr_multi_data(n, dev, rank=0, F=512, C=100):
    """BASELINE config 4 / SURVEY 8d rows: X ~ N(0, 1) fp64 n x F (seeded
    500 + rank, 512K-row chunks), labels drawn from softmax(X W) for
    W ~ N(0, 1/F) seeded 11; and scaledMean = mean / std per feature over
    every rank's rows (the Summarizer pre-pass of LogisticRegression.scala:
    511-516, :957-960: the unbiased variance of Summarizer.scala:673-690),
    a device tensor.  Returns (X, labels, scaledMean)."""
    import torch
    from cycloneml_amd import parallel
    g = torch.Generator(device=dev).manual_seed(11)
    Wt = torch.randn(F, C, generator=g, device=dev, dtype=torch.float64) / F ** 0.5
    gr = torch.Generator(device=dev).manual_seed(500 + rank)
    X = torch.empty(n, F, dtype=torch.float64, device=dev)
    y = torch.empty(n, dtype=torch.float64, device=dev)
    for s in range(0, n, 1 << 19):
        e = min(n, s + (1 << 19))
        X[s:e] = torch.randn(e - s, F, generator=gr, device=dev, dtype=torch.float64)
        pr = torch.softmax(X[s:e] @ Wt, dim=1)
        y[s:e] = torch.multinomial(pr, 1, generator=gr).squeeze(1).to(torch.float64)
    mean = torch.zeros(F, dtype=torch.float64, device=dev)
    sq = torch.zeros(F, dtype=torch.float64, device=dev)
    for s in range(0, n, 1 << 22):
        mean += X[s:s + (1 << 22)].sum(0)
        sq += (X[s:s + (1 << 22)] ** 2).sum(0)
    tot = torch.cat([mean, sq, torch.tensor([float(n)], dtype=torch.float64, device=dev)])
    parallel.allreduce_(tot)                   # the summary over every rank's rows
    s1, s2, n_all = tot[:F], tot[F:2 * F], tot[2 * F]
    mean = s1 / n_all
    std = ((s2 - n_all * mean ** 2) / (n_all - 1)).clamp_min(0).sqrt()
    return X, y, mean / std


LR_SPARSE_CHUNK = 64 * 8192            # whole row blocks of the tiles layout per append


def lr_sparse_chunks(n, dev, rank=0, F=1_000_000, k=64):
    """BASELINE config 5 / SURVEY 8d rows, LR_SPARSE_CHUNK rows at a time:
    yields (start, end, rowptr, colidx, values, labels) with k distinct sorted
    columns per row (one per F/k band + a uniform offset), values U(0, 1),
    labels ~ Bernoulli(sigmoid(w . x)) for w ~ N(0, 0.5^2) seeded 2; the rows
    seeded 900 + rank."""
    import torch
    g = torch.Generator(device=dev).manual_seed(2)
    w_true = torch.randn(F, generator=g, device=dev, dtype=torch.float64) * 0.5
    gr = torch.Generator(device=dev).manual_seed(900 + rank)
    band = F // k
    for s in range(0, n, LR_SPARSE_CHUNK):
        e = min(n, s + LR_SPARSE_CHUNK)
        c = (torch.arange(k, device=dev) * band).unsqueeze(0) + \
            torch.randint(0, band, (e - s, k), generator=gr, device=dev)
        v = torch.rand(e - s, k, generator=gr, device=dev, dtype=torch.float64)
        m = (v * w_true[c]).sum(1)
        y = (torch.rand(e - s, generator=gr, device=dev, dtype=torch.float64)
             < torch.sigmoid(m)).to(torch.float64)
        del m
        rowptr = torch.arange(0, (e - s) * k + 1, k, dtype=torch.int64, device=dev)
        yield s, e, rowptr, c.to(torch.int32).reshape(-1), v.reshape(-1), y


# ---------------------------------------------------------------- workloads

class KMeansWorkload:
    """One Lloyd iteration per step over a row image built once per fit.
    findClosest runs as the tiered exact screen of kmeans_i8.hip: the
    one-limb exact-integer i8 pass over every (row, center) pair
    (k_screen32<.., 1, false>, timed as k_kmeans_screen1), the two-limb
    refinement over each 32 rows' candidate union (k_kmeans_refine2), the
    full two-limb pass only for the rows those hand on (k_kmeans_screen2),
    then the fp64 tiers.  Kernels are priced in their own units: the
    one-limb pass against the i8 MFMA peak (2 ops per row, padded center
    and dimension), the cluster sums (k_chunk_sums) against HBM; the
    roofline line names the slowest priced kernel."""
    kernel = "k_chunk_sums"
    kernels = ("k_kmeans_screen1", "k_kmeans_refine2", "k_kmeans_screen2", "k_kmeans_cands3",
               "k_kmeans_cands", "k_kmeans_screen3", "k_kmeans_compact", "k_kmeans_assign_fp64",
               "k_kmeans_bounds", "k_kmeans_recheck", "k_kmeans_inc", "k_kmeans_exact",
               "k_chunk_sums")
    pmc_names = {"k_kmeans_screen1": "k_screen32_l1", "k_kmeans_screen2": "k_screen32_l2",
                 "k_kmeans_refine2": "k_screen32r", "k_chunk_sums": "k_chunk_sums_fast",
                 # the re-check's bytes scale with the rows the bounds list
                 # (data-dependent per launch): a profiled run's per-dispatch
                 # average is not this run's launch, so no PMC traffic
                 "k_kmeans_recheck": None}

    def __init__(self, n, dev, rank):
        import torch
        from cycloneml_amd import parallel
        from cycloneml_amd.clustering import KMeansPlan, row_norms
        self.n, self.d, self.k = n, 256, 1024
        d, k = self.d, self.k
        X = kmeans_data(n, dev, rank)
        self.X = X
        self.C0 = X[:k].clone()           # setInitialModel semantics: rows 0..k-1
        parallel.broadcast_(self.C0)
        self.C = self.C0.clone()
        self.cnorm = row_norms(self.C)
        self.plan = KMeansPlan(d, k, n)
        # per-fit preparation, once before the Lloyd loop and outside the
        # timed iterations: the cached norms (KMeans.scala:263-270) and the
        # row image (int8 limbs, 3 B/element).  Reported as prep_ms.
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        self.xnorm = row_norms(X)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        self.rows = self.plan.rows(X)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        self.prep = {"norms_ms": (t1 - t0) * 1e3, "row_image_ms": (t2 - t1) * 1e3,
                     "per_fit_ms": (t2 - t0) * 1e3,
                     "per_iteration_ms_at_maxIter_20": (t2 - t0) * 1e3 / 20,
                     "note": "once per fit, before the Lloyd loop; not in ms_per_step"}
        self.buf = torch.zeros(k * d + k + 1, dtype=torch.float64, device=dev)
        self.conv = torch.zeros(1, dtype=torch.int32, device=dev)
        self.parallel = parallel
        self._refine = (-1, -1, -1)

    def before_timing(self, steps):
        """Centers of the first timed step (the cpu_baseline's) and the
        carried bounds' / incremental sums' counters at the start of the
        clock."""
        self.C_timed = self.C.clone()
        self.steps_timed = steps
        self._b0 = self.rows.bounds_info()
        self._rc0 = self.rows.bounds_rechecked()
        self._i0 = self.rows.incremental_info()

    def after_steps(self):
        calls, screened = self.rows.bounds_info()
        self.screened_timed = screened - self._b0[1]
        self.bounded_calls = calls - self._b0[0]
        self.rechecked_timed = self.rows.bounds_rechecked() - self._rc0
        inc, moved = self.rows.incremental_info()
        self.inc_timed = inc - self._i0[0]
        self.moved_timed = moved - self._i0[1]

    def step(self):
        k, d = self.k, self.d
        buf = self.buf
        sums, wsum, cost = buf[:k * d], buf[k * d:k * d + k], buf[k * d + k:]
        buf.zero_()
        self.plan.accumulate(self.X, self.xnorm, None, self.C, self.cnorm, sums, wsum, cost,
                             rows=self.rows)
        self.parallel.allreduce_(buf)
        self.plan.update(self.C, self.cnorm, sums, wsum, 1e-4, self.conv)

    # bytes per re-checked row: its image (3 limb planes of D), its carried
    # set (6 int32), outside bound, (ub, lb), state byte and list entry
    RECHECK_BYTES = 3 * 256 + 24 + 4 + 8 + 1 + 4

    def _per_step(self, attr, default):
        v = getattr(self, attr, None)
        return default if v is None else v / self.steps_timed

    def work(self, kname, launches_per_step):
        D = 128 * ((self.d + 127) // 128)                 # 32-dim substeps, padded
        kpad = 32 * (2 * ((self.k + 63) // 64))           # 32-center tiles (even count)
        if kname == "k_kmeans_screen1":       # one limb product: 2 ops per (row, center, dim)
            # over the rows it screened (those the carried bounds did not keep)
            rows = self._per_step("screened_timed", self.n)
            return 2.0 * D * kpad * rows / launches_per_step, I8
        if kname == "k_kmeans_recheck":       # the carried sets' rows: image + state
            rows = self._per_step("rechecked_timed", self.n / 8)
            return self.RECHECK_BYTES * rows / launches_per_step, HBM
        if kname == "k_kmeans_inc":           # assignment + previous (8 B/row), moved rows twice,
            moved = self._per_step("moved_timed", 0.0)   # the clusters' state (S, P, C, S out)
            b = self.n * 8.0 + moved * 2 * 8 * self.d + 4.0 * self.k * self.d * 8
            return b / launches_per_step, HBM
        if kname == "k_chunk_sums":           # every row once (fp64) + its perm entry
            # launched every step; empty (gated off on the device) when the
            # incremental sums took the step, so priced over the full passes
            full = self.steps_timed - getattr(self, "inc_timed", 0) if hasattr(
                self, "steps_timed") else 1
            if full <= 0:
                return None
            per_step = self.n * (8 * self.d + 4) * full / getattr(self, "steps_timed", 1)
            return per_step / launches_per_step, HBM
        if kname == "k_kmeans_screen2" and self._refine[0] < 0:   # no refinement: every row
            return 6.0 * D * kpad * self.n / launches_per_step, I8
        return None

    def step_work(self):
        """The bytes a Lloyd iteration of this algorithm moves at least: every
        row's carried state (ub/lb 8 B, assignment 4 B, outside bound 4 B,
        norm 8 B read; bounds, state and outside bound 13 B written), the
        re-checked rows' image and sets, the screened rows' one-limb image
        (256 B), and the cluster sums' input -- every row's fp64 values on a
        full pass, the moved rows' (twice) on an incremental one."""
        steps = getattr(self, "steps_timed", None)
        if steps is None:
            return self.n * 8.0 * self.d, HBM
        inc = getattr(self, "inc_timed", 0) / steps
        sums = (1.0 - inc) * self.n * (8.0 * self.d + 4) + \
            self._per_step("moved_timed", 0.0) * 2 * 8 * self.d + inc * self.n * 8.0
        b = self.n * 37.0 + self._per_step("rechecked_timed", 0.0) * self.RECHECK_BYTES + \
            self._per_step("screened_timed", 0.0) * 256 + sums
        return b, HBM

    def after_timing(self):
        import torch
        self._refine = self.plan.last_refine()
        # the same steps with the full cluster-sums pass every step (the
        # incremental sums off), for comparison; then back on (the fit)
        self.rows.set_incremental(False)
        for _ in range(2):
            self.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            self.step()
        torch.cuda.synchronize()
        self.full_sums_ms = (time.perf_counter() - t0) / 5 * 1e3
        self.rows.set_incremental(True)

    def fit_once(self, max_iter=20):
        """One fit as the ml estimator runs it -- maxIter 20, tol 1e-4
        (ml/clustering/KMeans.scala:89, :336-343) -- from setInitialModel
        (rows 0..k-1): the cached norms, the plan and row image, then every
        Lloyd iteration (mllib/clustering/KMeans.scala:263-334) with its
        convergence check read back on the host."""
        from cycloneml_amd.clustering import KMeans, KMeansModel
        km = KMeans(k=self.k, maxIterations=max_iter, epsilon=1e-4)
        km.setInitialModel(KMeansModel(self.C0.cpu().numpy()))
        marks = [time.perf_counter()]
        # each iteration ends with the host's convergence check (a sync)
        model = km.run(self.X, iteration_callback=lambda it, c: marks.append(time.perf_counter()))
        return {"iterations": model.numIter,
                "carried_state": {k: v for k, v in km.lastFitInfo.items() if k != "per_iteration"},
                "iteration_ms": [round((b - a) * 1e3, 3) for a, b in zip(marks[:-1], marks[1:])],
                "iteration_ms_note": "wall time between the host's convergence checks; the first "
                                     "includes the norms, the plan and the row image",
                "note": "one fit from setInitialModel (rows 0..k-1), maxIter 20, tol 1e-4: "
                        "norms + plan + row image + every iteration with its host convergence "
                        "check, over iterations 1..maxIter (value times steady-state "
                        "iterations after the warmup)"}

    def extra_roofline(self, launches_per_step, avg_s):
        import torch
        listed, full, union = self._refine
        waves = (listed - 0) / 32 if listed and listed > 0 else None
        # screen tiers of one counted assign of every row, after the timed region
        a = torch.empty(self.n, dtype=torch.int32, device=self.X.device)
        c = torch.empty(self.n, dtype=torch.float64, device=self.X.device)
        self.plan.stats(self.C)
        exact = self.plan.assign(self.X, self.xnorm, self.C, self.cnorm, a, c,
                                 count_exact=True, rows=self.rows)
        tier2, _ = self.plan.last_tiers()
        scr = getattr(self, "screened_timed", None)
        rc = getattr(self, "rechecked_timed", None)
        inc = getattr(self, "inc_timed", None)
        return {"incremental_sums": {
            "incremental_steps": inc, "full_pass_steps": (self.steps_timed - inc) if inc is not None
            else None,
            "moved_rows_per_step": self._per_step("moved_timed", None),
            "full_sums_ms_per_step": getattr(self, "full_sums_ms", None),
            "note": "cluster sums carried across the fit (cyclone.h "
                    "cyc_kmeans_rows_set_incremental): a step folds only the rows whose "
                    "center changed into the carried sums and takes the cost from "
                    "Q + 2 (P - c).(S - W P) + W |P - c|^2 with its rounding bounded on the "
                    "device (<= 2^-40 of the cost, else the full pass); full_sums_ms_per_step: "
                    "the same steps with the full pass every step, timed after the clock"},
            "carried_bounds": {
            "rows_screened_per_step": scr / self.steps_timed if scr is not None else None,
            "rows_rechecked_per_step": rc / self.steps_timed if rc is not None else None,
            "rows_kept_per_step": self.n - scr / self.steps_timed if scr is not None else None,
            "bounded_calls": getattr(self, "bounded_calls", None),
            "note": "Hamerly bounds carried across the fit's iterations (cyclone.h "
                    "cyc_kmeans_rows_set_bounds): a row whose moved bounds still certify its "
                    "center keeps it and skips the screen; a row whose bounds fail but whose "
                    "carried candidate set still excludes every other center is re-checked "
                    "against that set (three-limb bounds); the rest get the full screen "
                    "(screened); every row's cost and sums are computed every step"},
            "screen_tiers": {
            "rows_listed_by_one_limb_pass": listed,
            "rows_to_full_two_limb_pass": full,
            "mean_union_centers_per_32_listed_rows": union / waves if waves else None,
            "rows_to_candidate_pass": self.plan.last_candidates(),
            "rows_to_fp64_candidate_pass": self.plan.last_candidates3(),
            "rows_to_three_limb_pass": self.plan.last_screen(),
            "rows_to_fp64_screen": tier2, "rows_to_exact": exact,
            "note": "the last timed iteration's one-limb pass / refinement (over the rows the "
                    "bounds left), then one counted assign of every row after the timed region "
                    "for the later tiers"}}

    def describe(self):
        return (f"KMeans k={self.k} Lloyd iteration, dense fp64 {self.n} x {self.d} rows per GPU "
                "(BASELINE configs[1])")

    def cpu_baseline(self, seconds):
        import numpy as np
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        threads = cpu_threads()
        m = min(self.n, 2_000_000)
        Xs = np.ascontiguousarray(self.X[:m].cpu().numpy())
        # the centers of the first timed step (after the warm-up iterations)
        C = getattr(self, "C_timed", self.C0).cpu().numpy()
        xn, cn = oracle.row_norms(Xs), oracle.row_norms(C)
        t0 = time.perf_counter()
        oracle.kmeans_iteration(Xs[:2000], xn[:2000], None, C, cn)
        t1 = time.perf_counter() - t0
        t0 = time.perf_counter()
        oracle.kmeans_stats(C)
        per_row = max((t1 - (time.perf_counter() - t0)) / 2000, 1e-9)
        rows = int(min(m, max(threads * 1000, seconds * threads / per_row)))
        rows -= rows % threads
        t0 = time.perf_counter()
        oracle.kmeans_iteration(Xs[:rows], xn[:rows], None, C, cn, num_partitions=threads,
                                threads=threads)
        el = time.perf_counter() - t0
        return {"value": rows / el, "unit": "rows/s", "cores": threads, "kind": "port",
                "sample": f"{rows} rows of the same data, the k={self.k} centers of the first "
                          f"timed step (iteration {getattr(self, 'warmup', 0) + 1} of the fit "
                          f"from rows 0..k-1), one Lloyd iteration (stats+findClosest+sums+"
                          f"merge+update) as {threads} partitions on {threads} threads, "
                          f"{el:.1f} s"}


class GramianWorkload:
    # at p = 1024 the syrk is k_gram_dma (gramian.hip, 8-row LDS-DMA chunks)
    kernel = "k_gram_dma"

    def __init__(self, n, dev, rank):
        import torch
        from cycloneml_amd import parallel
        from cycloneml_amd.linalg import GramianPlan
        self.n, self.p = n, 1024
        self.X = gramian_data(n, dev, rank, self.p)
        self.U = torch.zeros(self.p * (self.p + 1) // 2, dtype=torch.float64, device=dev)
        self.plan = GramianPlan(self.p)
        self.parallel = parallel

    def step(self):
        self.U.zero_()
        self.plan.accumulate(self.X, self.U)
        self.parallel.allreduce_(self.U)

    def work(self, kname, launches_per_step):
        return float(self.n) * self.p * (self.p + 1) / launches_per_step, FP64   # flops (upper)

    def step_work(self):
        return float(self.n) * self.p * (self.p + 1), FP64

    def describe(self):
        return (f"RowMatrix.computeGramianMatrix pass, dense fp64 {self.n} x {self.p} rows per "
                "GPU, U[0,1) (BASELINE configs[2]: 100M rows in total, split over the GPUs; "
                "one GPU holds at most a 30M-row shard, 246 GB)")

    def cpu_baseline(self, seconds):
        import numpy as np
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        threads = cpu_threads()
        Xs = np.ascontiguousarray(self.X[:200].cpu().numpy())
        t0 = time.perf_counter()
        oracle.gramian_partition(Xs)
        per_row = (time.perf_counter() - t0) / 200
        rows = int(min(self.n, 1_500_000, max(threads * 50, seconds * threads / per_row)))
        rows -= rows % threads
        Xs = np.ascontiguousarray(self.X[:rows].cpu().numpy())
        parts = np.array_split(Xs[:rows], threads)
        el, Us = timed_parallel(oracle.gramian_partition, parts, threads)
        return {"value": rows / el, "unit": "rows/s", "cores": threads, "kind": "port",
                "sample": f"{rows} rows x 1024 of the same data, per-row netlib dspr as "
                          f"{threads} partitions on {threads} threads, {el:.1f} s"}


class PCAWorkload:
    """The PCA variant of BASELINE configs[2]: RowMatrix.computeCovariance
    (RowMatrix.scala:452-467) per step on the Gramian workload's rows -- the
    isSparseMatrix (:462, a take(1): one 64K-row round on dense rows), the
    column moments of the leading 64K rows, then the syrk in the form the
    moments allow (these U[0, 1) rows have mean^2 = 3 variance: the plain
    syrk with the column sums (Statistics.colStats, :456) riding it, and the
    Gramian finish of :222-246; linalg.RowMatrix._near_centred states the bound), the
    all-reduce and the finish into the n x n matrix in HBM.  The reference's
    centred syrk (computeDenseVectorCovariance, :163-220) is timed after the
    steps for comparison (centred_form_ms_per_step).  The breeze SVD of
    computePrincipalComponentsAndExplainedVariance (:499-501) runs on the
    driver in the reference; here it is the host eigensolve, timed once
    outside the steps (eigensolve_ms)."""
    kernels = ("k_gram_dma", "k_gram_dma_cov", "k_col_sums")
    # no per-dispatch PMC figure for the column pass: the profiled
    # k_col_partial dispatches mix the 64K-row sample with the centred
    # comparison's whole-shard passes
    pmc_names = {"k_col_sums": None}

    @property
    def kernel(self):   # the timed steps' form (after_timing runs the centred one after them)
        form = getattr(self, "form", None) or getattr(self.mat, "lastCovarianceForm", "centred")
        return "k_gram_dma_cov" if form == "centred" else "k_gram_dma"

    def __init__(self, n, dev, rank):
        from cycloneml_amd.linalg import RowMatrix
        self.n, self.p = n, 1024
        self.X = gramian_data(n, dev, rank, self.p)
        self.mat = RowMatrix(self.X)
        self.G = None

    def step(self):
        self.G = self.mat.computeCovarianceDevice()

    def work(self, kname, launches_per_step):
        if kname == "k_col_sums":             # the rows its passes read once (fp64)
            rows = 0
            for ps in getattr(self, "passes", None) or getattr(self.mat, "lastCovariancePasses",
                                                                ["column sums"]):
                if ps.startswith("moments of the leading"):
                    rows += int(ps.split()[4])
                elif ps in ("column moments", "column sums"):
                    rows += self.n
            return float(rows) * self.p * 8 / launches_per_step, HBM
        return float(self.n) * self.p * (self.p + 1) / launches_per_step, FP64   # flops (upper)

    def step_work(self):
        return float(self.n) * self.p * (self.p + 1), FP64   # the syrk's n p (p + 1) flops

    def after_timing(self):
        import numpy as np
        import torch
        cov = self.G.cpu().numpy()
        self.form = self.mat.lastCovarianceForm
        self.passes = list(self.mat.lastCovariancePasses)
        t0 = time.perf_counter()
        _, s, _ = np.linalg.svd(cov)              # the driver's brzSvd(Cov) (:501)
        self.eig_ms = (time.perf_counter() - t0) * 1e3
        self.explained_top3 = (s[:3] / s.sum()).tolist()
        # the reference's centred form on the same rows, for comparison
        self.mat.covarianceForm = "centred"
        self.mat.computeCovarianceDevice()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            Gc = self.mat.computeCovarianceDevice()
        torch.cuda.synchronize()
        self.centred_ms = (time.perf_counter() - t0) * 1e3 / 3
        diff = (Gc - self.G).abs()
        self.form_diff = float(diff.max() / Gc.abs().max())
        dg = Gc.diagonal().clamp_min(0).sqrt()
        self.form_diff_entry = float((diff / (dg[:, None] * dg[None, :]).clamp_min(1e-300)).max())
        self.mat.covarianceForm = "auto"

    def extra_roofline(self, launches_per_step, avg_s):
        return {"eigensolve_ms": self.eig_ms, "explained_variance_top3": self.explained_top3,
                "covariance_form": self.form, "centred_form_ms_per_step": self.centred_ms,
                "forms_normwise_diff": self.form_diff,
                "forms_normwise_diff_is": "max |C_auto - C_centred| / max |C_centred|",
                "forms_entrywise_diff": self.form_diff_entry,
                "forms_entrywise_diff_is": "max over i, j of |C_auto - C_centred|_ij / "
                                           "sqrt(C_ii C_jj) (centred form's diagonal)",
                "covariance_passes": self.passes,
                "note": "step = computeCovariance on the device (isSparseMatrix take(1), the "
                        "passes of covariance_passes, finish); the reference's centred "
                        "form timed after the steps (3 steps); the host SVD timed once, outside"}

    def describe(self):
        return (f"RowMatrix.computeCovariance (PCA variant), dense fp64 {self.n} x {self.p} rows "
                "per GPU, U[0,1) (BASELINE configs[2]: 100M rows in total, split over the GPUs; "
                "one GPU holds at most a 30M-row shard, 246 GB)")

    def cpu_baseline(self, seconds):
        import numpy as np
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        threads = cpu_threads()
        mean = (self.X[:1 << 20].sum(0) / (1 << 20)).cpu().numpy()
        Xs = np.ascontiguousarray(self.X[:200].cpu().numpy())
        t0 = time.perf_counter()
        oracle.gramian_partition(Xs, mean)
        per_row = (time.perf_counter() - t0) / 200
        rows = int(min(self.n, 1_500_000, max(threads * 50, seconds * threads / per_row)))
        rows -= rows % threads
        Xs = np.ascontiguousarray(self.X[:rows].cpu().numpy())
        parts = np.array_split(Xs[:rows], threads)
        el, _ = timed_parallel(lambda x: oracle.gramian_partition(x, mean), parts, threads)
        return {"value": rows / el, "unit": "rows/s", "cores": threads, "kind": "port",
                "sample": f"{rows} rows x 1024 of the same data, x - mean then per-row netlib "
                          f"dspr (computeDenseVectorCovariance's seqOp) as {threads} partitions "
                          f"on {threads} threads, {el:.1f} s; the mean pass not included"}


class LRMultiWorkload:
    kernel = "k_mlr_margins"
    kernels = ("k_mlr_margins", "k_mlr_grad")

    def __init__(self, n, dev, rank):
        from cycloneml_amd.optim import (DeviceInstanceBlock, MultinomialLogisticBlockAggregator,
                                         RDDLossFunction)
        self.n, self.F, self.C = n, 512, 100
        F, C = self.F, self.C
        # scaledMean = mean / std per feature (the Summarizer pre-pass), untimed
        X, y, sm_dev = lr_multi_data(n, dev, rank, F, C)
        self.block = DeviceInstanceBlock(y, None, X=X)
        import numpy as np
        self.coef = np.random.default_rng(3).normal(size=C * F + C) * 0.01
        self.scaledMean = sm_dev.cpu().numpy()                     # bcScaledMean, once
        inv_std = np.ones(F)                                      # bcInverseStd, once
        self.fn = RDDLossFunction([self.block], lambda c: MultinomialLogisticBlockAggregator(
            inv_std, sm_dev, True, True, c, device=dev))

    def step(self):
        self.fn.calculate(self.coef)

    def fit_once(self, max_iter=20):
        """One LogisticRegression.fit as the reference runs it on these rows
        (LogisticRegression.scala:495-685): the Summarizer pre-pass (:511),
        standardization, then breeze LBFGS (m = 10, tol 1e-6, restated in
        cycloneml_amd/optimize.py) driving RDDLossFunction.calculate --
        coefficients broadcast, one device data pass, the gradient pulled
        back -- at least once per iteration (the line search may evaluate
        more: :999), maxIter 20, regParam 0, fitIntercept, multinomial."""
        from cycloneml_amd.classification import LogisticRegression
        lr = LogisticRegression(maxIter=max_iter, family="multinomial")
        model = lr.fit([self.block])
        ev = lr.lastCost.evaluations
        return {"iterations": model.totalIterations, "evaluations": ev,
                "evaluations_per_iteration": ev / max(model.totalIterations, 1),
                "note": "one LogisticRegression.fit (multinomial, maxIter 20, tol 1e-6, "
                        "regParam 0): Summarizer pass + LBFGS with its line-search "
                        "evaluations; each evaluation = coefficients to HBM, one data pass, "
                        "gradient to the host"}

    def work(self, kname, launches_per_step):
        return 2.0 * self.n * self.F * self.C / launches_per_step, FP64   # each pass: one gemm

    def step_work(self):
        return 2 * 2.0 * self.n * self.F * self.C, FP64   # margins gemm + gradient gemm

    def describe(self):
        return (f"multinomial LR ({self.C} classes) RDDLossFunction.calculate, dense fp64 "
                f"{self.n} x {self.F} rows per GPU, fitIntercept+standardization "
                "(BASELINE configs[3]: 50M rows in total, split over the GPUs)")

    def cpu_baseline(self, seconds):
        import numpy as np
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        threads = cpu_threads()
        X = self.block.X[:256].cpu().numpy()
        y = self.block.labels[:256].cpu().numpy()

        def part(rng_):
            a, b = rng_
            st = dict(grad=np.zeros(self.coef.size), loss=0.0, weight=0.0)
            for s in range(a, b, 256):      # InstanceBlock of 256 rows (1 MiB)
                e = min(b, s + 256)
                oracle.multinomial_logistic_add(dict(labels=y[s:e], weights=None, X=X[s:e]),
                                                self.coef, self.C, True, True, self.scaledMean,
                                                st)
            return st
        t0 = time.perf_counter()
        part((0, 256))
        per_row = (time.perf_counter() - t0) / 256
        rows = int(min(self.n, 2_000_000, max(threads * 256, seconds * threads / per_row)))
        rows -= rows % (threads * 256)
        X = self.block.X[:rows].cpu().numpy()
        y = self.block.labels[:rows].cpu().numpy()
        step = rows // threads
        el, _ = timed_parallel(part, [(i * step, (i + 1) * step) for i in range(threads)],
                               threads)
        return {"value": rows / el, "unit": "rows/s", "cores": threads, "kind": "port",
                "sample": f"{rows} rows of the same data in 256-row blocks (1 MiB), "
                          f"{threads} partitions on {threads} threads, {el:.1f} s"}


class LRSparseWorkload:
    """BASELINE configs[4] at full size on one GPU: 200M CSR rows x 1M
    features, 64 nonzeros per row, fitIntercept => fitWithMean
    (LogisticRegression.scala:950-954) with a synthetic scaledMean of the
    data's scale (U(0, 0.014) per feature, not computed from the rows).
    The shard lives only in the row-block x column-tile layout (tiles.hip):
    it is generated on the device 512K rows at a time, appended, and each
    CSR chunk freed (157 GB resident for 200M rows).  Both passes are priced
    at SURVEY 8(d)'s 784 B/row (one fused pass's reads); the roofline line
    names the slower (dominant) one."""
    kernel = "k_tiles_grad"
    kernels = ("k_tiles_margin", "k_tiles_rows", "k_tiles_grad")

    def __init__(self, n, dev, rank):
        import numpy as np
        import torch
        from cycloneml_amd.optim import (BinaryLogisticBlockAggregator, DeviceInstanceBlock,
                                         RDDLossFunction, SparseTiles)
        self.n, self.F, self.k = n, 1_000_000, 64
        F, k = self.F, self.k
        # the layout's entry format: "auto" (compact for these rows' density),
        # CYC_TILES_FORMAT=wide|compact forces one
        self.tiles = SparseTiles(F, n, n * k, format=os.environ.get("CYC_TILES_FORMAT", "auto"))
        y = torch.empty(n, dtype=torch.float64, device=dev)
        self.sample = []                            # host copy of the first rows (CPU leg)
        sample_rows = min(n, 4 * LR_SPARSE_CHUNK)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s, e, rowptr, cols, vals, yc in lr_sparse_chunks(n, dev, rank, F, k):
            y[s:e] = yc
            self.tiles.append(rowptr, cols, vals)   # the CSR chunk is freed after
            if s < sample_rows:
                self.sample.append((cols.cpu().numpy(), vals.cpu().numpy()))
            del rowptr, cols, vals, yc
        torch.cuda.synchronize()
        self.prep_ms = (time.perf_counter() - t0) * 1e3
        self.labels = y
        self.block = DeviceInstanceBlock(y, None, tiles=self.tiles, numFeatures=F)
        self.coef = np.random.default_rng(4).normal(size=F + 1) * 0.01
        # scaledMean = mean / std per feature: nonzero with probability k / F,
        # values U(0, 1) -- mean ~ 3.2e-5, std ~ 4.6e-3 -> scaledMean ~ 7e-3
        self.scaledMean = np.random.default_rng(5).uniform(0.0, 0.014, F)
        sm_dev = torch.as_tensor(self.scaledMean, device=dev)    # bcScaledMean, once
        inv_std = np.ones(F)                                      # bcInverseStd, once
        self.fn = RDDLossFunction([self.block], lambda c: BinaryLogisticBlockAggregator(
            inv_std, sm_dev, True, True, c, device=dev))

    def step(self):
        self.fn.calculate(self.coef)

    def work(self, kname, launches_per_step):
        if kname == "k_tiles_rows":           # the rows' epilogue: dot + label in, multiplier out
            return self.n * 24.0 / launches_per_step, HBM
        return self.n * (self.k * 12 + 8 + 8) / launches_per_step, HBM   # bytes

    def step_work(self):
        return self.n * (self.k * 12 + 8 + 8.0), HBM   # one evaluation's reads

    def extra_roofline(self, launches_per_step, avg_s):
        return {"layout_bytes": self.tiles.nbytes, "layout_format": self.tiles.format,
                "layout_entries": self.tiles.entries, "nonzeros": self.tiles.nnz,
                "note": "784 B/row = one fused pass (SURVEY 8d); the evaluation reads the "
                        "layout twice (margin pass, then gradient pass), 12 B per nonzero each"}

    def describe(self):
        return (f"binomial LR RDDLossFunction.calculate on CSR {self.n} rows x {self.F} "
                f"features, {self.k} nnz/row per GPU, fitIntercept+fitWithMean "
                "(BASELINE configs[4]: 200M rows in total, split over the GPUs, resident "
                "in the row-block x column-tile layout)")

    def cpu_baseline(self, seconds):
        import numpy as np
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        threads = cpu_threads()
        ci = np.concatenate([a for a, _ in self.sample])
        vv = np.concatenate([b for _, b in self.sample])
        m = ci.size // self.k
        rp = np.arange(0, m * self.k + 1, self.k, dtype=np.int64)
        y = self.labels[:m].cpu().numpy()

        def part(rng_):
            a, b = rng_
            st = dict(grad=np.zeros(self.F + 1), loss=0.0, weight=0.0)
            for s in range(a, b, 1345):     # CSR InstanceBlock of 1345 rows (1 MiB)
                e = min(b, s + 1345)
                oracle.binary_logistic_add(dict(labels=y[s:e], weights=None,
                                                rowptr=rp[s:e + 1] - rp[s],
                                                colidx=ci[rp[s]:rp[e]], values=vv[rp[s]:rp[e]],
                                                F=self.F), self.coef, True, True,
                                           self.scaledMean, st)
            return st
        t0 = time.perf_counter()
        part((0, 1345 * 4))
        per_row = (time.perf_counter() - t0) / (1345 * 4)
        rows = int(min(m, max(threads * 1345, seconds * threads / per_row)))
        step = rows // threads
        rows = step * threads
        ranges = [(i * step, (i + 1) * step) for i in range(threads)]
        el, _ = timed_parallel(part, ranges, threads)
        reps = 1
        if seconds > 0 and el < 0.5 * seconds:
            # the host sample is smaller than the CPU budget: repeat the data
            # pass (one RDDLossFunction.calculate each) to reach ~seconds of work
            reps = max(2, int(round(seconds / el)))
            el, _ = timed_parallel(lambda r: [part(r) for _ in range(reps)], ranges, threads)
        return {"value": rows * reps / el, "unit": "rows/s", "cores": threads, "kind": "port",
                "sample": f"{rows} rows of the same CSR data in 1345-row blocks (1 MiB), "
                          f"fitWithMean, {threads} partitions on {threads} threads, {reps} "
                          f"pass(es), {el:.1f} s"}


WORKLOADS = {"kmeans": KMeansWorkload, "gramian": GramianWorkload, "pca": PCAWorkload,
             "lr_multi": LRMultiWorkload, "lr_sparse": LRSparseWorkload}

# BLASBenchmark's published rates (values/s, best of >= 100 iterations) on a
# Xeon E5-2673 v4, OpenJDK 17: mllib-local/benchmarks/BLASBenchmark-jdk17-
# results.txt (line of the java / native row), the shapes of
# mllib-local/src/test/scala/org/apache/spark/ml/linalg/BLASBenchmark.scala.
BLAS_PUBLISHED = {   # name: (values per call, java M/s, native M/s, results.txt lines)
    "daxpy": (1e8, 175.0, 173.6, "10-11"),
    "ddot": (1e8, 682.2, 663.7, "62-63"),
    "dscal": (1e8, 190.9, 199.9, "114-115"),
    "dgemv[N]": (1e8, 1152.8, 951.8, "140-141"),
    "dgemv[T]": (1e8, 1241.1, 845.3, "153-154"),
    "dger": (1e8, 200.3, 198.1, "192-193"),
    "dspmv[U]": (1e4 * (1e4 + 1) / 2, 858.1, 815.4, "205-206"),
    "dspr[U]": (1e4 * (1e4 + 1) / 2, 194.8, 201.2, "218-219"),
    "dsyr[U]": (1e4 * (1e4 + 1) / 2, 111.8, 112.9, "231-232"),
    "dgemm[N,N]": (1e9, 2511.5, 1429.6, "244-245"),
    "dgemm[N,T]": (1e9, 2402.5, 1344.7, "257-258"),
    "dgemm[T,N]": (1e9, 2448.6, 900.4, "270-271"),
    "dgemm[T,T]": (1e9, 2818.4, 909.5, "283-284"),
}


def run_blas(args, cpu_seconds):
    """The per-call drop-in layer (libcyclone_blas.so, include/cyclone_blas.h)
    timed the way BLASBenchmark times netlib: host arrays in, host arrays
    out, one synchronous Fortran-ABI call per iteration at the benchmark's
    shapes (BLASBenchmark.scala:76-340), the output operand cloned inside
    the iteration as the benchmark's `y.clone` / `a.clone` does; rate =
    values / best time (core/src/test/.../benchmark/Benchmark.scala:163-169).
    PCIe is inside every call (operands to HBM and the result back).
    vs_baseline = rate / the published java rate (the faster JVM provider
    on that host for every routine but dspr/dsyr)."""
    import numpy as np
    from cycloneml_amd import blas as B
    L = B.load()
    nb = B.nativeBLAS
    rnd = np.random.default_rng(0)
    iters = max(3, args.steps)
    n1 = int(1e8)
    x1, y1 = rnd.random(n1), rnd.random(n1)
    m2 = int(1e4)
    A2 = rnd.random(m2 * m2)
    xv, yv = rnd.random(m2), rnd.random(m2)
    AP = rnd.random(m2 * (m2 + 1) // 2)
    g = int(1e3)
    Ag, Bg, Cg = rnd.random(g * g), rnd.random(g * g), rnd.random(g * g)
    a, b = 0.7, 0.3
    cases = {
        "daxpy": lambda: nb.daxpy(n1, a, x1, 1, y1.copy(), 1),
        "ddot": lambda: nb.ddot(n1, x1, 1, y1, 1),
        "dscal": lambda: nb.dscal(n1, a, x1.copy(), 1),
        "dgemv[N]": lambda: nb.dgemv("N", m2, m2, a, A2, m2, xv, 1, b, yv.copy(), 1),
        "dgemv[T]": lambda: nb.dgemv("T", m2, m2, a, A2, m2, xv, 1, b, yv.copy(), 1),
        "dger": lambda: nb.dger(m2, m2, a, xv, 1, yv, 1, A2.copy(), m2),
        "dspmv[U]": lambda: nb.dspmv("U", m2, a, AP, xv, 1, b, yv.copy(), 1),
        "dspr[U]": lambda: nb.dspr("U", m2, a, xv, 1, AP.copy()),
        "dsyr[U]": lambda: nb.dsyr("U", m2, a, xv, 1, A2.copy(), m2),
        "dgemm[N,N]": lambda: nb.dgemm("N", "N", g, g, g, a, Ag, g, Bg, g, b, Cg.copy(), g),
        "dgemm[N,T]": lambda: nb.dgemm("N", "T", g, g, g, a, Ag, g, Bg, g, b, Cg.copy(), g),
        "dgemm[T,N]": lambda: nb.dgemm("T", "N", g, g, g, a, Ag, g, Bg, g, b, Cg.copy(), g),
        "dgemm[T,T]": lambda: nb.dgemm("T", "T", g, g, g, a, Ag, g, Bg, g, b, Cg.copy(), g),
    }
    rates = {}
    t_all = time.perf_counter()
    for name, fn in cases.items():
        vals, java, native, lines = BLAS_PUBLISHED[name]
        for _ in range(2):
            fn()
        best, tot = float("inf"), 0.0
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            t = time.perf_counter() - t0
            best, tot = min(best, t), tot + t
        rate = vals / best / 1e6
        rates[name] = {"rate_M_per_s": rate, "best_ms": best * 1e3, "avg_ms": tot / iters * 1e3,
                       "published_java_M_per_s": java, "published_native_M_per_s": native,
                       "vs_java": rate / java, "vs_native": rate / native,
                       "published_source": f"BLASBenchmark-jdk17-results.txt:{lines}"}
    el = time.perf_counter() - t_all
    del L
    # the oracle's netlib restatements on one host core, same shapes (a
    # netlib call is single-threaded: docs/ml-linalg-guide.md:79-91)
    cpu = None
    if cpu_seconds > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        O = oracle.lib()
        t0 = time.perf_counter()
        O.orc_ddot(oracle._p(x1), oracle._p(y1), n1)
        t_dot = time.perf_counter() - t0
        U = AP.copy()
        t0 = time.perf_counter()
        O.orc_dspr_upper(m2, a, oracle._p(xv), oracle._p(U))
        t_spr = time.perf_counter() - t0
        cpu = {"value": n1 / t_dot, "unit": "values/s (ddot n=1e8)", "cores": 1, "kind": "port",
               "dspr_values_per_s": BLAS_PUBLISHED["dspr[U]"][0] / t_spr,
               "sample": "the oracle's netlib ddot (n = 1e8) and dspr('U', n = 1e4) loops "
                         "(-ffp-contract=off), one call each on one host core",
               "host": _cores_info()}
    geo = float(np.exp(np.mean([np.log(r["vs_java"]) for r in rates.values()])))
    return {
        "metric": "BLASBenchmark rate (values/s) through the per-call netlib ABI",
        "value": rates["dgemm[N,N]"]["rate_M_per_s"] * 1e6, "unit": "values/s (dgemm[N,N])",
        "n_gpus": 1, "steps": iters, "warmup": 2,
        "ms_per_step": rates["dgemm[N,N]"]["best_ms"], "higher_is_better": True,
        "scaling": "none", "vs_baseline": rates["dgemm[N,N]"]["vs_java"],
        "vs_baseline_geomean_all_routines": geo,
        "dtype": "f64", "data": "synthetic host arrays (numpy PCG64 seed 0)",
        "config": {"workload": "BLASBenchmark shapes through libcyclone_blas.so: level 1 "
                               "n = 1e8, level 2 1e4 x 1e4 (packed n = 1e4), dgemm 1e3^3; host "
                               "operands, PCIe in every call",
                   "baseline": "published java rate, Xeon E5-2673 v4 @ 2.3 GHz, OpenJDK 17"},
        "routines": rates, "cpu_baseline": cpu, "elapsed_s": el,
    }


def launch_ranks(args) -> int:
    """`--gpus N` without a torch.distributed environment: start N fresh rank
    processes (one per GPU) through torch.distributed.run as a CHILD process
    -- this process has not touched the GPU -- and return its exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def run_workload(name, args, dev, rank, world, cpu_seconds):
    """Build one workload's resident data, time args.steps steps after
    args.warmup, and return its result dict (the JSON line's fields)."""
    import torch
    import torch.distributed as dist
    from cycloneml_amd import _native as N
    from cycloneml_amd import parallel
    n, mode, total_rows = rows_per_gpu(name, args.scaling, world, rank, args.rows)
    t_build = time.perf_counter()
    wl = WORKLOADS[name](n, dev, rank)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t_build
    for _ in range(args.warmup):
        wl.step()
    torch.cuda.synchronize()
    kernels = getattr(wl, "kernels", (wl.kernel,))
    # The timed steps carry HIP events only around the PRICED kernels (those
    # with an algorithmic work figure): each timed launch adds two event
    # markers to the stream (~0.12 ms of a 9.6 ms KMeans iteration with all
    # eight tiers timed).  The other kernels' times come from a short pass
    # after the clock (diag_kernels_ms_per_step).  CYC_BENCH_NO_EVENTS=1: no
    # events at all (a measurement switch; the roofline fields read zero).
    priced = [k for k in kernels if wl.work(k, 1) is not None]
    wl.warmup = args.warmup
    if hasattr(wl, "before_timing"):
        wl.before_timing(args.steps)
    N.profile_only(priced)
    N.profile_enable(os.environ.get("CYC_BENCH_NO_EVENTS") != "1")
    for kname in kernels:
        N.profile_query(kname)            # reset
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wl.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if hasattr(wl, "after_steps"):
        wl.after_steps()
    prof = {kname: N.profile_query(kname) for kname in kernels}
    N.profile_enable(False)
    N.profile_only(None)
    el = parallel.max_over_ranks(el, dev)
    value = total_rows * args.steps / el
    diag = {}
    rest = [k for k in kernels if k not in priced]
    if rest and os.environ.get("CYC_BENCH_NO_EVENTS") != "1":
        dsteps = min(3, args.steps)
        N.profile_only(rest)
        N.profile_enable(True)
        for _ in range(dsteps):
            wl.step()
        torch.cuda.synchronize()
        for k in rest:
            ms_k, _ = N.profile_query(k)
            diag[k] = ms_k / dsteps
        N.profile_enable(False)
        N.profile_only(None)

    if hasattr(wl, "after_timing"):
        wl.after_timing()
    fit = None
    if hasattr(wl, "fit_once"):
        # a whole fit beside the steady-state iterations (same clock rules)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        iters = wl.fit_once()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        fel = parallel.max_over_ranks(time.perf_counter() - t0, dev)
        its = iters["iterations"]
        fit = {"fit_ms": fel * 1e3, "fit_ms_per_iteration": fel * 1e3 / max(its, 1),
               "rows_per_s_per_iteration": total_rows * its / fel, **iters}
    # Every priced kernel in its own units (work per launch / mean launch
    # duration from its HIP events), and the dominant one: the priced kernel
    # with the most time per step.
    priced_rows = {}
    for k in kernels:
        kms_k, launches_k = prof[k]
        if not launches_k or wl.work(k, 1) is None:
            continue
        per_launch_k, (bound_k, unit_k, peak_k, scale_k) = wl.work(k, launches_k / args.steps)
        avg_k = kms_k / launches_k / 1e3
        ach = per_launch_k / avg_k / scale_k
        pmc_k = getattr(wl, "pmc_names", {}).get(k, k)
        traffic_k, src_k = pmc_traffic(name, pmc_k, n)
        priced_rows[k] = {"bound": bound_k, "achieved": ach, "peak": peak_k, "unit": unit_k,
                          "frac": ach / peak_k, "avg_launch_ms": avg_k * 1e3,
                          "ms_per_step": kms_k / args.steps, "launches": launches_k,
                          "work_per_launch": per_launch_k, "traffic": traffic_k,
                          "traffic_source": src_k}
    kname = wl.kernel
    if priced_rows:
        kname = max(priced_rows, key=lambda k: priced_rows[k]["ms_per_step"])
    dom = priced_rows.get(kname)
    # the whole step against the roofline of its algorithmic work
    sw, (sbound, sunit, speak, sscale) = wl.step_work()
    step_ach = sw / (el / args.steps) / sscale
    step_frac = {"step_frac": step_ach / speak, "step_achieved": step_ach,
                 "step_bound": sbound, "step_unit": sunit, "step_work": sw,
                 "step_frac_rule": "algorithmic work per step / ms_per_step / peak"}
    kms, launches = prof[kname]
    avg_s = kms / max(launches, 1) / 1e3
    extra = wl.extra_roofline(launches / args.steps, avg_s) if (
        launches and hasattr(wl, "extra_roofline")) else {}
    cpu = None
    if rank == 0 and world == 1 and cpu_seconds > 0:
        cpu = wl.cpu_baseline(cpu_seconds)
        cpu["host"] = _cores_info()
    out = {
        "metric": "rows/s per training iteration",
        "value": value,
        "unit": "rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": mode,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic, generated on device (torch Philox, seeded per rank)",
        "config": {"workload": wl.describe(), "rows_per_gpu": n, "rows_total": total_rows,
                   "config_rows": CONFIG_ROWS[name],
                   "config_rows_are": "per GPU" if PER_GPU_CONFIG[name] else "total",
                   "parallelism": f"dp{world} (row shards, RCCL all-reduce merge)"},
        "roofline": {"kernel": kname,
                     "bound": dom["bound"] if dom else None,
                     "achieved": dom["achieved"] if dom else None,
                     "peak": dom["peak"] if dom else None,
                     "unit": dom["unit"] if dom else None,
                     "frac": dom["frac"] if dom else None,
                     "traffic": dom["traffic"] if dom else None,
                     "traffic_source": dom["traffic_source"] if dom else None,
                     "avg_launch_ms": avg_s * 1e3, "launches": launches,
                     "work_per_launch": dom["work_per_launch"] if dom else None,
                     "dominant_rule": "the priced kernel with the most time per step",
                     **step_frac,
                     "priced_kernels": priced_rows,
                     "kernels_ms_per_step": {k: prof[k][0] / args.steps for k in priced},
                     "diag_kernels_ms_per_step": diag,
                     **extra},
        "cpu_baseline": cpu,
        "build_s": build_s,
    }
    if getattr(wl, "prep", None):
        out["prep_ms"] = wl.prep
    if fit is not None:
        out["fit"] = fit
        out["fit_ms_per_iteration"] = fit["fit_ms_per_iteration"]
    if hasattr(wl, "close"):
        wl.close()
    del wl
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU")
    from cycloneml_amd.config import device_for_local_rank
    dev = torch.device("cuda", device_for_local_rank(local))   # CYCLONE_DEVICES
    torch.cuda.set_device(dev)
    if world > 1:
        # host-side group only (rendezvous, RCCL id, barriers): every device
        # collective goes through libcyclone's communicator below
        dist.init_process_group(DIST_BACKEND)

    from cycloneml_amd import _native as N
    from cycloneml_amd import parallel
    N.load()
    comm = parallel.init(dev)          # libcyclone's RCCL communicator (cyc_comm_*)
    if comm is not None:
        world = comm.world_size        # n_gpus as the live communicator reports it
    names = ORDER if args.workload == "all" else (args.workload,)
    if args.workload == "all" and world == 1:
        names = names + ("blas",)     # the per-call layer: one process, host operands
    results = {}
    for name in names:
        t0 = time.perf_counter()
        cpu_s = args.cpu_seconds if name == names[0] else min(args.cpu_seconds, 8.0)
        if name == "blas":
            results[name] = run_blas(args, cpu_s)
        else:
            results[name] = run_workload(name, args, dev, rank, world, cpu_s)
        if rank == 0:
            print(f"[bench] {name}: {results[name]['value'] / 1e6:.1f} M rows/s, "
                  f"{results[name]['ms_per_step']:.2f} ms/step "
                  f"(value {results[name]['value']:.4g} {results[name]['unit']}) "
                  f"({time.perf_counter() - t0:.0f} s with data build)",
                  file=sys.stderr, flush=True)
    if rank == 0:
        line = dict(results[names[0]])
        if len(names) > 1:
            line["workloads"] = {k: results[k] for k in names[1:]}
        print(json.dumps(line), flush=True)
    if world > 1:
        parallel.shutdown()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
