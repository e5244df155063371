#!/usr/bin/env python3
"""bench.py -- fp64 CSR SpMV on MI355X (BASELINE.json metric).

Workload (BASELINE configs[1]): synthetic non-uniform
n = 2e6 CSR, rows < n/8 hold 96 nnz and the rest 9 (nnz = 39,750,000),
distinct uniform-random sorted columns (seed 42), values U[0,1), x U[0,1)
(seed 43), y0 = 0, alpha/beta = the test_spmv constants (glibc rand(),
0.8401877172 / 0.3943829268).  One step = one y = alpha*A*x + beta*y over
the whole matrix with every input already resident in HBM; at N > 1 the
rows are dealt to the ranks in equal cyclic chunks (x replicated) and a step
also includes the RCCL allgather of the y slices plus their device-side
placement (strong scaling: the same matrix at every N).  The headline is
cold-cache (a 1 GiB read-only sweep before each
of the K timed steps, so that at N = 8 a rank's ~67 MB slice cannot sit in the
256 MB Infinity Cache; each step between its own barrier + synchronize pair,
the sweep outside the timed region; `--scrub write` is round 1's read+write
scrub, whose dirty lines the next step had to write back).  A cold step's time is its device span: HIP
events on the launch stream from before the kernel to after the exchange and
merge, max over ranks (the host's barrier round trips between scrub and step
are reported beside as `cold_host_wall_ms_per_step`).  The warm number (K
back-to-back steps between one barrier pair, host wall clock) is reported
beside it under `warm`.

  python bench.py [--gpus N --steps K --warmup W] [--algo auto|xsort|panel|rowsplit|csr5]
                  [--cache cold|warm] [--partition cyclic|nnz]

Default kernel (`auto`): the library's choice per rank slice (sblas_csr_pick):
`rowsplit` where consecutive entries of a row share x lines (e.g. --cols prefix),
else `xsort` while a rank holds >= 2M nonzeros (every N <= 8 on config 2), else
`panel`.  `xsort` (csrc/xsort.hip) = entries sorted by column inside
(row range x column group) blocks, column groups dealt to the XCDs so every
x gather stays in the XCD's own L2, lane-consecutive gathers, LDS fp64 row
accumulators.  Within the fp64 error bound of the sequential row sum but not
bitwise repeatable (LDS atomics); `--algo panel` (XCD-affine column panels of
the row-split kernel) is the fastest bitwise-deterministic kernel.
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Drivers (choose_driver): under a launcher (WORLD_SIZE set) one process per
GPU over torch.distributed + RCCL.  Without one, `--gpus N` (N > 1) runs ONE
process that drives N GPUs through the C-ABI context (sblas_ctx_*:
ncclCommInitAll over devices 0..N-1, resident slices, per-device kernels,
ncclAllGather or ncclAllReduce of y), the reference's own shape
(dspmv_test.cu:355-383 -> dspmv_mgpu_v1.cu:16-280: one host call drives all
GPUs); `--driver ctx` forces it at N = 1.  N above the visible devices exits
non-zero instead of measuring fewer GPUs.

Rank 0 prints ONE JSON line.  `roofline.achieved` = algorithmic bytes per
launch (12*nnz + 4*(m+1) + 8*n + 8*m + 8*m[beta!=0]) / average
duration of the SpMV kernel measured with HIP events on the launch stream.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "s-blas_amd"))

METRIC = "fp64 CSR SpMV GFLOP/s + achieved HBM GB/s (% roofline) at 1/2/4/8 MI355X"
ALPHA = 0.8401877171547095  # dspmv_test.cu:281 (glibc rand(), unseeded)
BETA = 0.39438292681909304  # dspmv_test.cu:282
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


class Workload:
    """The matrix a run measures.  `synth` (default) is BASELINE configs[1]'s
    scaled generator (rows generated per slice, as before); the others are
    SuiteSparse-class matrices generated once on the host: `stencil7` /
    `stencil27` (3-D finite-difference / FEM-block pattern on a grid^3 mesh,
    sblas_gen_stencil3d) and `rmat` (power-law graph, 2^scale vertices,
    sblas_gen_rmat).  rows(a, b) returns the (col, val) of rows [a, b)."""

    def __init__(self, args, sblas):
        self.kind, self.args, self.sblas = args.matrix, args, sblas
        if self.kind == "synth":
            self.n = args.nrows
            self.rowptr = sblas.gen_synth_rowptr(self.n, args.heavy, args.light)
            self._cv = None
        elif self.kind.startswith("stencil"):
            g = args.grid
            self.rowptr, col, val = sblas.gen_stencil3d(g, g, g, int(self.kind[7:]), seed=49)
            self.n = len(self.rowptr) - 1
            self._cv = (col, val)
        else:
            self.rowptr, col, val = sblas.gen_rmat(args.scale, 16, seed=50)
            self.n = len(self.rowptr) - 1
            self._cv = (col, val)
        self.nnz = int(self.rowptr[-1])

    def rows(self, a: int, b: int):
        if self._cv is None:
            return self.sblas.gen_synth_rows(self.n, self.rowptr, a, b, self.args.heavy, self.args.light,
                                             prefix=self.args.cols == "prefix", seed=42)
        rp = self.rowptr
        return self._cv[0][rp[a]:rp[b]], self._cv[1][rp[a]:rp[b]]

    @property
    def default(self) -> bool:
        """The configuration the committed PMC summaries were collected on."""
        a = self.args
        return self.kind == "synth" and a.cols == "random" and self.n == 2_000_000 and \
            (a.heavy, a.light) == (96, 9)

    def describe(self, algo: str) -> str:
        a = self.args
        if self.kind == "synth":
            return (f"synthetic non-uniform n={self.n} CSR fp64 SpMV, rows<n/8: {a.heavy} "
                    f"nnz else {a.light}, {a.cols} sorted cols (seed 42), "
                    f"y=alpha*A*x+beta*y, {algo} kernel")
        if self.kind.startswith("stencil"):
            return (f"{self.kind[7:]}-point 3-D stencil on a {a.grid}^3 grid (n={self.n}, nnz={self.nnz}; "
                    f"SuiteSparse-class structured matrix), y=alpha*A*x+beta*y, {algo} kernel")
        return (f"R-MAT power-law graph, scale {a.scale} (n={self.n}, nnz={self.nnz}, edge factor 16), "
                f"y=alpha*A*x+beta*y, {algo} kernel")


def _cpu_lib():
    import ctypes as C
    lib = C.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    f = lib.orc_csr_spmv_omp
    f.restype = None
    f.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_double,
                  C.c_double, C.c_void_p, C.c_int]
    g = lib.orc_csr_spmv
    g.restype = None
    g.argtypes = f.argtypes[:-1]
    return f, g


def _time_cpu(fn, args, extra, share, max_reps=200):
    """(reps, seconds per call) of fn over about `share` seconds, after one
    warm-up call (page-in, thread pool)."""
    fn(*args, *extra)
    reps, t0 = 0, time.perf_counter()
    while True:
        fn(*args, *extra)
        reps += 1
        el = time.perf_counter() - t0
        if el > share or reps >= max_reps:
            return reps, el / reps


def _interleave_memory():
    """Interleave this process's future pages over every online NUMA node
    (set_mempolicy(MPOL_INTERLEAVE), what `numactl --interleave=all` does; the
    image has no numactl), so a multi-socket host's threads read the matrix
    from every socket's memory.  Returns the node list string, or None."""
    try:
        with open("/sys/devices/system/node/online") as fh:
            spec = fh.read().strip()
    except OSError:
        return None
    nodes = []
    for part in spec.split(","):
        a, _, b = part.partition("-")
        nodes.extend(range(int(a), int(b or a) + 1))
    if len(nodes) < 2:
        return spec + " (one node: nothing to interleave)"
    import platform
    if platform.machine() != "x86_64":  # syscall 238 is set_mempolicy on x86_64 only
        return spec + f" (not interleaved: set_mempolicy syscall number unknown on {platform.machine()})"
    import ctypes as C
    mask = (C.c_ulong * 16)()
    for nd in nodes:
        mask[nd // 64] |= 1 << (nd % 64)
    libc = C.CDLL(None, use_errno=True)
    MPOL_INTERLEAVE, SYS_set_mempolicy = 3, 238  # x86_64
    if libc.syscall(SYS_set_mempolicy, MPOL_INTERLEAVE, mask, C.c_ulong(16 * 64)) != 0:
        return spec + f" (set_mempolicy failed: errno {C.get_errno()})"
    return spec + " (pages interleaved)"


def _cpu_quota():
    """The cgroup CPU quota (cores), or None when unlimited / unreadable."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as fh:
                txt = fh.read().strip()
        except OSError:
            continue
        if parse:
            q, per = parse(txt)
            if q == "max":
                return None
            return float(q) / float(per)
        q = float(txt)
        if q < 0:
            return None
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
            return q / float(fh.read().strip())
    return None


def cpu_baseline_child(args) -> int:
    """`bench.py --cpu-baseline-only`: regenerate the workload on the host (the
    generators are deterministic) and time the oracle port; prints one JSON
    object.  Runs in its own process so that the OpenMP runtime starts with
    the pinning environment cpu_baseline() sets (OMP_PROC_BIND is read once,
    when libgomp initialises -- in the bench process torch/libsblas have
    already done that).  SURVEY §8 M1-cpu asks for all host cores: the
    thread count is swept (16, 32, 64, 128, ... up to the affinity mask's
    CPU count, which is included), each count timed briefly, and the best
    count timed again as the median of 3 runs; pages are interleaved over
    the NUMA nodes first."""
    try:  # before libgomp loads: it pins the initial thread to the first place
        mask = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        mask = os.cpu_count() or 1
    numa = _interleave_memory()
    if args.cpu_leg == "spmm":
        return cpu_baseline_spmm_child(args, mask, numa)
    if args.cpu_leg == "sptrsv":
        return cpu_baseline_sptrsv_child(args)
    import sblas
    W = Workload(args, sblas)
    col, val = W.rows(0, W.n)
    x = sblas.gen_vector(W.n, 43)
    rp = np.ascontiguousarray(W.rowptr, np.int64)
    col = np.ascontiguousarray(col, np.int32)
    val = np.ascontiguousarray(val, np.float64)
    f, g = _cpu_lib()
    y = np.zeros(W.n)
    cargs = (W.n, rp.ctypes.data, col.ctypes.data, val.ctypes.data, x.ctypes.data, ALPHA, BETA, y.ctypes.data)
    counts = sorted({c for c in (16, 32, 64, 128, 256, 512) if c < mask} | {mask})
    gf = lambda t: 2.0 * W.nnz / t / 1e9  # noqa: E731
    budget = args.cpu_budget
    sweep = {}
    for c in counts:
        sweep[c] = gf(_time_cpu(f, cargs, (c,), budget * 0.25 / len(counts))[1])
    best = max(sweep, key=sweep.get)
    mt = [_time_cpu(f, cargs, (best,), budget * 0.4 / 3) for _ in range(3)]
    st = [_time_cpu(g, cargs, (), budget * 0.35 / 3) for _ in range(3)]
    t_mt = float(np.median([t for _, t in mt]))
    t_st = float(np.median([t for _, t in st]))
    quota = _cpu_quota()
    print(json.dumps({
        "value": round(gf(t_mt), 3), "unit": "GFLOP/s", "cores": best,
        "kind": "port", "cpu_model": _cpu_model(),
        "sample": (f"full matrix of the workload, orc_csr_spmv_omp (OpenMP, schedule dynamic, "
                   f"OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND')} OMP_PLACES={os.environ.get('OMP_PLACES')}, "
                   f"{mask} CPUs in the affinity mask, cgroup quota "
                   f"{'none' if quota is None else f'{quota:.1f} CPUs'}, NUMA {numa}); thread sweep "
                   + ", ".join(f"{c}: {v:.1f}" for c, v in sweep.items()) +
                   f" GFLOP/s; best {best} threads, median of {len(mt)} runs of "
                   f"{'/'.join(str(r) for r, _ in mt)} reps = {t_mt * 1e3:.2f} ms/SpMV (runs: "
                   f"{', '.join(f'{gf(t):.1f}' for _, t in mt)} GFLOP/s); single-core scalar port orc_csr_spmv, "
                   f"median of {len(st)} runs: {t_st * 1e3:.1f} ms/SpMV = {gf(t_st):.3f} GFLOP/s"),
        "thread_sweep_gflops": {str(c): round(v, 3) for c, v in sweep.items()},
        "affinity_cpus": mask, "cgroup_cpu_quota": quota, "numa": numa,
        "runs_gflops": [round(gf(t), 3) for _, t in mt],
        "single_core_value": round(gf(t_st), 3),
    }), flush=True)
    return 0


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_spmm_child(args, mask, numa) -> int:
    """configs[3]'s CPU baseline: the oracle's
    csrmm restatement orc_spmm_omp (OpenMP over rows of A, B row-major, the
    same C = -0.7*A*B + 0.8*C over the rail4284-shaped stand-in x 64 columns)
    with the SpMV baseline's thread sweep; the best count is timed again,
    median of 3.  B / C0 are host U[0,1) draws of the same shapes (the GPU leg
    draws them on the device: timing only, the values do not matter)."""
    import ctypes as C
    m, k, n = 4284, 1_092_610, 64
    rp, col, val, _ = _rail_matrix()
    rng = np.random.default_rng(45)
    B = rng.random((k, n))
    C0 = np.asfortranarray(rng.random((m, n)))
    lib = C.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    f = lib.orc_spmm_omp
    f.restype = None
    f.argtypes = [C.c_int, C.c_int, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                  C.c_int, C.c_double, C.c_void_p, C.c_int, C.c_void_p, C.c_int]
    rp32 = np.ascontiguousarray(rp, np.int32)
    Cw = np.array(C0, copy=True, order="F")
    cargs = (m, n, -0.7, rp32.ctypes.data, col.ctypes.data, val.ctypes.data, B.ctypes.data, n, 1, 0.8,
             Cw.ctypes.data, m, None)
    nnz = int(rp[-1])
    gf = lambda t: 2.0 * nnz * n / t / 1e9  # noqa: E731
    counts = sorted({c for c in (16, 32, 64, 128, 256, 512) if c < mask} | {mask})
    budget = args.cpu_budget * 0.5
    sweep = {c: gf(_time_cpu(f, cargs, (c,), budget * 0.4 / len(counts), 50)[1]) for c in counts}
    best = max(sweep, key=sweep.get)
    mt = [_time_cpu(f, cargs, (best,), budget * 0.6 / 3, 50) for _ in range(3)]
    t_mt = float(np.median([t for _, t in mt]))
    quota = _cpu_quota()
    print(json.dumps({
        "value": round(gf(t_mt), 3), "unit": "GFLOP/s", "cores": best, "kind": "port",
        "cpu_model": _cpu_model(),
        "sample": (f"full configs[3] product (m {m}, k {k}, nnz {nnz}, 64 columns), orc_spmm_omp (oracle "
                   f"restatement of cusparseDcsrmm's definition, OpenMP over rows, B row-major), "
                   f"OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND')} OMP_PLACES={os.environ.get('OMP_PLACES')}, "
                   f"{mask} CPUs in the affinity mask, cgroup quota "
                   f"{'none' if quota is None else f'{quota:.1f} CPUs'}, NUMA {numa}; thread sweep "
                   + ", ".join(f"{c}: {v:.1f}" for c, v in sweep.items()) +
                   f" GFLOP/s; best {best} threads, median of 3 runs of "
                   f"{'/'.join(str(r) for r, _ in mt)} reps = {t_mt * 1e3:.2f} ms per product"),
        "ms_per_call": round(t_mt * 1e3, 3),
        "thread_sweep_gflops": {str(c): round(v, 3) for c, v in sweep.items()},
        "affinity_cpus": mask, "cgroup_cpu_quota": quota,
    }), flush=True)
    return 0


def cpu_baseline_sptrsv_child(args) -> int:
    """configs[4]'s CPU baseline: the
    reference's OWN serial sync-free solver (sptrsv_syncfree_analyser +
    _executor, sptrsv/sptrsv_v1/src/sptrsv_syncfree_serialref.h:6-108,
    compiled in place into oracle/_ref/libsblas_ref.so) on the same
    known-answer system, one core; the figure is the executor time the
    reference itself prints (serialref.h:142-155: flop = 2*nnz over the
    executor), median of 3 solves, x checked against x_ref exactly.  Without
    oracle/_ref (reference checkout absent when the tree was built) the
    oracle's restatement orc_sptrsv_serial is timed instead (kind "port")."""
    import ctypes as C
    import sblas
    cp, ri, vi, xref, bi = config5_system(sblas)
    n, nnz = CONFIG5_N, len(ri)
    ref_path = os.path.join(ROOT, "oracle", "_ref", "libsblas_ref.so")
    P = C.c_void_p
    runs, exact = [], True
    if os.path.exists(ref_path):
        f = C.CDLL(ref_path).ref_sptrsv_serial_timed
        f.restype = C.c_int
        f.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P]
        kind, what = "reference", ("sptrsv_syncfree_analyser + _executor (the reference's serialref, "
                                   "oracle/_ref, compiled in place)")
        for _ in range(3):
            x = np.zeros(n)
            an, ex = C.c_double(), C.c_double()
            f(cp.ctypes.data, ri.ctypes.data, vi.ctypes.data, n, nnz, 0, 1, bi.ctypes.data, x.ctypes.data,
              C.byref(an), C.byref(ex))
            runs.append((an.value, ex.value))
            exact = exact and bool(np.array_equal(x, xref))
    else:
        g = C.CDLL(os.path.join(ROOT, "oracle", "liboracle.so")).orc_sptrsv_serial
        g.restype = C.c_int
        g.argtypes = [P, P, P, C.c_int, C.c_int, C.c_int, P, P]
        kind, what = "port", "orc_sptrsv_serial (oracle restatement; oracle/_ref absent)"
        for _ in range(3):
            x = np.zeros(n)
            t0 = time.perf_counter()
            g(cp.ctypes.data, ri.ctypes.data, vi.ctypes.data, n, 0, 1, bi.ctypes.data, x.ctypes.data)
            runs.append((0.0, (time.perf_counter() - t0) * 1e3))
            exact = exact and bool(np.array_equal(x, xref))
    ex_ms = float(np.median([e for _, e in runs]))
    an_ms = float(np.median([a for a, _ in runs]))
    print(json.dumps({
        "value": round(2.0 * nnz / (ex_ms * 1e-3) / 1e9, 4), "unit": "GFLOP/s", "cores": 1, "kind": kind,
        "cpu_model": _cpu_model(),
        "sample": (f"full configs[4] system (n {n}, nnz {nnz}), {what}, single core, median of 3 solves: "
                   f"executor {ex_ms:.1f} ms (the figure serialref.h:150-155 prints), analyser {an_ms:.1f} ms"),
        "executor_ms": round(ex_ms, 3), "analyser_ms": round(an_ms, 3),
        "check_exact_vs_xref": exact,
    }), flush=True)
    return 0


def cpu_baseline(args, leg="spmv"):
    """The oracle restatement (oracle/liboracle.so; for configs[4] the
    reference's own serial solver, oracle/_ref) timed on this host's cores, in
    a child process (cpu_baseline_child) with the threads pinned
    (OMP_PROC_BIND=close, OMP_PLACES=cores) and the thread count swept.  Only
    these legs of bench.py (and the post-timing checks) touch oracle/."""
    import subprocess
    env = dict(os.environ, OMP_PROC_BIND="close", OMP_PLACES="cores")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", "--cpu-leg", leg,
           "--matrix", args.matrix,
           "--nrows", str(args.nrows), "--heavy", str(args.heavy), "--light", str(args.light),
           "--cols", args.cols, "--grid", str(args.grid), "--scale", str(args.scale),
           "--cpu-budget", str(args.cpu_budget)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": f"cpu baseline child exited {r.returncode}: {r.stderr[-400:]}"}
    return json.loads(r.stdout.strip().splitlines()[-1])


def attach_cpu_baselines(out, args):
    """N = 1 lines: the headline's `cpu_baseline` plus one per BASELINE leg
    that the line carries: `config4.cpu_baseline`
    (SpMM, OpenMP restatement, thread-swept) and `config5.cpu_baseline` (the
    reference's own serial SpTRSV, one core)."""
    out["cpu_baseline"] = cpu_baseline(args)
    if isinstance(out.get("config4"), dict):
        out["config4"]["cpu_baseline"] = cpu_baseline(args, "spmm")
    if isinstance(out.get("config5"), dict):
        out["config5"]["cpu_baseline"] = cpu_baseline(args, "sptrsv")


def measured_peak(torch, sblas, dev, stream):
    """this GPU's streaming ceiling, measured with the
    library's hand-written probes (csrc/probe.hip: 16-B loads, 8 in flight
    per lane, grid-stride) over a 4 GiB buffer (16x the 256 MB Infinity
    Cache, so every pass streams from HBM): plain and non-temporal reads, and
    a 1 GiB -> 1 GiB copy; 4 / 8 / 16 workgroups per CU; best of 3 per shape,
    HIP events on the launch stream.  Reported beside the 8 TB/s spec, which
    stays the roofline's `peak`."""
    nbytes = 4 << 30
    src = torch.ones(nbytes // 8, dtype=torch.float64, device=dev)
    sink = torch.zeros(1, dtype=torch.float64, device=dev)
    dst = torch.empty(1 << 27, dtype=torch.float64, device=dev)  # 1 GiB
    sp = stream.cuda_stream
    best = {}
    with torch.cuda.stream(stream):
        for mode, nb, out in ((0, nbytes, sink), (1, nbytes, sink), (3, nbytes, sink), (4, nbytes, sink),
                              (2, 1 << 30, dst)):
            for wg in (2, 4, 8, 16):
                sblas.hbm_probe(mode, src.data_ptr(), out.data_ptr(), nb, wg, sp)
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    sblas.hbm_probe(mode, src.data_ptr(), out.data_ptr(), nb, wg, sp)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    moved = nb * (2 if mode == 2 else 1)
                    gbs = moved / (e0.elapsed_time(e1) * 1e-3) / 1e9
                    if gbs > best.get(mode, (0.0, 0))[0]:
                        best[mode] = (gbs, wg)
    del src, sink, dst
    names = {0: "read_grid_stride", 1: "read_nt_grid_stride", 3: "read_blocked", 4: "read_nt_blocked"}
    rd = max(best[k][0] for k in names)
    return {"read_GBps": round(rd, 1),
            **{f"{v}_GBps": round(best[k][0], 1) for k, v in names.items()},
            "copy_GBps": round(best[2][0], 1),
            "wg_per_cu": {**{v: best[k][1] for k, v in names.items()}, "copy": best[2][1]},
            "how": ("sblas_hbm_probe (csrc/probe.hip): 16-B loads, 8 in flight per lane, plain / non-temporal, "
                    "grid-stride / one contiguous span per workgroup, over 4 GiB (read) and 1 GiB -> 1 GiB "
                    "(copy, bytes read + written), 2/4/8/16 WG per CU, best of 3, HIP events")}


def choose_driver(gpus: int, env, ndev: int, requested: str = "auto", loopback: bool = False) -> str:
    """How `bench.py --gpus N` runs: "torch" (one process per GPU, started by
    a launcher that set WORLD_SIZE), "ctx" (one process driving N GPUs through
    sblas_ctx), or "single" (one process, one GPU, the persistent device
    API).  Raises ValueError (-> non-zero exit) when N cannot be measured as
    asked -- never silently fewer GPUs."""
    if gpus < 1:
        raise ValueError(f"--gpus {gpus}: need at least one GPU")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if requested == "ctx" and world > 1:
            raise ValueError("--driver ctx drives every GPU from one process: run it without a launcher")
        if world != gpus:
            raise ValueError(f"--gpus {gpus} but the launcher started WORLD_SIZE {world} ranks")
        return "ctx" if requested == "ctx" else "torch"
    if loopback:  # rehearsal of the ctx path: N context ranks wrapped onto the visible GPUs
        if ndev < 1:
            raise ValueError("--ctx-loopback needs at least one GPU")
        return "ctx"
    if gpus > ndev:
        raise ValueError(f"--gpus {gpus} but {ndev} GPU(s) visible: refusing to measure fewer GPUs")
    if requested == "torch" and gpus > 1:
        raise ValueError("--driver torch needs a launcher (torch.distributed.run) for --gpus > 1")
    if gpus == 1 and requested != "ctx":
        return "single"
    return "ctx"


def lib_sha256() -> str:
    """sha256 of the libsblas.so this process loaded (sblas.LIB_PATH)."""
    import hashlib
    import sblas
    h = hashlib.sha256()
    with open(sblas.LIB_PATH, "rb") as fh:
        for blk in iter(lambda: fh.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


TRAFFIC_NOTES = {}


def _stamped_traffic(name: str):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary
    profiles/pmc_<name>.json (tools/pmc_traffic.py: 2 x FETCH_SIZE + WRITE_SIZE,
    separate passes), reported only while that summary's `lib_sha256` equals
    the hash of the libsblas.so loaded now: a kernel change invalidates it
    and the line says so (TRAFFIC_NOTES) instead of carrying a stale number."""
    p = os.path.join(ROOT, "profiles", f"pmc_{name}.json")
    if not os.path.exists(p):
        TRAFFIC_NOTES[name] = "no committed PMC summary"
        return None
    try:
        with open(p) as fh:
            d = json.load(fh)
        stamp = d.get("lib_sha256")
        if stamp is None:
            TRAFFIC_NOTES[name] = f"{os.path.relpath(p, ROOT)} carries no lib_sha256 stamp"
            return None
        if stamp != lib_sha256():
            TRAFFIC_NOTES[name] = (f"{os.path.relpath(p, ROOT)} was measured on libsblas.so {stamp[:12]}, "
                                   f"this run loaded {lib_sha256()[:12]}: not reported")
            return None
        TRAFFIC_NOTES[name] = f"{os.path.relpath(p, ROOT)} (libsblas.so {stamp[:12]}, the loaded build)"
        return float(d["hbm_bytes_per_launch"])
    except Exception as e:  # noqa: BLE001
        TRAFFIC_NOTES[name] = f"unreadable PMC summary: {e}"
        return None


def pmc_traffic(algo_name: str):
    """HBM bytes per launch of the SpMV kernel `algo_name` (_stamped_traffic)."""
    return _stamped_traffic(algo_name)


CONFIG3 = ("BASELINE configs[2]: the same matrix, CSR5 segmented-sum kernel, rows split by nnz "
           "(spMV_mgpu_v1, dspmv_mgpu_v1.cu:60-94), y reduced with an all-reduce of the zero-padded "
           "y (dspmv_mgpu_v1.cu:235-248's merge as one collective)")


def config3_object(N, kern_max, xch_max, step_ms, nnz, dev_bytes, dev_kern, check, how, exchange=None,
                   traffic=None, **extra):
    """The `config3` object every bench line carries:
    kernel-only, exchange-only and total, max over devices."""
    achieved0 = dev_bytes[0] / (dev_kern[0] * 1e-3) / 1e9 if dev_kern[0] > 0 else 0.0
    agg = sum(dev_bytes) / (kern_max * 1e-3) / 1e9 if kern_max > 0 else 0.0
    out = {
        "what": CONFIG3,
        "n_gpus": N, "algo": "csr5", "partition": "nnz-balanced (spMV_mgpu_v1)",
        "exchange": exchange or ("allreduce" if N > 1 else "none (one device)"),
        "kernel_ms_max": round(kern_max, 5),
        "exchange_ms_max": round(xch_max, 5),
        "step_ms": round(step_ms, 5),
        "gflops": round(2.0 * nnz / (step_ms * 1e-3) / 1e9, 3),
        "kernel_only_gflops": round(2.0 * nnz / (kern_max * 1e-3) / 1e9, 3),
        "roofline": {"bound": "hbm", "achieved": round(achieved0, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved0 / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "aggregate_GBps": round(agg, 1), "aggregate_frac": round(agg / (HBM_PEAK_GBS * N), 4)},
        "kernel_ms_per_device": [round(k, 5) for k in dev_kern],
        "algorithmic_bytes_per_device": [int(b) for b in dev_bytes],
        "timing": how,
        "check": check,
    }
    out.update(extra)
    return out


ROW_COST = 3.0  # the cost-weighted split's per-row weight (ctx.hip kCtxRowCost)


def cost_weighted(c3):
    """The compact record of the cost-weighted partition's config3 leg."""
    keep = ("kernel_ms_max", "exchange_ms_max", "step_ms", "gflops", "kernel_only_gflops", "kernel_ms_per_device",
            "nnz_per_device", "check")
    out = {k: c3[k] for k in keep if k in c3}
    out["partition"] = (f"cost-weighted whole rows: contiguous ranges balancing sum(nnz_r + {ROW_COST:g}) "
                        "(sblas_partition_cost), no split rows, same all-reduce of the zero-padded y")
    return out


def ctx_config3(ctx, args, sblas, n, rowptr, col, val, x_h, evict, delay_us, profiled=False, partition=1):
    """configs[2] through the C-ABI context: the matrix re-uploaded as CSR5
    slices of the nnz split (partition 2: the cost-weighted whole-row split)
    with the SBLAS_CTX_ALLREDUCE exchange, timed with the default leg's cold
    protocol (scrub, device-side hold, aligning all-reduce, per-device
    spans), then one fresh step checked against the oracle (--check) with
    every device's y bit-identical."""
    N = ctx.ngpu
    ctx.upload(n, n, rowptr, col, val, sblas.CSR5, partition, sblas.CTX_ALLREDUCE)
    ctx.set_x(x_h)
    ctx.set_y(np.zeros(n))
    info = [ctx.slice_info(d) for d in range(N)]
    dev_bytes = [b if BETA != 0.0 else b - 8 * r for r, _, b in info]
    for _ in range(max(1, args.warmup)):
        ctx.spmv_ex(ALPHA, BETA)
    rows = []
    for _ in range(args.steps):
        evict()
        rows.append(ctx.spmv_ex(ALPHA, BETA, delay_us=delay_us, wait=True))
    st = np.array(rows)
    check = None
    if args.check:
        y0 = np.zeros(n)
        ctx.set_y(y0)
        ctx.spmv_ex(ALPHA, BETA)
        ys = [ctx.get_y(d) for d in range(N)]
        check = _oracle_check(rowptr, col, val, x_h, y0, ys)
    return config3_object(
        N, float(np.mean(st[:, 0])), float(np.mean(st[:, 1])), float(np.mean(st[:, 2])), int(rowptr[-1]),
        dev_bytes, [float(np.mean(st[:, 3 + 3 * d])) for d in range(N)], check,
        "cold steps (1 GiB read sweep before each), sblas_ctx_spmv_ex per-device spans, max over devices",
        exchange="allreduce", traffic=pmc_traffic("csr5") if profiled else None, nnz_per_device=[int(z) for _, z, _ in info])


CONFIG4 = ("BASELINE configs[3]: C = -0.7*A*B + 0.8*C (dspmm_baseline_test.cu:518-519), B dense of width 64 "
           "resident row-major, on a rail4284-shaped stand-in (m 4,284, k 1,092,610, nnz 11,279,748, uniform-random "
           "distinct sorted columns, seed 44; rail4284 itself is not in the container)")
CONFIG5 = ("BASELINE configs[4]: sync-free SpTRSV, forward solve of a unit-lower circuit5M-class stand-in "
           "(n 5,558,326, 5 off-diagonals per column in a band of 80,000, ~985 level sets; circuit5M is not in the "
           "container), integer known-answer system (off-diagonals 1..10, x_ref in 1..10, b = L x_ref exact)")


def _hold_events(torch, stream, fn):
    """One cold step's device time: a device-side hold queued ahead of the
    start event (so the host has enqueued the step before the stream reaches
    it), then HIP events on the launch stream around fn's two phases.
    fn(ev) records ev[1] between its phases; returns (phase 1, phase 2) ms."""
    ev = tuple(torch.cuda.Event(enable_timing=True) for _ in range(3))
    with torch.cuda.stream(stream):
        torch.cuda._sleep(500_000)
        ev[0].record(stream)
        fn(ev)
        ev[2].record(stream)
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])


_RAIL = {}


def _rail_matrix():
    """configs[3]'s rail4284-shaped stand-in, generated once per process."""
    if not _RAIL:
        sys.path.insert(0, os.path.join(ROOT, "s-blas_amd", "tools"))
        from bench_spmm import rail_like
        t0 = time.perf_counter()
        rp, col = rail_like(4284, 1_092_610, 11_279_748, 44)
        val = np.random.default_rng(45).random(11_279_748)
        _RAIL.update(rp=rp, col=col, val=val, gen_s=time.perf_counter() - t0)
    return _RAIL["rp"], _RAIL["col"], _RAIL["val"], _RAIL["gen_s"]


def config4_leg(args, torch, sblas, sblas_dist, dist, rank, world, dev_idx, evict, sync_barrier, split="rows"):
    """configs[3] on every line: the SpMM, rows of A split
    by nnz over the ranks (B replicated, C row slices all-gathered; the
    reference's dspmm_mgpu_baseline.cu:147-150 splits B/C columns instead),
    timed with the SpMV leg's cold protocol (1 GiB sweep, barrier, device-side
    hold, HIP events on the launch stream around kernel and all-gather), max
    over ranks; then one fresh product from C0 whose EVERY entry rank 0
    checks against the oracle's csrmm restatement under the per-entry fp64
    bound (dspmm_baseline_test.cu:544-549 checks every entry too).  split
    "grid" (N > 1, reported beside): row blocks x B/C column groups
    (sblas_dist.spmm_grid_shape)."""
    m, k, n = 4284, 1_092_610, 64
    alpha, beta = -0.7, 0.8
    rp, col, val, gen_s = _rail_matrix()
    dev = torch.device("cuda", dev_idx)
    B = torch.rand((k, n), dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(45))
    C0 = torch.rand((n, m), dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(46))
    stream = torch.cuda.Stream(device=dev)
    op = sblas_dist.DistSpMM(rp, col, val, k, n, world, rank, dev_idx, torch, dist, split=split)
    sp = stream.cuda_stream
    with torch.cuda.stream(stream):
        op.load_c(C0)
        t0 = time.perf_counter()
        op.kernel(alpha, B, beta, sp)  # first call: builds the C-tile plan
        op.exchange()
        torch.cuda.synchronize()
        first_s = time.perf_counter() - t0
        for _ in range(max(1, args.warmup)):
            op.kernel(alpha, B, beta, sp)
            op.exchange()
        torch.cuda.synchronize()

    def step(ev):
        op.kernel(alpha, B, beta, sp)
        ev[1].record(stream)
        op.exchange()

    kern, xch = [], []
    for _ in range(args.steps):
        evict()
        sync_barrier()
        a, b = _hold_events(torch, stream, step)
        kern.append(a)
        xch.append(b)
        sync_barrier()
    r0, r1 = op.r0, op.r1
    wc = op.wc if split == "grid" else n  # the rank's C (and B) columns
    lnnz = int(rp[r1] - rp[r0])
    lbytes = 12 * lnnz + 4 * (r1 - r0 + 1) + 8 * k * wc + 16 * (r1 - r0) * wc
    mine = np.array([np.mean(kern), np.mean(xch), np.mean(np.array(kern) + np.array(xch)), lbytes, lnnz])
    per = _gather_rows(torch, dist, dev, mine, world)
    check = None
    if args.check_legs:
        with torch.cuda.stream(stream):
            op.load_c(C0)
            op.kernel(alpha, B, beta, sp)
            op.exchange()
        torch.cuda.synchronize()
        if rank == 0:
            got = op.result().cpu().numpy()  # (n, m): C column-major
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import orc  # oracle: checker only
            want, bound = orc.spmm_checked(m, n, alpha, rp, col, val, B.cpu().numpy(), beta, C0.cpu().numpy().T)
            diff = np.abs(got.T - want)
            check = {"entries": int(diff.size), "pass": bool(np.all(diff <= bound)),
                     "max_excess_over_bound": float(np.max(diff - bound)),
                     "abs_1e-3": bool(np.all(diff < 1e-3 * np.maximum(1.0, np.abs(want))))}
    shape = (op.R, op.Cg) if split == "grid" else None
    op.close()
    del B, C0
    if split == "grid":
        return config4_grid_object(per, shape, check)
    return config4_object(world, per, first_s, gen_s, check,
                          _stamped_traffic("spmm_ctile") if world == 1 else None)


def config4_grid_object(per, shape, check):
    """`config4.grid` (N > 1): the same step over the 2-D split."""
    per = np.asarray(per, np.float64)
    kmax, xmax, smax = (float(per[:, i].max()) for i in range(3))
    flops = 2.0 * 11_279_748 * 64
    return {
        "partition": (f"{shape[0]} row block(s) of A by nnz x {shape[1]} column group(s) of B/C "
                      "(sblas_dist.spmm_grid_shape), C blocks all-gathered"),
        "row_blocks": shape[0], "column_groups": shape[1],
        "kernel_ms_max": round(kmax, 5), "exchange_ms_max": round(xmax, 5), "step_ms": round(smax, 5),
        "gflops": round(flops / (smax * 1e-3) / 1e9, 3),
        "kernel_ms_per_rank": [round(float(v), 5) for v in per[:, 0]],
        "algorithmic_bytes_per_rank": [int(b) for b in per[:, 3]],
        "check": check,
    }


def config4_object(world, per, first_s, gen_s, check, traffic):
    """The `config4` object: per = one row per rank of
    (kernel ms, all-gather ms, step ms, algorithmic bytes, nnz)."""
    per = np.asarray(per, np.float64)
    kmax, xmax, smax = (float(per[:, i].max()) for i in range(3))
    achieved0 = float(per[0, 3]) / (per[0, 0] * 1e-3) / 1e9
    flops = 2.0 * float(per[:, 4].sum()) * 64
    return {
        "what": CONFIG4,
        "n_gpus": world, "algo": "C tile (k_spmm_ctile, column-sorted, LDS accumulators)",
        "partition": "single GPU" if world == 1 else "whole-row blocks of A by nnz, B replicated, C all-gathered",
        "kernel_ms_max": round(kmax, 5), "exchange_ms_max": round(xmax, 5), "step_ms": round(smax, 5),
        "gflops": round(flops / (smax * 1e-3) / 1e9, 3),
        "kernel_only_gflops": round(flops / (kmax * 1e-3) / 1e9, 3),
        "algorithmic_bytes_per_rank": [int(b) for b in per[:, 3]],
        "algorithmic_bytes_formula": "12*nnz + 4*(m+1) + 8*k*ncols + 16*m*ncols (SURVEY M1-bytes-SpMM)",
        "roofline": {"bound": "hbm", "achieved": round(achieved0, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved0 / HBM_PEAK_GBS, 4), "traffic": traffic},
        "kernel_ms_per_rank": [round(float(v), 5) for v in per[:, 0]],
        "nnz_per_rank": [int(v) for v in per[:, 4]],
        "first_call_s": round(first_s, 3), "host_gen_s": round(gen_s, 2),
        "timing": ("cold steps (1 GiB read sweep before each, barrier, device-side hold), HIP events on the "
                   "launch stream around the kernel and the C all-gather, max over ranks"),
        "check": check,
    }


CONFIG5_N = 5_558_326


def config5_system(sblas):
    """configs[4]'s integer known-answer system: the unit-lower CSC stand-in
    (colptr, rowidx, val), x_ref in 1..10 and b = L x_ref (exact in fp64)."""
    n = CONFIG5_N
    cp, ri, _ = sblas.gen_lower_banded(n, 5, 80_000, 47)
    nnz = len(ri)
    cols = np.repeat(np.arange(n, dtype=np.int64), np.diff(cp))
    vi = np.random.default_rng(5).integers(1, 11, nnz).astype(np.float64)
    vi[cp[:-1]] = 1.0  # unit diagonal
    xref = np.floor(sblas.gen_vector(n, 48) * 10.0) + 1.0
    bi = np.bincount(ri, weights=vi * xref[cols], minlength=n)  # integers < 2^53: exact
    return cp, ri, vi, xref, bi


def config5_leg(args, torch, sblas, rank, world, evict, sync_barrier):
    """configs[4] on every line: the sync-free SpTRSV.
    Rank 0 solves the integer known-answer system (x must equal x_ref
    exactly) with (1) the single-device pull executor (algo 4 = AUTO ticket
    order; sptrsv_syncfree_cuda.h:545-636's solve) and (2) configs[4]'s
    4-block partition (sblas_trsv_mgpu: nnz-balanced blocks of the solve
    order, block d on device d % visible, producers pushing x_i into later
    blocks' fine-grained x), each timed cold (1 GiB sweep on every device it
    uses before each solve).  The other ranks wait at the barrier."""
    n = CONFIG5_N
    out = {"what": CONFIG5, "n": n}
    if rank == 0:
        t0 = time.perf_counter()
        cp, ri, vi, xref, bi = config5_system(sblas)
        nnz = len(ri)
        gen_s = time.perf_counter() - t0
        dev = torch.device("cuda", torch.cuda.current_device())
        stream = torch.cuda.Stream(device=dev)
        dcp, dri, dv, db = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (cp, ri, vi, bi))
        dx = torch.zeros(n, dtype=torch.float64, device=dev)
        t0 = time.perf_counter()
        T = sblas.DeviceTRSV(dev.index, n, nnz, dcp.data_ptr(), dri.data_ptr(), dv.data_ptr(), 0)
        setup_s = time.perf_counter() - t0
        levels, order = T.levels(), T.pick()
        sp = stream.cuda_stream
        with torch.cuda.stream(stream):
            T.solve(4, db.data_ptr(), dx.data_ptr(), sp)  # warm-up
        torch.cuda.synchronize()
        ms = []
        for _ in range(args.steps):
            evict()
            torch.cuda.synchronize()  # the sweep runs on another stream: finish it first
            ms.append(_hold_events(torch, stream, lambda ev: (T.solve(4, db.data_ptr(), dx.data_ptr(), sp),
                                                              ev[1].record(stream)))[0])
        exact = bool(np.array_equal(dx.cpu().numpy(), xref))
        T.close()
        del dcp, dri, dv, db, dx
        out.update(config5_single(nnz, levels, order, float(np.mean(ms)), exact, gen_s, setup_s))
        # configs[4]'s 4-way partition: on min(4, visible) GPUs when this
        # process is the only one (N = 1); under a launcher the other GPUs
        # belong to the other ranks (busy in the barrier), so the 4 blocks
        # stay on this rank's GPU.  A failure here is reported, not raised:
        # the blocks' cross-GPU protocol must not take the line down with it.
        ndev = torch.cuda.device_count() if world == 1 else 1
        gpus = 4 if ndev >= 4 else 2 if ndev >= 2 else 1
        try:
            out["blocks4"] = config5_blocks4(args, torch, sblas, cp, ri, vi, n, nnz, bi, xref, gpus, evict)
        except Exception as e:  # noqa: BLE001
            out["blocks4"] = {"blocks": 4, "gpus": gpus, "error": f"{type(e).__name__}: {e}"}
    sync_barrier()
    return out


STRUCTURED = (("stencil27", "27-point 3-D stencil, 128^3 mesh (FEM-block pattern)", 128),
              ("stencil7", "7-point 3-D stencil, 160^3 mesh (finite-difference pattern)", 160),
              ("rmat", "R-MAT power-law graph, 2^21 vertices, edge factor 16", 21))


def structured_leg(args, torch, sblas, evict):
    """North star's ">= 60% of the HBM roofline on fp64 CSR SpMV for
    SuiteSparse-class matrices at 1 GPU" on every N = 1 line: SuiteSparse
    itself is not in the container, so the generators' structured stand-ins
    (sblas_gen_stencil3d, sblas_gen_rmat) run through the same persistent API
    as the headline -- AUTO's pick, y = alpha*A*x + beta*y, the call's device
    span (sblas_spmv_timed) after the 1 GiB sweep, mean of --steps -- and the
    roofline is the same algorithmic-bytes formula over 8 TB/s.  Correctness
    on these matrices is the -m gpu suite's (tests/test_spmv_gpu.py)."""
    out = {"what": "SuiteSparse-class stand-ins (north star: >= 0.60 of the HBM roofline at 1 GPU), "
                   "AUTO's kernel, cold device span, algorithmic bytes / 8 TB/s"}
    dev = torch.device("cuda", torch.cuda.current_device())
    stream = torch.cuda.Stream(device=dev)
    sp = stream.cuda_stream
    names = {sblas.ROWSPLIT: "rowsplit", sblas.CSR5: "csr5", sblas.PANEL: "panel", sblas.XSORT: "xsort"}
    for kind, what, size in STRUCTURED:
        t0 = time.perf_counter()
        A = None
        try:
            if kind == "rmat":
                rp, col, val = sblas.gen_rmat(size, 16, seed=50)
            else:
                rp, col, val = sblas.gen_stencil3d(size, size, size, int(kind[7:]), seed=49)
            n, nnz = len(rp) - 1, int(rp[-1])
            A = sblas.DeviceCSR.upload(dev.index, n, rp, col, val)
            del rp, col, val
            algo = A.pick(sp)
            A.analyse(algo, sp)
            build_s = time.perf_counter() - t0
            x = torch.from_numpy(sblas.gen_vector(n, 43)).to(dev)
            y = torch.from_numpy(sblas.gen_vector(n, 44)).to(dev)
            with torch.cuda.stream(stream):
                for _ in range(2):
                    A.spmv(algo, ALPHA, x.data_ptr(), BETA, y.data_ptr(), sp)
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.steps):
                evict()
                torch.cuda.synchronize()
                ts.append(A.spmv_timed(algo, ALPHA, x.data_ptr(), BETA, y.data_ptr(), sp))
            t = float(np.mean(ts))
            abytes = A.algorithmic_bytes(True)
            out[kind] = {"matrix": what, "n": n, "nnz": nnz, "algo": names.get(algo, str(algo)),
                         "kernel_ms": round(t, 5), "gflops": round(2.0 * nnz / (t * 1e-3) / 1e9, 3),
                         "algorithmic_bytes": abytes,
                         "roofline_frac": round(abytes / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "build_s": round(build_s, 2)}
            del x, y
        except Exception as e:  # noqa: BLE001 -- reported, not raised: the headline must not fall with it
            out[kind] = {"matrix": what, "error": f"{type(e).__name__}: {e}"}
        finally:
            if A is not None:
                A.close()
    return out


def config5_blocks4(args, torch, sblas, cp, ri, vi, n, nnz, bi, xref, gpus, evict):
    """configs[4]'s 4 blocks (sblas_trsv_mgpu, 4 // gpus blocks per GPU), cold."""
    t0 = time.perf_counter()
    H = sblas.TrsvMgpu(cp, ri, vi, n, gpus, tasks=4 // gpus)
    try:
        build_s = time.perf_counter() - t0
        H.run(bi)  # warm-up
        scr = [torch.zeros(args.scrub_gib << 30, dtype=torch.uint8, device=torch.device("cuda", d))
               for d in range(1, gpus)]
        mms, ok = [], True
        for _ in range(args.steps):
            evict()
            torch.cuda.synchronize()
            for sc in scr:
                sc.sum(dtype=torch.int64)
            for d in range(gpus):
                torch.cuda.synchronize(d)
            x, t4 = H.run(bi)
            mms.append(t4)
            ok = ok and bool(np.array_equal(x, xref))
        del scr
        where = H.info()
    finally:
        H.close()
    out = config5_blocks(nnz, gpus, float(np.mean(mms)), ok, build_s)
    out["block_devices"] = [d for d, _ in where]
    out["block_rows"] = [r for _, r in where]
    return out


def config5_single(nnz, levels, order, t, exact, gen_s, setup_s):
    """configs[4]'s single-device figures, t in ms."""
    n = CONFIG5_N
    abytes = 12 * nnz + 4 * (n + 1) + 16 * n
    ach = abytes / (t * 1e-3) / 1e9
    return {
        "nnz": nnz, "levels": levels,
        "executor": "pull (CSR rows, NaN-sentinel x, ticketed waves), " +
                    ("level-order tickets" if order == 3 else "natural-order tickets"),
        "ms": round(t, 5), "gflops": round(2.0 * nnz / (t * 1e-3) / 1e9, 3),
        "algorithmic_bytes": int(abytes),
        "algorithmic_bytes_formula": "12*nnz + 4*(n+1) + 16*n (SURVEY M1-bytes-TRSV)",
        "roofline": {"bound": "latency (level chain); hbm reported", "achieved": round(ach, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None},
        "us_per_level": round(t * 1e3 / max(levels, 1), 3),
        "check_exact_vs_xref": exact,
        "timing": "cold steps (1 GiB sweep before each), device-side hold, HIP events on the launch stream",
        "host_gen_s": round(gen_s, 2), "analyse_s": round(setup_s, 3),
    }


def config5_blocks(nnz, gpus, t4, ok, build_s):
    """configs[4]'s 4-block partition figures (4 // gpus blocks per GPU), t4 in ms."""
    return {
        "blocks": 4, "gpus": gpus, "blocks_per_gpu": 4 // gpus, "ms": round(t4, 5), "gflops": round(2.0 * nnz / (t4 * 1e-3) / 1e9, 3),
        "check_exact_vs_xref": ok, "build_s": round(build_s, 3),
        "timing": ("cold steps; host wall clock from the first block's launch to the last device's "
                   "synchronize (sblas_trsv_mgpu_run), b upload and x reset before, x download after"),
        "note": ("blocks on distinct GPUs, x pushed over xGMI with system-scope stores" if gpus > 1 else
                 "one GPU visible: the 4 blocks run concurrently on it (the peer-store protocol on local "
                 "fine-grained memory)"),
    }


def peer_matrix(torch):
    """hipDeviceCanAccessPeer over the visible devices (1 on the diagonal)."""
    nd = torch.cuda.device_count()
    return [[1 if i == j else int(torch.cuda.can_device_access_peer(i, j)) for j in range(nd)]
            for i in range(nd)]


def _pci_bus(torch, d):
    p = torch.cuda.get_device_properties(d)
    bus = getattr(p, "pci_bus_id", None)
    return None if bus is None else f"{getattr(p, 'pci_domain_id', 0):04x}:{bus:02x}:{getattr(p, 'pci_device_id', 0):02x}"


def topology_object(driver, backend, nranks, ordinals, pci, peers, note=None):
    """What a multi-GPU line ran on: the communicator's
    rank count and each rank's device ordinal / PCI address, and the
    hipDeviceCanAccessPeer matrix of the visible devices."""
    out = {"driver": driver, "backend": backend, "comm_ranks": int(nranks),
           "device_ordinals": [int(d) for d in ordinals], "pci_bus": list(pci),
           "visible_devices": len(peers), "peer_access": peers,
           "all_pairs_peer": bool(all(all(r) for r in peers))}
    if note:
        out["note"] = note
    return out


def deterministic_leg(args, torch, sblas, op, algo, x, local_bytes, nnz, stream, evict):
    """`deterministic_beside` (N = 1): the headline's
    handle switched to deterministic mode (sblas_csr_set_deterministic: the
    same plan, xsort's ordered-add form), the same cold protocol; then two
    fresh launches from one y0 compared bit for bit."""
    A = op.A
    sp = stream.cuda_stream
    A.deterministic = True
    try:
        with torch.cuda.stream(stream):
            for _ in range(2):
                A.spmv(algo, ALPHA, x.data_ptr(), BETA, op.y_local.data_ptr(), sp)
            ts = []
            for _ in range(args.steps):
                evict()
                torch.cuda.synchronize()
                ts.append(A.spmv_timed(algo, ALPHA, x.data_ptr(), BETA, op.y_local.data_ptr(), sp))
            y0 = op.y_local.clone()
            ys = []
            for _ in range(2):
                y = y0.clone()
                A.spmv(algo, ALPHA, x.data_ptr(), BETA, y.data_ptr(), sp)
                ys.append(y)
            torch.cuda.synchronize()
        same = bool(torch.equal(ys[0], ys[1]))
    finally:
        A.deterministic = False
    t = float(np.mean(ts))
    names = {sblas.ROWSPLIT: "rowsplit", sblas.CSR5: "csr5", sblas.PANEL: "panel", sblas.XSORT: "xsort"}
    return {"algo": names.get(algo, str(algo)) + (" (ordered adds)" if algo == sblas.XSORT else ""),
            "kernel_ms": round(t, 5), "gflops": round(2.0 * nnz / (t * 1e-3) / 1e9, 3),
            "roofline_frac": round(local_bytes / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "bitwise_equal_two_launches": same, "cache": "cold",
            "how": "sblas_csr_set_deterministic(A, 1) on the headline's plan (SBLAS_DETERMINISTIC=1 sets it "
                   "for every new handle); AUTO's pick unchanged"}


def _gather_rows(torch, dist, dev, row, world):
    """Every rank's stats row (numpy), as a (world, len) array."""
    if dist is None:
        return np.asarray(row, np.float64)[None, :]
    use_dev = dist.get_backend() == "nccl"
    t = torch.tensor(np.asarray(row, np.float64), device=dev if use_dev else "cpu")
    parts = [t.clone() for _ in range(world)]
    dist.all_gather(parts, t)
    return np.stack([p.cpu().numpy() for p in parts])


def _oracle_check(rowptr, col, val, x_h, y0, ys):
    """Post-timing verification (oracle = checker only): ys[0] within the
    per-row fp64 bound of the sequential row sum, every other y bit-identical."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import orc  # oracle: checker only
    want = orc.csr_spmv(rowptr, col, val, x_h, ALPHA, BETA, y0)
    bound = orc.spmv_bound(rowptr, col, val, x_h, ALPHA, BETA, y0)
    return bool(np.all(np.abs(ys[0] - want) <= bound)) and all(np.array_equal(ys[0], y) for y in ys[1:])


def torch_config3(args, W, sblas, sblas_dist, torch, dist, rank, world, dev_idx, x, x_h, stream, evict,
                  sync_barrier, row_cost=None):
    """configs[2] under the launcher (one process per GPU): the nnz split's
    slice as a CSR5 handle (sblas_dist.DistSpMV, exchange "allreduce" =
    torch.distributed.all_reduce = ncclAllReduce of the zero-padded y), timed
    cold like the default leg: per step a 1 GiB sweep, barrier, device-side
    hold, HIP events on the launch stream around kernel and exchange, max
    over ranks.  At world 1 the span is sblas_spmv_timed's (no exchange)."""
    n, rowptr = W.n, W.rowptr
    plan = sblas_dist.make_plan(rowptr, n, world, row_cost=row_cost)
    r0, r1, i0, i1, _ = plan.local(rank)
    col_rows, val_rows = W.rows(r0, r1)
    off = i0 - int(rowptr[r0])
    col = np.ascontiguousarray(col_rows[off:off + (i1 - i0)])
    val = np.ascontiguousarray(val_rows[off:off + (i1 - i0)])
    op = sblas_dist.DistSpMV(plan, rank, dev_idx, rowptr, col, val, sblas.CSR5, torch, dist, "allreduce")
    sp = stream.cuda_stream
    local_bytes = op.A.algorithmic_bytes(BETA != 0.0)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        op.kernel(ALPHA, x, BETA, sp)
        if ev is not None:
            ev[1].record(stream)
        op.exchange(sp)
        if ev is not None:
            ev[2].record(stream)

    kern, xch, span = [], [], []
    with torch.cuda.stream(stream):
        for _ in range(max(1, args.warmup)):
            step()
        for _ in range(args.steps):
            evict()
            sync_barrier()
            if world == 1:
                ms = op.A.spmv_timed(op.algo, ALPHA, x.data_ptr(), BETA, op.y_local.data_ptr(), sp)
                kern.append(ms)
                xch.append(0.0)
                span.append(ms)
            else:
                ev = tuple(torch.cuda.Event(enable_timing=True) for _ in range(3))
                torch.cuda._sleep(500_000)
                step(ev)
                sync_barrier()
                kern.append(ev[0].elapsed_time(ev[1]))
                xch.append(ev[1].elapsed_time(ev[2]))
                span.append(ev[0].elapsed_time(ev[2]))
        sync_barrier()
    dev = torch.device("cuda", dev_idx)
    use_dev = dist is None or dist.get_backend() == "nccl"
    mine = torch.tensor([np.mean(kern), np.mean(xch), np.mean(span)], dtype=torch.float64,
                        device=dev if use_dev else "cpu")
    per = [mine.clone() for _ in range(world)]
    byts = torch.tensor([float(local_bytes)], dtype=torch.float64, device=mine.device)
    allb = [byts.clone() for _ in range(world)]
    if dist is not None:
        dist.all_gather(per, mine)
        dist.all_gather(allb, byts)
    per = [p.cpu().numpy() for p in per]
    check = None
    if args.check:
        with torch.cuda.stream(stream):
            op.load_y(torch.zeros(plan.m, dtype=torch.float64, device=dev))
            step()
        torch.cuda.synchronize()
        y = op.result().clone()
        same = True
        if dist is not None:  # every rank's y bit-identical: elementwise max == min == own
            yy = y if use_dev else y.cpu()
            hi, lo = yy.clone(), yy.clone()
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            same = bool(torch.equal(hi, yy) and torch.equal(lo, yy))
        if rank == 0:
            col_all, val_all = W.rows(0, n)
            check = _oracle_check(rowptr, col_all, val_all, x_h, np.zeros(plan.m), [y.cpu().numpy()]) and same
        elif not same:
            check = False
    panels = op.A.panels(sblas.CSR5)
    op.close()
    return config3_object(
        world, max(p[0] for p in per), max(p[1] for p in per), max(p[2] for p in per), W.nnz,
        [float(b.item()) for b in allb], [float(p[0]) for p in per], check,
        ("cold steps: sblas_spmv_timed device span (one GPU, no exchange)" if world == 1 else
         "cold steps: HIP events on the launch stream around kernel and exchange after a device-side "
         "hold, max over ranks"),
        traffic=pmc_traffic("csr5") if (world == 1 and W.default) else None,
        xcd_panels_rank0=panels,
        nnz_per_device=[int(plan.end_idx[d] - plan.start_idx[d] + 1) for d in range(world)])


def run_ctx(args) -> int:
    """One process drives args.gpus GPUs through the C-ABI context
    (csrc/ctx.hip): ncclCommInitAll over devices 0..N-1, each device's slice
    resident, per-device SpMV kernels, then the exchange (ncclAllGather +
    device placement, or the literal ncclAllReduce of the zero-padded y).
    A cold step: a 1 GiB sweep on every device, then sblas_ctx_spmv_ex with
    its timing protocol (each stream waits on the device while the host
    enqueues the step, a one-word all-reduce lines the devices up), so a
    device's span runs from its start event to the end of its exchange; the
    step is the max over devices.  Replaces dspmv_test.cu:355-383 ->
    dspmv_mgpu_v1.cu:16-280 (one host call driving every GPU)."""
    import torch
    import sblas

    N = args.gpus
    ndev = torch.cuda.device_count()
    if args.ctx_loopback:
        os.environ["SBLAS_CTX_LOOPBACK"] = "1"  # read by sblas_ctx_create
    algo_ids = {"rowsplit": sblas.ROWSPLIT, "csr5": sblas.CSR5, "panel": sblas.PANEL,
                "xsort": sblas.XSORT}
    t_gen = time.perf_counter()
    W = Workload(args, sblas)
    n, rowptr, nnz = W.n, W.rowptr, W.nnz
    col, val = W.rows(0, n)
    x_h = sblas.gen_vector(n, 43)
    t_gen = time.perf_counter() - t_gen
    exchange = sblas.CTX_ALLREDUCE if args.exchange == "allreduce" else sblas.CTX_ALLGATHER
    partition = 1 if (args.partition == "nnz" or exchange == sblas.CTX_ALLREDUCE) else 0
    algo = sblas.AUTO if args.algo == "auto" else algo_ids[args.algo]
    # RCCL prints its version banner on stdout at communicator creation; the
    # contract's stdout is ONE JSON line, so fd 1 points at stderr meanwhile
    sys.stdout.flush()
    saved_fd = os.dup(1)
    os.dup2(2, 1)
    try:
        ctx = sblas.DeviceCtx(N)
    finally:
        sys.stdout.flush()
        os.dup2(saved_fd, 1)
        os.close(saved_fd)
    t0 = time.perf_counter()
    if args.overlap > 1 and partition == 0 and exchange == sblas.CTX_ALLGATHER:
        # exchange overlapped over K parts of each device's chunks
        ctx.upload_parts(n, n, rowptr, col, val, algo, args.overlap)
    else:
        ctx.upload(n, n, rowptr, col, val, algo, partition, exchange)
    parts = ctx.parts()
    plan_s = time.perf_counter() - t0
    # AUTO: each device's slice decided by the library (sblas_csr_pick); the
    # line names device 0's and lists all of them
    names = {v: k for k, v in algo_ids.items()}
    dev_algos = [names[ctx.slice_algo(d)] for d in range(N)]
    args.algo = dev_algos[0]
    ctx.set_x(x_h)
    ctx.set_y(np.zeros(n))
    info = [ctx.slice_info(d) for d in range(N)]
    beta_nz = BETA != 0.0
    # per-device algorithmic bytes (sblas_spmv_algorithmic_bytes; beta != 0)
    dev_bytes = [b if beta_nz else b - 8 * r for r, _, b in info]
    delay_us = 300.0 + 150.0 * N
    for _ in range(args.warmup):
        ctx.spmv_ex(ALPHA, BETA)
    devs = sorted({d % ndev for d in range(N)})  # physical devices (wrapped in loopback)
    scrubs = [torch.zeros(args.scrub_gib << 30, dtype=torch.uint8, device=torch.device("cuda", d)) for d in devs]

    def sync_all():
        for d in devs:
            torch.cuda.synchronize(d)

    def evict():
        for sc in scrubs:
            if args.scrub == "write":
                sc.add_(1)
            else:
                sc.sum(dtype=torch.int64)
        sync_all()

    def cold():
        rows = []
        for _ in range(args.steps):
            evict()
            rows.append(ctx.spmv_ex(ALPHA, BETA, delay_us=delay_us, wait=True))
        return np.array(rows)

    def warm():
        sync_all()
        t = time.perf_counter()
        for _ in range(args.steps):
            ctx.spmv_ex(ALPHA, BETA, wait=False)
        last = ctx.sync()
        sync_all()
        return time.perf_counter() - t, last

    if args.cache == "cold":
        st = cold()
        warm_el, warm_last = warm()
    else:
        warm_el, warm_last = warm()
        st = cold()
    # st[:, 0..2] = max over devices of kernel / exchange / step (ms); then
    # per device d: st[:, 3+3d .. 5+3d]
    step_ms = float(np.mean(st[:, 2]))
    kern_max = float(np.mean(st[:, 0]))
    xch_max = float(np.mean(st[:, 1]))
    dev_kern = [float(np.mean(st[:, 3 + 3 * d])) for d in range(N)]
    check = None
    if args.check:
        y0 = np.zeros(n)
        ctx.set_y(y0)
        ctx.spmv_ex(ALPHA, BETA)
        ys = [ctx.get_y(d) for d in range(N)]
        check = _oracle_check(rowptr, col, val, x_h, y0, ys)
    config3 = None
    if not args.no_config3:
        config3 = ctx_config3(ctx, args, sblas, n, rowptr, col, val, x_h, evict, delay_us,
                              profiled=N == 1 and W.default)
        if N > 1:  # beside the literal nnz split: the cost-weighted whole-row split
            config3["cost_weighted"] = cost_weighted(ctx_config3(ctx, args, sblas, n, rowptr, col, val, x_h, evict,
                                                                 delay_us, partition=2))
    config4 = config5 = structured = None
    if N == 1 and not args.ctx_loopback:  # one device: the same single-GPU legs as the torch driver
        import sblas_dist
        torch.cuda.set_device(0)
        if not args.no_config4:
            config4 = config4_leg(args, torch, sblas, sblas_dist, None, 0, 1, 0, evict, sync_all)
        if not args.no_config5:
            config5 = config5_leg(args, torch, sblas, 0, 1, evict, sync_all)
        if not args.no_structured:
            structured = structured_leg(args, torch, sblas, evict)
    del scrubs
    total_flops = 2.0 * nnz
    achieved0 = dev_bytes[0] / (dev_kern[0] * 1e-3) / 1e9
    agg = sum(dev_bytes) / (kern_max * 1e-3) / 1e9
    profiled = N == 1 and W.default
    out = {
        "metric": METRIC,
        "value": round(total_flops / (step_ms * 1e-3) / 1e9, 3),
        "unit": "GFLOP/s",
        "n_gpus": N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 5),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (deterministic generator, DESIGN.md)",
        "config": {
            "workload": W.describe(args.algo),
            "n": n, "nnz": nnz, "algo": args.algo, "matrix": args.matrix,
            "partition": ("cyclic row chunks" if partition == 0 else "nnz-balanced (spMV_mgpu_v1)"),
            "exchange": args.exchange if exchange == sblas.CTX_ALLREDUCE else "allgather",
            "driver": "ctx (one process, sblas_ctx over RCCL, ncclCommInitAll)",
            "overlap_parts": parts,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved0, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved0 / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic(args.algo) if profiled else None,
            "aggregate_GBps": round(agg, 1),
            "aggregate_frac": round(agg / (HBM_PEAK_GBS * N), 4),
        },
        "kernel_ms": round(dev_kern[0], 5),
        "kernel_ms_max_over_ranks": round(kern_max, 5),
        "kernel_ms_per_device": [round(k, 5) for k in dev_kern],
        "kernel_only_gflops": round(total_flops / (kern_max * 1e-3) / 1e9, 3),
        "algorithmic_bytes_per_launch": int(dev_bytes[0]),
        "algorithmic_bytes_all_ranks": int(sum(dev_bytes)),
        "nnz_per_device": [int(z) for _, z, _ in info],
        "algo_per_device": dev_algos,
        "host_gen_s": round(t_gen, 2),
        "plan": {"upload_and_build_s": round(plan_s, 3),
                 # the one-off plan in SpMV steps: calls before it is paid back
                 "equals_steps": int(round(plan_s / max(step_ms * 1e-3, 1e-12)))},
        "exchange_ms_max_over_ranks": round(xch_max, 5),
        "timing": ("cold steps: per-device span (start event .. end of exchange) after a device-side "
                   "hold and a one-word all-reduce that align the devices (sblas_ctx_spmv_ex), max "
                   "over devices" if args.cache == "cold"
                   else "warm: host wall clock over K back-to-back steps"),
        "cache": args.cache,
        "scrub": f"{args.scrub} {args.scrub_gib} GiB",
        ("warm" if args.cache == "cold" else "cold"): (
            {"value": round(total_flops / (warm_el / args.steps) / 1e9, 3),
             "ms_per_step": round(warm_el / args.steps * 1e3, 5),
             "last_step_kernel_ms_max": round(float(warm_last[0]), 5)}
            if args.cache == "cold" else
            {"value": round(total_flops / (step_ms * 1e-3) / 1e9, 3), "ms_per_step": round(step_ms, 5)}),
    }
    if args.cache == "warm":
        out["value"] = round(total_flops / (warm_el / args.steps) / 1e9, 3)
        out["ms_per_step"] = round(warm_el / args.steps * 1e3, 5)
    if check is not None:
        out["check_vs_oracle"] = check
    if config3 is not None:
        out["config3"] = config3
    if config4 is not None:
        out["config4"] = config4
    if config5 is not None:
        out["config5"] = config5
    if structured is not None:
        out["structured"] = structured
    out["traffic_source"] = dict(TRAFFIC_NOTES)
    if args.ctx_loopback:
        out["note"] = (f"loopback rehearsal: {N} context ranks on {ndev} GPU(s), collectives as "
                       "stream-ordered device copies (no RCCL); not a measurement")
    nranks, ords = ctx.comm_info()
    out["topology"] = topology_object(
        "ctx (one process, ncclCommInitAll)", "rccl" if nranks else "loopback (no communicator)", nranks, ords,
        [_pci_bus(torch, d) for d in ords], peer_matrix(torch),
        note=None if nranks else "loopback: ranks wrapped onto the visible GPUs, no RCCL communicator")
    if N == 1 and not args.no_cpu_baseline and not args.ctx_loopback:
        attach_cpu_baselines(out, args)
    print(json.dumps(out), flush=True)
    ctx.close()
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--algo", choices=["auto", "rowsplit", "csr5", "panel", "xsort"], default="auto",
                    help="auto (default): the library's per-slice choice (sblas_csr_pick): rowsplit "
                         "for coalescing columns, else xsort from 2M nonzeros, else panel")
    ap.add_argument("--nrows", type=int, default=2_000_000)
    ap.add_argument("--heavy", type=int, default=96)
    ap.add_argument("--light", type=int, default=9)
    ap.add_argument("--cols", choices=["random", "prefix"], default="random")
    ap.add_argument("--matrix", choices=["synth", "stencil7", "stencil27", "rmat"], default="synth",
                    help="synth (default): BASELINE configs[1]'s scaled generator; stencil7 / "
                         "stencil27: 3-D finite-difference / FEM-block pattern on a --grid^3 mesh; "
                         "rmat: power-law graph with 2^--scale vertices (SuiteSparse-class checks "
                         "of the north star's >= 60% target; not the headline)")
    ap.add_argument("--grid", type=int, default=160, help="stencil mesh edge (n = grid^3)")
    ap.add_argument("--scale", type=int, default=21, help="R-MAT scale (n = 2^scale)")
    ap.add_argument("--exchange", choices=["allgather", "allreduce"], default="allgather")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl (= RCCL over xGMI) for real runs; gloo only to rehearse the "
                         "multi-rank path with several ranks on one GPU")
    ap.add_argument("--check", action="store_true",
                    help="(default; kept for old command lines) after timing, verify the assembled y "
                         "of one fresh step against the oracle on rank 0 -> `check_vs_oracle`")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the post-timing oracle check of the headline y (on by default)")
    ap.add_argument("--cache", choices=["cold", "warm"], default="cold",
                    help="cold (default; SURVEY M1-cache / BASELINE.md: the headline uses cold "
                         "timing): a 1 GiB sweep (--scrub) before every timed step evicts the 256 MB "
                         "Infinity Cache and the L2s, each of the K steps bracketed by its own "
                         "barrier + synchronize; warm: K back-to-back steps bracketed by one "
                         "barrier + synchronize on each side.  The other mode is always measured "
                         "too and reported under `warm`/`cold`.")
    ap.add_argument("--partition", choices=["cyclic", "nnz"], default="cyclic",
                    help="N > 1 row distribution: cyclic equal-row chunks (default; no padding, "
                         "whole rows) or one nnz-balanced range per rank (spMV_mgpu_v1's split, "
                         "with split-row carries; always used with --exchange allreduce)")
    ap.add_argument("--scrub", choices=["read", "write"], default="read",
                    help="cold-cache eviction before each cold step: a 1 GiB read-only sweep "
                         "(default: leaves no dirty lines whose write-back the next step would "
                         "pay) or read+write (add_, round 1's method)")
    ap.add_argument("--scrub-gib", type=int, default=1,
                    help="size of the cold-cache sweep buffer in GiB (default 1: 4x the 256 MB Infinity Cache)")
    ap.add_argument("--no-rowsplit-beside", action="store_true",
                    help="skip the row-split kernel's figure reported beside the headline")
    ap.add_argument("--overlap", nargs="?", type=int, const=2, default=0, metavar="K",
                    help="N>1 cyclic allgather: cut each rank's chunks into K parts (default 2) "
                         "and all-gather part p while the kernel runs part p+1 (ctx driver: "
                         "sblas_ctx_matrix_upload_parts, any K; torch driver: two halves)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-peak", action="store_true", help="skip the measured HBM probe ceiling (N = 1)")
    ap.add_argument("--dist-always", action="store_true",
                    help="join a process group even at WORLD_SIZE 1 (torchrun --nproc-per-node 1): "
                         "runs the N > 1 exchange and timing path, RCCL included, on one GPU")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--ctx-loopback", action="store_true",
                    help="rehearsal only: the ctx driver with its N ranks wrapped onto the visible "
                         "GPUs and the collectives done as stream-ordered device copies instead of "
                         "RCCL (SBLAS_CTX_LOOPBACK=1); checks the N > 1 partition / exchange / "
                         "placement logic on a one-GPU box (use with --check)")
    ap.add_argument("--driver", choices=["auto", "ctx", "torch"], default="auto",
                    help="auto: torch.distributed ranks under a launcher, else one process over "
                         "sblas_ctx for --gpus > 1 (the persistent single-GPU path at N = 1); "
                         "ctx: force the C-ABI context (also at N = 1)")
    ap.add_argument("--no-config3", action="store_true",
                    help="skip the BASELINE configs[2] leg (CSR5, nnz split, all-reduce of y) that every "
                         "line carries under `config3`")
    ap.add_argument("--no-config4", action="store_true",
                    help="skip the BASELINE configs[3] leg (SpMM, rail4284-shaped x 64) every line carries")
    ap.add_argument("--no-config5", action="store_true",
                    help="skip the BASELINE configs[4] leg (sync-free SpTRSV, circuit5M-class) every line carries")
    ap.add_argument("--no-structured", action="store_true",
                    help="skip the SuiteSparse-class stand-ins leg (N = 1: stencil27, stencil7, rmat)")
    ap.add_argument("--no-check-legs", action="store_true",
                    help="skip the config4 / config5 post-timing checks (every C entry under the fp64 bound; "
                         "the SpTRSV known answer exactly)")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-leg", choices=["spmv", "spmm", "sptrsv"], default="spmv", help=argparse.SUPPRESS)
    args = ap.parse_args()
    args.check_legs = not args.no_check_legs
    args.check = not args.no_check
    if args.cpu_baseline_only:  # child of cpu_baseline(): host only, no torch, no GPU
        return cpu_baseline_child(args)

    import torch

    ndev = torch.cuda.device_count()  # does not initialise the GPU
    try:
        driver = choose_driver(args.gpus, os.environ, ndev, args.driver, args.ctx_loopback)
    except ValueError as e:
        print(f"bench.py: {e}", file=sys.stderr)
        return 2
    if driver == "ctx":
        return run_ctx(args)

    import sblas
    import sblas_dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev_idx = local_rank % max(ndev, 1)
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    dist = None
    if world > 1 or args.dist_always:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    # the communicator and devices this line runs on (rank 0 reports them)
    ordinals = _gather_rows(torch, dist, dev, [float(dev_idx)], world)[:, 0] if dist is not None else [dev_idx]
    topo = topology_object("torch (one process per GPU)", dist.get_backend() if dist is not None else "none",
                           dist.get_world_size() if dist is not None else 1, ordinals,
                           [_pci_bus(torch, int(d)) for d in ordinals], peer_matrix(torch))

    algo_ids = {"rowsplit": sblas.ROWSPLIT, "csr5": sblas.CSR5, "panel": sblas.PANEL,
                "xsort": sblas.XSORT}
    t_gen = time.perf_counter()
    W = Workload(args, sblas)
    n, rowptr, nnz = W.n, W.rowptr, W.nnz
    # auto: the library decides per rank slice (sblas_csr_pick: row split
    # where consecutive entries share x lines, else xsort from ~2M nonzeros,
    # else the XCD-panel row split; DESIGN.md §4 "Algorithm choice")
    algo = sblas.AUTO if args.algo == "auto" else algo_ids[args.algo]
    if args.partition == "cyclic" and args.exchange == "allgather":
        plan = sblas_dist.make_cyclic_plan(rowptr, n, world)
        lrp, col, val = sblas_dist.cyclic_local_csr(rowptr, plan, rank, W.rows)
        t_gen = time.perf_counter() - t_gen
        op = sblas_dist.DistSpMVCyclic(plan, rank, dev_idx, lrp, col, val, algo, torch, dist,
                                       overlap=args.overlap > 0)
        local_nnz = int(lrp[-1])
        partition = f"cyclic row chunks ({plan.chunk_rows} rows, {plan.nchunks} chunks)"
        if op.overlap:
            partition += ", two-half overlapped all-gather"
    else:
        plan = sblas_dist.make_plan(rowptr, n, world)
        r0, r1, i0, i1, _ = plan.local(rank)
        col_rows, val_rows = W.rows(r0, r1)
        off = i0 - int(rowptr[r0])
        col = np.ascontiguousarray(col_rows[off:off + (i1 - i0)])
        val = np.ascontiguousarray(val_rows[off:off + (i1 - i0)])
        t_gen = time.perf_counter() - t_gen
        op = sblas_dist.DistSpMV(plan, rank, dev_idx, rowptr, col, val, algo, torch, dist,
                                 args.exchange)
        local_nnz = i1 - i0
        partition = "nnz-balanced (spMV_mgpu_v1)"
    algo = op.algo  # resolved (AUTO: rank 0's slice decides the reported name)
    args.algo = {v: k for k, v in algo_ids.items()}[algo]
    x_h = sblas.gen_vector(n, 43)
    x = torch.from_numpy(x_h).to(dev)

    stream = torch.cuda.Stream(device=dev)
    sp = stream.cuda_stream
    local_bytes = op.A.algorithmic_bytes(BETA != 0.0)
    local_flops = 2.0 * local_nnz
    torch.cuda.synchronize()

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        op.kernel(ALPHA, x, BETA, sp)
        if ev is not None:
            ev[1].record(stream)
        op.exchange(sp)
        if ev is not None:
            ev[2].record(stream)  # after the collective and the device merge

    scrub = torch.zeros(args.scrub_gib << 30, dtype=torch.uint8, device=dev)

    def evict():
        if args.scrub == "write":
            scrub.add_(1)
        else:
            scrub.sum(dtype=torch.int64)

    def sync_barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def events():
        return [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3))
                for _ in range(args.steps)]

    def run_warm():
        # the contract's timed region: K back-to-back steps between barrier +
        # synchronize, host wall clock
        evs = events()
        sync_barrier()
        t0 = time.perf_counter()
        for k in range(args.steps):
            step(evs[k])
        sync_barrier()
        run_warm.xch = float(np.mean([b.elapsed_time(c) for _, b, c in evs]))
        return time.perf_counter() - t0, float(np.mean([a.elapsed_time(b) for a, b, _ in evs]))

    def run_cold():
        # every step starts from scrubbed caches, so the steps cannot run back
        # to back: each is timed on the device, HIP events on its stream from
        # before the kernel to after the exchange + merge (a rank that waits
        # in the collective for a slower one counts that wait); the host
        # barrier that separates scrub and step is not part of the step.
        # A short device-side spin queued ahead of the start event lets the
        # host enqueue the whole step before the stream reaches it, so the
        # events see device time, not the host's launch latency (with the
        # stream idle after the barrier, the start event would fire at once
        # and the kernel arrive ~10 us later: rocprofv3's kernel trace of the
        # same command reads ~12 us less than unpadded events did).
        # The host wall clock around each cold step is measured in a second,
        # spin-free pass and kept beside (wall_el).
        # At N = 1 the step is the SpMV call alone (no exchange): its device
        # span is read from events the runtime stamps at the call's first
        # kernel start and last kernel end (sblas_spmv_timed), which excludes
        # the remaining dispatch / event-record gaps of stream events
        # (~5 us on config 2; rocprofv3's kernel trace agrees with the span).
        evs = events()
        span_ms = []
        for k in range(args.steps):
            evict()  # 1 GiB sweep: evicts MALL (256 MB) and L2
            sync_barrier()
            if dist is None and op.dm > 0:
                span_ms.append(op.A.spmv_timed(op.algo, ALPHA, x.data_ptr(), BETA, op.y_local.data_ptr(), sp))
            else:
                torch.cuda._sleep(500_000)
                step(evs[k])
            sync_barrier()
        if span_ms:
            run_cold.wall_el = 0.0
            run_cold.xch = 0.0
            wall_el = 0.0
            for k in range(args.steps):
                evict()
                sync_barrier()
                t0 = time.perf_counter()
                step()
                sync_barrier()
                wall_el += time.perf_counter() - t0
            run_cold.wall_el = wall_el
            return float(np.sum(span_ms)) * 1e-3, float(np.mean(span_ms))
        wall_el = 0.0
        for k in range(args.steps):
            evict()
            sync_barrier()
            t0 = time.perf_counter()
            step()
            sync_barrier()
            wall_el += time.perf_counter() - t0
        run_cold.wall_el = wall_el
        run_cold.xch = float(np.mean([b.elapsed_time(c) for _, b, c in evs]))
        el = float(np.sum([a.elapsed_time(c) for a, _, c in evs])) * 1e-3
        return el, float(np.mean([a.elapsed_time(b) for a, b, _ in evs]))
    run_cold.wall_el = 0.0
    run_cold.xch = run_warm.xch = 0.0

    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if args.cache == "cold":
            el, kern_ms = run_cold()
            el_o, kern_o = run_warm()
        else:
            el, kern_ms = run_warm()
            el_o, kern_o = run_cold()
    xch_ms = run_cold.xch if args.cache == "cold" else run_warm.xch
    rowsplit_beside = None
    if world == 1 and algo != sblas.ROWSPLIT and not args.no_rowsplit_beside:
        # configs[1] names the row-split kernel: its figure on the same
        # matrix, same cold protocol, kernel events only
        op.A.analyse(sblas.ROWSPLIT)
        with torch.cuda.stream(stream):
            for _ in range(2):
                op.A.spmv(sblas.ROWSPLIT, ALPHA, x.data_ptr(), BETA, op.y_local.data_ptr(), sp)
            rs = []
            for _ in range(args.steps):
                evict()
                torch.cuda.synchronize()
                rs.append(op.A.spmv_timed(sblas.ROWSPLIT, ALPHA, x.data_ptr(), BETA, op.y_local.data_ptr(), sp))
            torch.cuda.synchronize()
        rk = float(np.mean(rs))
        rowsplit_beside = {"kernel_ms": round(rk, 5),
                           "gflops": round(2.0 * nnz / (rk * 1e-3) / 1e9, 3),
                           "roofline_frac": round(local_bytes / (rk * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                           "cache": "cold",
                           # the row blocks' layout: 0 = plain, P = per XCD column panel
                           "xcd_panels": op.A.panels(sblas.ROWSPLIT)}
    deterministic_beside = None
    if world == 1 and not args.no_rowsplit_beside:
        deterministic_beside = deterministic_leg(args, torch, sblas, op, algo, x, local_bytes, nnz, stream, evict)
    config3 = None
    if not args.no_config3:
        config3 = torch_config3(args, W, sblas, sblas_dist, torch, dist, rank, world, dev_idx, x, x_h, stream,
                                evict, sync_barrier)
        if world > 1:  # beside the literal nnz split: the cost-weighted whole-row split
            config3["cost_weighted"] = cost_weighted(torch_config3(
                args, W, sblas, sblas_dist, torch, dist, rank, world, dev_idx, x, x_h, stream, evict, sync_barrier,
                row_cost=ROW_COST))
    config4 = config5 = None
    if not args.no_config4:
        config4 = config4_leg(args, torch, sblas, sblas_dist, dist, rank, world, dev_idx, evict, sync_barrier)
        if world > 1:  # beside the literal row split: row blocks x column groups
            config4["grid"] = config4_leg(args, torch, sblas, sblas_dist, dist, rank, world, dev_idx, evict,
                                          sync_barrier, split="grid")
    if not args.no_config5:
        config5 = config5_leg(args, torch, sblas, rank, world, evict, sync_barrier)
    structured = None
    if world == 1 and not args.no_structured:
        structured = structured_leg(args, torch, sblas, evict)
    del scrub
    peak = measured_peak(torch, sblas, dev, stream) if world == 1 and not args.no_peak else None

    check = None
    if args.check:
        # one fresh step from y0 = 0, then compare the assembled y (every rank
        # holds it) with the oracle on rank 0 -- verification only
        with torch.cuda.stream(stream):
            op.load_y(torch.zeros(plan.m, dtype=torch.float64, device=dev))
            step()
        torch.cuda.synchronize()
        y_dev = op.result().cpu().numpy()
        if rank == 0:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import orc  # oracle: checker only
            col_all, val_all = W.rows(0, n)
            want = orc.csr_spmv(rowptr, col_all, val_all, x_h, ALPHA, BETA, np.zeros(plan.m))
            bound = orc.spmv_bound(rowptr, col_all, val_all, x_h, ALPHA, BETA, np.zeros(plan.m))
            check = bool(np.all(np.abs(y_dev - want) <= bound))
    stats_dev = dev if (dist is None or args.dist_backend == "nccl") else torch.device("cpu")
    stats = torch.tensor([el, kern_ms, local_bytes, local_flops, el_o, kern_o, run_cold.wall_el, xch_ms,
                          getattr(op, "plan_s", 0.0)],
                         dtype=torch.float64,
                         device=stats_dev)
    if dist is not None:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        el, kern_ms_max = float(mx[0]), float(mx[1])
        el_o, kern_o_max = float(mx[4]), float(mx[5])
        cold_wall = float(mx[6])
        xch_max, plan_s_max = float(mx[7]), float(mx[8])
        tot_bytes = float(sm[2])
    else:
        kern_ms_max, tot_bytes, kern_o_max = kern_ms, float(local_bytes), kern_o
        cold_wall = run_cold.wall_el
        xch_max, plan_s_max = xch_ms, getattr(op, "plan_s", 0.0)
    ms_step = el / args.steps * 1e3
    total_flops = 2.0 * nnz

    if rank == 0:
        achieved = local_bytes / (kern_ms * 1e-3) / 1e9  # rank 0's kernel
        # the committed PMC summary was collected on the default workload only
        profiled = world == 1 and W.default
        traffic = pmc_traffic(args.algo) if profiled else None
        out = {
            "metric": METRIC,
            "value": round(total_flops / (ms_step * 1e-3) / 1e9, 3),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 5),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (deterministic generator, DESIGN.md)",
            "config": {
                "workload": W.describe(args.algo),
                "n": n, "nnz": nnz, "algo": args.algo, "matrix": args.matrix,
                "partition": partition if world > 1 else "single GPU",
                "exchange": args.exchange if world > 1 else "none",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
            },
            **({"measured_peak": dict(peak, frac_of_read_peak=round(achieved / peak["read_GBps"], 4))}
               if peak else {}),
            "kernel_ms": round(kern_ms, 5),
            "kernel_ms_max_over_ranks": round(kern_ms_max, 5),
            "kernel_only_gflops": round(total_flops / (kern_ms_max * 1e-3) / 1e9, 3),
            "algorithmic_bytes_per_launch": int(local_bytes),
            "algorithmic_bytes_all_ranks": int(tot_bytes),
            "host_gen_s": round(t_gen, 2),
            "plan": {"build_s_max_over_ranks": round(plan_s_max, 3),
                     # the one-off plan in SpMV steps (excluded from the timed region)
                     "equals_steps": int(round(plan_s_max / max(ms_step * 1e-3, 1e-12))),
                     "device_bytes_rank0": int(op.A.plan_bytes(algo)),
                     "csr_device_bytes_rank0": int(12 * local_nnz + 4 * (op.A.info()[0] + 1))},
            "exchange_ms_max_over_ranks": round(xch_max, 5),
            "timing": (("cold steps: device span of the SpMV call (events stamped by the runtime at "
                        "its first kernel's start and last kernel's end, sblas_spmv_timed); host wall "
                        "clock beside" if world == 1 else
                        "cold steps: device time, HIP events on the launch stream from before the "
                        "kernel to after exchange + merge, max over ranks; host wall clock beside")
                       if args.cache == "cold" else "warm: host wall clock over K back-to-back steps"),
            "cache": args.cache,
            "scrub": f"{args.scrub} {args.scrub_gib} GiB",
            # cold steps are timed on the device (run_cold); the host wall
            # clock around each, barrier round trips included, for comparison
            "cold_host_wall_ms_per_step": round(cold_wall / args.steps * 1e3, 5),
            ("warm" if args.cache == "cold" else "cold"): {
                "value": round(total_flops / (el_o / args.steps) / 1e9, 3),
                "ms_per_step": round(el_o / args.steps * 1e3, 5),
                "kernel_ms": round(kern_o, 5),
                "kernel_ms_max_over_ranks": round(kern_o_max, 5),
                "roofline_frac": round(local_bytes / (kern_o * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            },
        }
        if world > 1 and args.dist_backend != "nccl":
            out["note"] = f"rehearsal: {world} ranks on {ndev} GPU(s) over {args.dist_backend}"
        out["topology"] = topo
        if check is not None:
            out["check_vs_oracle"] = check
        if rowsplit_beside is not None:
            out["rowsplit_beside"] = rowsplit_beside
        if deterministic_beside is not None:
            out["deterministic_beside"] = deterministic_beside
        if config3 is not None:
            out["config3"] = config3
        if config4 is not None:
            out["config4"] = config4
        if config5 is not None:
            out["config5"] = config5
        if structured is not None:
            out["structured"] = structured
        out["traffic_source"] = dict(TRAFFIC_NOTES)
        if world == 1 and not args.no_cpu_baseline:
            attach_cpu_baselines(out, args)
        print(json.dumps(out), flush=True)
    op.close()
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
