#!/usr/bin/env python3
"""Matrix-Market loader benchmark, host only.

Writes a synthetic general real .mtx of --nnz entries (uniform rows/cols,
17-digit values), then times, each in a fresh process so OMP_NUM_THREADS
takes effect:
  * the reference's own loader, mmio_info + mmio_data
    (sptrsv_v1/src/mmio_highlevel.h, compiled in place into oracle/_ref) when
    it is present -- the CPU baseline;
  * sblas_mm_read mode 0 with 1 thread and with --threads threads (one parse
    for the size + data calls);
  * a load served from the .csrbin cache (SBLAS_MM_CACHE).
Prints one JSON line.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

CHILD = r"""
import sys, time, os
sys.path.insert(0, os.path.join(sys.argv[1], "s-blas_amd"))
kind, path = sys.argv[2], sys.argv[3]
if kind == "ref":
    import ctypes as C, numpy as np
    lib = C.CDLL(os.path.join(sys.argv[1], "oracle", "_ref", "libsblas_ref.so"))
    t0 = time.perf_counter()
    m, n, nnz, sym = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    assert lib.ref_mmio_info(path.encode(), C.byref(m), C.byref(n), C.byref(nnz), C.byref(sym)) == 0
    rp = np.zeros(m.value + 1, np.int32); col = np.zeros(nnz.value, np.int32); val = np.zeros(nnz.value)
    assert lib.ref_mmio_data(path.encode(), rp.ctypes.data_as(C.c_void_p), col.ctypes.data_as(C.c_void_p),
                             val.ctypes.data_as(C.c_void_p)) == 0
    print(time.perf_counter() - t0, int(rp[-1]))
else:
    import sblas
    t0 = time.perf_counter()
    m, n, rp, col, val = sblas.mm_read(path, 0)
    print(time.perf_counter() - t0, int(rp[-1]))
"""


def child(kind, path, threads, cache=None):
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    env.pop("SBLAS_MM_CACHE", None)
    if cache:
        env["SBLAS_MM_CACHE"] = cache
    out = subprocess.run([sys.executable, "-c", CHILD, ROOT, kind, path], env=env, check=True,
                         capture_output=True, text=True).stdout.split()
    return float(out[0]), int(out[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nnz", type=int, default=10_000_000)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    ap.add_argument("--dir", default=None)
    args = ap.parse_args()
    d = args.dir or tempfile.mkdtemp(prefix="sblas_loader_")
    path = os.path.join(d, "synthetic.mtx")
    rng = np.random.default_rng(7)
    t0 = time.perf_counter()
    with open(path, "w") as fh:
        fh.write("%%MatrixMarket matrix coordinate real general\n")
        fh.write(f"{args.n} {args.n} {args.nnz}\n")
        step = 1_000_000
        for s in range(0, args.nnz, step):
            k = min(step, args.nnz - s)
            r = rng.integers(1, args.n + 1, k)
            c = rng.integers(1, args.n + 1, k)
            v = rng.standard_normal(k)
            fh.write("\n".join(f"{a} {b} {x:.17g}" for a, b, x in zip(r.tolist(), c.tolist(),
                                                                     v.tolist())))
            fh.write("\n")
    t_write = time.perf_counter() - t0
    size = os.path.getsize(path)
    res = {}
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libsblas_ref.so")
    if os.path.exists(ref_so):
        res["reference_mmio_data_1thread_s"], nnz_ref = child("ref", path, 1)
    res["sblas_1thread_s"], nnz1 = child("sblas", path, 1)
    res[f"sblas_{args.threads}threads_s"], nnzt = child("sblas", path, args.threads)
    cache = os.path.join(d, "cache")
    os.makedirs(cache, exist_ok=True)
    res["sblas_cache_fill_s"], _ = child("sblas", path, args.threads, cache)
    res["sblas_cache_hit_s"], nnzc = child("sblas", path, args.threads, cache)
    assert nnz1 == nnzt == nnzc == args.nnz
    out = {"metric": "Matrix-Market load time (mode 0, general real)", "unit": "s",
           "file_mb": round(size / 1e6, 1), "nnz": args.nnz, "threads": args.threads,
           "host_cpus": os.cpu_count(), "write_s": round(t_write, 1),
           **{k: round(v, 3) for k, v in res.items()}}
    print(json.dumps(out), flush=True)
    if not args.dir:
        for f in os.listdir(cache):
            os.remove(os.path.join(cache, f))
        os.rmdir(cache)
        os.remove(path)
        os.rmdir(d)


if __name__ == "__main__":
    main()
