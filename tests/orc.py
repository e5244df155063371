"""ctypes view of oracle/liboracle.so (the CPU restatement) and, when built,
oracle/_ref/libsblas_ref.so (the reference's own host code compiled in place).

TEST INFRASTRUCTURE ONLY -- the checker, never the thing measured or shipped.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "liboracle.so")
REF = os.path.join(ORACLE_DIR, "_ref", "libsblas_ref.so")

if not os.path.exists(LIB):
    subprocess.run(["make", "-C", ORACLE_DIR, "liboracle.so"], check=True,
                   stdout=subprocess.DEVNULL)
lib = C.CDLL(LIB)
ref = C.CDLL(REF) if os.path.exists(REF) else None

_p, _i, _ll, _d = C.c_void_p, C.c_int, C.c_longlong, C.c_double


def _sig(L, name, res, *args):
    f = getattr(L, name)
    f.restype = res
    f.argtypes = list(args)


_sig(lib, "orc_ref_alpha_beta", None, _ll, _p, _p)
_sig(lib, "orc_mm_info", _i, C.c_char_p, _p, _p, _p, _p)
_sig(lib, "orc_mm_load_testspmv", _i, C.c_char_p, C.c_char, _p, _p, _p)
_sig(lib, "orc_mm_load_mmio", _i, C.c_char_p, _p, _p, _p, _p, _p, _p, _p)
_sig(lib, "orc_csr_spmv", None, _i, _p, _p, _p, _p, _d, _d, _p)
_sig(lib, "orc_csr_spmv_omp", None, _i, _p, _p, _p, _p, _d, _d, _p, _i)
_sig(lib, "orc_get_row_from_index_ref", _i, _i, _p, _ll)
_sig(lib, "orc_row_of_index", _i, _i, _p, _ll)
_sig(lib, "orc_partition_rowblock", None, _i, _i, _p)
_sig(lib, "orc_partition_nnz", None, _i, _ll, _p, _i, _p, _p, _p, _p, _p)
_sig(lib, "orc_spmv_mgpu_v1", None, _i, _i, _ll, _d, _p, _p, _p, _p, _d, _p, _i)
_sig(lib, "orc_spmv_mgpu_baseline", None, _i, _i, _ll, _d, _p, _p, _p, _p, _d, _p, _i)
_sig(lib, "orc_gen_ref_nnz", _ll, _i)
_sig(lib, "orc_gen_ref", None, _i, _p, _p, _p)
_sig(lib, "orc_gen_synth_rowptr", None, _i, _i, _i, _p)
_sig(lib, "orc_gen_synth", None, _i, _i, _i, _i, C.c_ulonglong, _p, _p, _p)
_sig(lib, "orc_gen_vector", None, _i, C.c_ulonglong, _p)
_sig(lib, "orc_transpose", None, _i, _i, _i, _p, _p, _p, _p, _p, _p)
_sig(lib, "orc_build_tri", _i, _i, _p, _p, _i, C.c_uint, _p, _p, _p)
_sig(lib, "orc_tri_rhs", None, _i, _p, _p, _p, _p, _p)
_sig(lib, "orc_sptrsv_serial", _i, _p, _p, _p, _i, _i, _i, _p, _p)
_sig(lib, "orc_levels_lower", _i, _i, _p, _p, _p)
_sig(lib, "orc_spmm", None, _i, _i, _i, _d, _p, _p, _p, _p, _i, _d, _p, _i)
_sig(lib, "orc_coo_sort_to_csr", None, _i, _i, _p, _p, _p, _p)
_sig(lib, "orc_spmv_bound", None, _i, _p, _p, _p, _p, _d, _d, _p, _p)
_sig(lib, "orc_spmm_omp", None, _i, _i, _d, _p, _p, _p, _p, _i, _i, _d, _p, _i, _p, _i)
if ref is not None:
    _sig(ref, "ref_mm_header", _i, C.c_char_p, _p, _p, _p, _p)
    _sig(ref, "ref_mmio_info", _i, C.c_char_p, _p, _p, _p, _p)
    _sig(ref, "ref_mmio_data", _i, C.c_char_p, _p, _p, _p)
    _sig(ref, "ref_sptrsv_serial", _i, _p, _p, _p, _i, _i, _i, _i, _p, _p)


def P(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def alpha_beta(skip=0):
    a, b = C.c_double(), C.c_double()
    lib.orc_ref_alpha_beta(skip, C.byref(a), C.byref(b))
    return a.value, b.value


def mm_info(path):
    m, n, nz, fl = C.c_int(), C.c_int(), C.c_longlong(), C.c_int()
    assert lib.orc_mm_info(path.encode(), C.byref(m), C.byref(n), C.byref(nz), C.byref(fl)) == 0
    return m.value, n.value, nz.value, fl.value


def load_testspmv(path, data_type="f"):
    m, n, nz, _ = mm_info(path)
    rp = np.zeros(m + 1, np.int64)
    col = np.zeros(max(nz, 1), np.int32)
    val = np.zeros(max(nz, 1), np.float64)
    assert lib.orc_mm_load_testspmv(path.encode(), data_type.encode(), P(rp), P(col), P(val)) == 0
    return m, n, rp, col[:nz], val[:nz]


def load_mmio(path):
    m, n, nnz, sym = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    args = (C.byref(m), C.byref(n), C.byref(nnz), C.byref(sym))
    assert lib.orc_mm_load_mmio(path.encode(), *args, None, None, None) == 0
    rp = np.zeros(m.value + 1, np.int32)
    col = np.zeros(max(nnz.value, 1), np.int32)
    val = np.zeros(max(nnz.value, 1), np.float64)
    assert lib.orc_mm_load_mmio(path.encode(), *args, P(rp), P(col), P(val)) == 0
    return m.value, n.value, rp, col[:nnz.value], val[:nnz.value], sym.value


def csr_spmv(rowptr, col, val, x, alpha, beta, y):
    rp = np.ascontiguousarray(rowptr, np.int64)
    out = np.array(y, np.float64, copy=True)
    lib.orc_csr_spmv(len(rp) - 1, P(rp), P(col), P(val), P(x), alpha, beta, P(out))
    return out


def csr_spmv_omp(rowptr, col, val, x, alpha, beta, y, nthreads=0):
    rp = np.ascontiguousarray(rowptr, np.int64)
    lib.orc_csr_spmv_omp(len(rp) - 1, P(rp), P(col), P(val), P(x), alpha, beta, P(y), nthreads)
    return y


def spmv_bound(rowptr, col, val, x, alpha, beta, y0):
    """Per-row fp64 bound of DESIGN.md: 4*gamma_k*sum|alpha*a*x| + 4u|beta*y0|
    (orc_spmv_bound, OpenMP over rows)."""
    rp = np.ascontiguousarray(rowptr, np.int64)
    m = len(rp) - 1
    out = np.zeros(m)
    lib.orc_spmv_bound(m, P(rp), P(np.ascontiguousarray(col, np.int32)),
                       P(np.ascontiguousarray(val, np.float64)),
                       P(np.ascontiguousarray(x, np.float64)), alpha, beta,
                       P(np.ascontiguousarray(y0, np.float64)), P(out))
    return out


def partition_nnz(rowptr, g):
    rp = np.ascontiguousarray(rowptr, np.int64)
    si = np.zeros(g, np.int64); ei = np.zeros(g, np.int64)
    sr = np.zeros(g, np.int32); er = np.zeros(g, np.int32); sf = np.zeros(g, np.int32)
    lib.orc_partition_nnz(len(rp) - 1, int(rp[-1]), P(rp), g, P(si), P(ei), P(sr), P(er), P(sf))
    return si, ei, sr, er, sf


def spmv_mgpu(version, m, n, rowptr, col, val, x, alpha, beta, y, g):
    rp = np.ascontiguousarray(rowptr, np.int64)
    out = np.array(y, np.float64, copy=True)
    f = lib.orc_spmv_mgpu_v1 if version == "v1" else lib.orc_spmv_mgpu_baseline
    f(m, n, int(rp[-1]), alpha, P(val), P(rp), P(col), P(x), beta, P(out), g)
    return out


def gen_synth(n, heavy=96, light=9, prefix=False, seed=42):
    rp = np.zeros(n + 1, np.int64)
    lib.orc_gen_synth_rowptr(n, heavy, light, P(rp))
    nnz = int(rp[-1])
    col = np.zeros(max(nnz, 1), np.int32)
    val = np.zeros(max(nnz, 1), np.float64)
    lib.orc_gen_synth(n, heavy, light, int(prefix), seed, P(rp), P(col), P(val))
    return rp, col[:nnz], val[:nnz]


def gen_vector(n, seed):
    v = np.zeros(max(n, 1))
    lib.orc_gen_vector(n, seed, P(v))
    return v[:n]


def gen_ref(n):
    nnz = lib.orc_gen_ref_nnz(n)
    r = np.zeros(nnz, np.int32); c = np.zeros(nnz, np.int32); v = np.zeros(nnz)
    lib.orc_gen_ref(n, P(r), P(c), P(v))
    return r, c, v


def transpose(m, n, rowptr, col, val):
    rp = np.ascontiguousarray(rowptr, np.int32)
    nnz = int(rp[-1])
    cp = np.zeros(n + 1, np.int32); ri = np.zeros(max(nnz, 1), np.int32); cv = np.zeros(max(nnz, 1))
    lib.orc_transpose(m, n, nnz, P(rp), P(np.ascontiguousarray(col, np.int32)),
                      P(np.ascontiguousarray(val, np.float64)), P(cp), P(ri), P(cv))
    return cp, ri[:nnz], cv[:nnz]


def build_tri(rowptr, col, substitution, seed):
    """L (or U) CSR with unit diagonal from A's pattern + CSC + x_ref + b
    (sptrsv_v1/src/main.cu:150-355 with a fixed seed)."""
    rp = np.ascontiguousarray(rowptr, np.int32)
    ci = np.ascontiguousarray(col, np.int32)
    m = len(rp) - 1
    nnz = lib.orc_build_tri(m, P(rp), P(ci), substitution, seed, None, None, None)
    trp = np.zeros(m + 1, np.int32); tc = np.zeros(nnz, np.int32); tv = np.zeros(nnz)
    lib.orc_build_tri(m, P(rp), P(ci), substitution, seed, P(trp), P(tc), P(tv))
    cp, ri, cv = transpose(m, m, trp, tc, tv)
    xref = np.zeros(m); b = np.zeros(m)
    lib.orc_tri_rhs(m, P(cp), P(ri), P(cv), P(xref), P(b))
    return (trp, tc, tv), (cp, ri, cv), xref, b


def sptrsv_serial(cp, ri, cv, b, substitution=0):
    n = len(cp) - 1
    x = np.zeros(n)
    lib.orc_sptrsv_serial(P(cp), P(ri), P(cv), n, substitution, 1, P(b), P(x))
    return x


def levels_lower(cp, ri):
    n = len(cp) - 1
    lev = np.zeros(n, np.int32)
    return lib.orc_levels_lower(n, P(cp), P(ri), P(lev))


def spmm(m, n, k, alpha, rowptr, col, val, B, beta, C):
    out = np.array(C, np.float64, copy=True, order="F")
    rp = np.ascontiguousarray(rowptr, np.int32)
    Bf = np.asfortranarray(B, np.float64)
    lib.orc_spmm(m, n, k, alpha, P(rp), P(np.ascontiguousarray(col, np.int32)),
                 P(np.ascontiguousarray(val, np.float64)), P(Bf), k, beta, P(out), m)
    return out


def spmm_checked(m, n, alpha, rowptr, col, val, B, beta, C, b_rowmajor=True, nthreads=0):
    """orc_spmm's arithmetic in OpenMP (orc_spmm_omp) plus the per-entry bound.
    B: (k, n) array; C: (m, n) array.  Returns (C_out, bound) as (m, n)."""
    rp = np.ascontiguousarray(rowptr, np.int32)
    if b_rowmajor:
        Bc = np.ascontiguousarray(B, np.float64)
        ldb = n
    else:
        Bc = np.asfortranarray(B, np.float64)
        ldb = B.shape[0]
    out = np.array(C, np.float64, copy=True, order="F")
    bound = np.zeros((m, n), np.float64, order="F")
    lib.orc_spmm_omp(m, n, alpha, P(rp), P(np.ascontiguousarray(col, np.int32)),
                     P(np.ascontiguousarray(val, np.float64)), P(Bc), ldb, int(b_rowmajor), beta,
                     P(out), m, P(bound), nthreads)
    return out, bound
