"""sblas -- Python view of libsblas.so (the MI355X-native sparse-BLAS hot path).

Thin ctypes binding of include/sblas.h.  This is the host-side mirror the
tests and bench.py drive; all compute happens in libsblas.so's HIP kernels.
Importing fails loudly when the library has not been built -- there is no
CPU fallback anywhere on the product path.

Device arrays are passed as raw pointers: torch tensors (``t.data_ptr()``)
serve as device memory and ``torch.cuda.Stream.cuda_stream`` as the stream
handle, so torch is only plumbing (allocation, streams, torch.distributed).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SBLAS_LIB: an alternative build of the same library (A/B timing of two
# builds on one box); the default is the in-tree build
LIB_PATH = os.environ.get("SBLAS_LIB") or os.path.join(_HERE, "libsblas.so")

AUTO = 0      # chosen per handle (sblas_csr_pick: column-locality probe)
ROWSPLIT = 1  # test_spmv kernel 1 (csrmv)
CSR5 = 2      # test_spmv kernel 2/3 (csrmv_mp / CSR5)
PANEL = 4     # XCD-affine column panels (row-split per panel + reduce)
XSORT = 5     # column-sorted XCD groups (LDS row accumulators)

_STATUS = {0: "ok", 1: "invalid argument", 2: "HIP runtime error",
           3: "insufficient device memory", 4: "no device", 5: "unsupported",
           6: "RCCL error", 7: "I/O error", -1: "footprint > 0.8 x free memory"}


class SblasError(RuntimeError):
    pass


def _load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise SblasError(
            f"{LIB_PATH} missing: build it with `make -C s-blas_amd` "
            "(or __graft_entry__.build()); there is no fallback path")
    return C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)


lib = _load()

_p = C.c_void_p
_i = C.c_int
_ll = C.c_longlong
_d = C.c_double


def _sig(name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_sig("sblas_status_string", C.c_char_p, _i)
_sig("sblas_last_error", C.c_char_p)
_sig("sblas_version", _i)
_sig("sblas_device_count", _i, _p)
_sig("sblas_spMV_mgpu_baseline", _i, _i, _i, _ll, _p, _p, _p, _p, _p, _p, _p, _i)
_sig("sblas_spMV_mgpu_v1", _i, _i, _i, _ll, _p, _p, _p, _p, _p, _p, _p, _i, _i)
_sig("sblas_spMV_mgpu_v2", _i, _i, _i, _ll, _p, _p, _p, _p, _p, _p, _p, _i, _i, _ll, _i)
_sig("sblas_get_row_from_index", _i, _i, _p, _ll)
_sig("sblas_get_time", _d)
_sig("sblas_get_gpu_availble_mem", _d, _i)
_sig("sblas_csrmm_mgpu", _i, _i, _i, _i, _p, _i, _p, _p, _p, _p, _p, _p, _i)
_sig("sblas_csrmm_mgpu_colsplit", _i, _i, _i, _i, _p, _i, _p, _p, _p, _p, _p, _p, _i)
_sig("sblas_sptrsv_syncfree", _i, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _i)
_sig("sblas_csr_upload_slice", _i, _p, _i, _i, _p, _p, _p, _i, _i, _ll, _ll, _p)
_sig("sblas_csr_from_device", _i, _p, _i, _i, _i, _i, _p, _p, _p, _p)
_sig("sblas_csr_destroy", _i, _p)
_sig("sblas_csr_info", _i, _p, _p, _p, _p)
_sig("sblas_csr_analyse", _i, _p, _i, _p)
_sig("sblas_spmv", _i, _p, _i, _d, _p, _d, _p, _p)
_sig("sblas_spmv_timed", _i, _p, _i, C.c_double, _p, C.c_double, _p, _p, _p)
_sig("sblas_spmv_algorithmic_bytes", _ll, _p, _i)
_sig("sblas_hbm_probe", _i, _i, _p, _p, _ll, _i, _p)
_sig("sblas_hbm_probe_timed", _i, _i, _p, _p, _ll, _i, _p, _p)
_sig("sblas_csr_plan_bytes", _ll, _p, _i)
_sig("sblas_csr_pick", _i, _p, _p, _p)
_sig("sblas_spmm", _i, _p, _i, _d, _p, _i, _i, _d, _p, _i, _p)
_sig("sblas_csr_transpose", _i, _p, _p, _p, _p, _p)
_sig("sblas_trsv_create", _i, _p, _i, _i, _i, _p, _p, _p, _i, _p)
_sig("sblas_trsv_solve", _i, _p, _i, _p, _p, _p)
_sig("sblas_trsv_pick", _i, _p, _p, _p)
_sig("sblas_trsv_levels", _i, _p, _p)
_sig("sblas_trsv_destroy", _i, _p)
_sig("sblas_trsv_mgpu_solve", _i, _p, _p, _p, _i, _i, _i, _p, _p, _i, _p)
_sig("sblas_trsv_solve_rhs", _i, _p, _i, _p, _p, _p)
_sig("sblas_trsv_solve_rhs_opt", _i, _p, _i, _i, _i, _p, _p, _p)
_sig("sblas_trsv_mgpu_solve_tasks", _i, _p, _p, _p, _i, _i, _i, _p, _p, _i, _i, _i, _p)
_sig("sblas_sptrsv_syncfree_v3", _i, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _i, _i)
_sig("sblas_spmv_ooc", _i, _i, _i, _ll, _d, _p, _p, _p, _p, _d, _p, _i, _ll, _i, _p)
_sig("sblas_csr2csc_mgpu", _i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p)
_sig("sblas_sptrans", _i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p)
_sig("sblas_assemble_slices", _i, _p, _i, _ll, _p, _p, _i, _p, _p)
_sig("sblas_assemble_cyclic", _i, _p, _i, _ll, _ll, _ll, _p, _p)
_sig("sblas_mm_read", _i, C.c_char_p, _i, _p, _p, _p, _p, _p, _p)
_sig("sblas_csrbin_write", _i, C.c_char_p, _i, _i, _ll, _p, _p, _p)
_sig("sblas_csrbin_read", _i, C.c_char_p, _p, _p, _p, _p, _p, _p)
_sig("sblas_partition_nnz", _i, _i, _ll, _p, _i, _p, _p, _p, _p, _p)
_sig("sblas_partition_cost", _i, _i, _p, _i, C.c_double, _p, _p, _p, _p, _p)
_sig("sblas_partition_rowblock", _i, _i, _i, _p)
_sig("sblas_coo_sortbyrow", _i, _i, _ll, _p, _p, _p, _p)
_sig("sblas_trsv_mgpu_create", _i, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i)
_sig("sblas_trsv_mgpu_run", _i, _p, _p, _p, _p)
_sig("sblas_trsv_mgpu_destroy", _i, _p)
_sig("sblas_trsv_mgpu_info", _i, _p, _p, _p, _p)
_sig("sblas_ctx_comm_info", _i, _p, _p, _p)
_sig("sblas_test_deny_peer_access", _i, _i)
_sig("sblas_peer_refs", _i, _i, _i)
_sig("sblas_test_set_option", _i, C.c_char_p, _d, _i)
_sig("sblas_csr_set_deterministic", _i, _p, _i)
_sig("sblas_csr_xsort_info", _i, _p, _p)
_sig("sblas_csr_get_deterministic", _i, _p, _p)
_sig("sblas_ctx_create", _i, _p, _i, _p)
_sig("sblas_ctx_destroy", _i, _p)
_sig("sblas_ctx_ngpu", _i, _p, _p)
_sig("sblas_ctx_matrix_upload", _i, _p, _i, _i, _p, _p, _p, _i, _i)
_sig("sblas_ctx_set_x", _i, _p, _p)
_sig("sblas_ctx_set_y", _i, _p, _p)
_sig("sblas_ctx_spmv", _i, _p, _d, _d, _p)
_sig("sblas_ctx_matrix_upload_ex", _i, _p, _i, _i, _p, _p, _p, _i, _i, _i)
_sig("sblas_ctx_slice_info", _i, _p, _i, _p, _p, _p)
_sig("sblas_ctx_slice_algo", _i, _p, _i, _p)
_sig("sblas_ctx_matrix_upload_parts", _i, _p, _i, _i, _p, _p, _p, _i, _i)
_sig("sblas_ctx_parts", _i, _p, _p)
_sig("sblas_csr_panels", _i, _p, _i, _p)
_sig("sblas_ctx_spmv_ex", _i, _p, _d, _d, _d, _i, _p)
_sig("sblas_ctx_sync", _i, _p, _p)
_sig("sblas_ctx_get_y", _i, _p, _i, _p)
_sig("sblas_ctx_bind", _i, _p)
_sig("sblas_cyclic_plan", _i, _ll, _i, _i, _p, _p)
_sig("sblas_cyclic_local_csr", _i, _i, _p, _p, _p, _i, _ll, _i, _p, _p, _p, _p, _p)
_sig("sblas_gen_synth_rowptr", _i, _i, _i, _i, _p)
_sig("sblas_gen_synth_rows", _i, _i, _i, _i, _i, C.c_ulonglong, _p, _i, _i, _p, _p)
_sig("sblas_gen_vector", _i, _i, C.c_ulonglong, _p)
_sig("sblas_gen_lower_banded", _i, _i, _i, _i, C.c_ulonglong, _p, _p, _p)
_sig("sblas_gen_stencil3d", _i, _i, _i, _i, _i, C.c_ulonglong, _p, _p, _p)
_sig("sblas_gen_rmat", _i, _i, _i, C.c_ulonglong, _p, _p, _p, C.c_longlong)


def check(st: int, what: str = "") -> None:
    if st != 0:
        msg = _STATUS.get(st, str(st))
        detail = lib.sblas_last_error().decode(errors="replace")
        raise SblasError(f"{what}: {msg} ({detail})")


def ptr(a) -> Optional[int]:
    """Raw address of a numpy array or torch tensor (None passes NULL)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()


def device_count() -> int:
    c = C.c_int(0)
    lib.sblas_device_count(C.byref(c))
    return c.value


# --------------------------------------------------------------------------
# host utilities
# --------------------------------------------------------------------------
def mm_read(path: str, mode: int = 0):
    """Matrix-Market -> (m, n, rowptr int64, col int32, val f64).
    mode 0 = mmio_data semantics, 1 = test_spmv 'f', 2 = test_spmv 'b',
    3 = test_spmm's loader (rows bucketed stably, no symmetric expansion)."""
    m, n, nnz = C.c_int(), C.c_int(), C.c_longlong()
    check(lib.sblas_mm_read(path.encode(), mode, C.byref(m), C.byref(n), C.byref(nnz),
                            None, None, None), f"mm_read {path}")
    rp = np.zeros(m.value + 1, np.int64)
    ci = np.zeros(max(nnz.value, 1), np.int32)
    v = np.zeros(max(nnz.value, 1), np.float64)
    check(lib.sblas_mm_read(path.encode(), mode, C.byref(m), C.byref(n), C.byref(nnz),
                            ptr(rp), ptr(ci), ptr(v)), f"mm_read {path}")
    return m.value, n.value, rp, ci[:nnz.value], v[:nnz.value]


def csrbin_write(path: str, m: int, n: int, rowptr, col, val) -> None:
    rp = np.ascontiguousarray(rowptr, np.int64)
    ci = np.ascontiguousarray(col, np.int32)
    v = np.ascontiguousarray(val, np.float64)
    check(lib.sblas_csrbin_write(path.encode(), m, n, int(rp[-1]), ptr(rp), ptr(ci), ptr(v)),
          f"csrbin_write {path}")


def csrbin_read(path: str):
    m, n, nnz = C.c_int(), C.c_int(), C.c_longlong()
    check(lib.sblas_csrbin_read(path.encode(), C.byref(m), C.byref(n), C.byref(nnz), None, None,
                                None), f"csrbin_read {path}")
    rp = np.zeros(m.value + 1, np.int64)
    ci = np.zeros(max(nnz.value, 1), np.int32)
    v = np.zeros(max(nnz.value, 1), np.float64)
    check(lib.sblas_csrbin_read(path.encode(), C.byref(m), C.byref(n), C.byref(nnz), ptr(rp),
                                ptr(ci), ptr(v)), f"csrbin_read {path}")
    return m.value, n.value, rp, ci[:nnz.value], v[:nnz.value]


def partition_nnz(rowptr: np.ndarray, g: int):
    m = len(rowptr) - 1
    nnz = int(rowptr[-1])
    si = np.zeros(g, np.int64); ei = np.zeros(g, np.int64)
    sr = np.zeros(g, np.int32); er = np.zeros(g, np.int32); sf = np.zeros(g, np.int32)
    rp = np.ascontiguousarray(rowptr, np.int64)
    check(lib.sblas_partition_nnz(m, nnz, ptr(rp), g, ptr(si), ptr(ei), ptr(sr), ptr(er), ptr(sf)),
          "partition_nnz")
    return si, ei, sr, er, sf


def partition_cost(rowptr: np.ndarray, g: int, w: float = 3.0):
    """Cost-weighted whole-row split (sblas_partition_cost): contiguous row
    ranges balancing sum(nnz_r + w); same outputs as partition_nnz."""
    m = len(rowptr) - 1
    si = np.zeros(g, np.int64); ei = np.zeros(g, np.int64)
    sr = np.zeros(g, np.int32); er = np.zeros(g, np.int32); sf = np.zeros(g, np.int32)
    rp = np.ascontiguousarray(rowptr, np.int64)
    check(lib.sblas_partition_cost(m, ptr(rp), g, float(w), ptr(si), ptr(ei), ptr(sr), ptr(er), ptr(sf)),
          "partition_cost")
    return si, ei, sr, er, sf


def coo_sortbyrow(m: int, row, col, val):
    """sortbyrow + COO -> CSR of test_spmm (sblas_coo_sortbyrow): returns
    sorted (row, col, val) copies and the int32 rowptr."""
    r = np.array(row, np.int32, copy=True)
    c = np.array(col, np.int32, copy=True)
    v = np.array(val, np.float64, copy=True)
    rp = np.zeros(m + 1, np.int32)
    check(lib.sblas_coo_sortbyrow(m, len(r), ptr(r), ptr(c), ptr(v), ptr(rp)), "coo_sortbyrow")
    return r, c, v, rp


def cyclic_plan(m: int, g: int, chunks_per_rank: int = 8):
    """(chunk_rows, stride) of the cyclic row-chunk distribution."""
    R, S = C.c_longlong(), C.c_longlong()
    check(lib.sblas_cyclic_plan(m, g, chunks_per_rank, C.byref(R), C.byref(S)), "cyclic_plan")
    return R.value, S.value


def cyclic_local_csr(rowptr, col, val, g: int, chunk_rows: int, d: int):
    """Partition d's local CSR (int64 rowptr, col, val) under the cyclic plan."""
    rp = np.ascontiguousarray(rowptr, np.int64)
    ci = np.ascontiguousarray(col, np.int32)
    v = np.ascontiguousarray(val, np.float64)
    m = len(rp) - 1
    lm, lz = C.c_longlong(), C.c_longlong()
    check(lib.sblas_cyclic_local_csr(m, ptr(rp), ptr(ci), ptr(v), g, chunk_rows, d, C.byref(lm),
                                     C.byref(lz), None, None, None), "cyclic_local_csr")
    lrp = np.zeros(lm.value + 1, np.int64)
    lc = np.zeros(max(lz.value, 1), np.int32)
    lv = np.zeros(max(lz.value, 1), np.float64)
    check(lib.sblas_cyclic_local_csr(m, ptr(rp), ptr(ci), ptr(v), g, chunk_rows, d, C.byref(lm),
                                     C.byref(lz), ptr(lrp), ptr(lc), ptr(lv)), "cyclic_local_csr")
    return lrp, lc[:lz.value], lv[:lz.value]


def partition_rowblock(m: int, g: int) -> np.ndarray:
    rs = np.zeros(g + 1, np.int32)
    check(lib.sblas_partition_rowblock(m, g, ptr(rs)), "partition_rowblock")
    return rs


def gen_synth_rowptr(n: int, heavy: int = 96, light: int = 9) -> np.ndarray:
    rp = np.zeros(n + 1, np.int64)
    check(lib.sblas_gen_synth_rowptr(n, heavy, light, ptr(rp)), "gen_synth_rowptr")
    return rp


def gen_synth_rows(n: int, rowptr: np.ndarray, r0: int, r1: int, heavy: int = 96,
                   light: int = 9, prefix: bool = False, seed: int = 42):
    cnt = int(rowptr[r1] - rowptr[r0])
    col = np.zeros(max(cnt, 1), np.int32)
    val = np.zeros(max(cnt, 1), np.float64)
    check(lib.sblas_gen_synth_rows(n, heavy, light, int(prefix), seed, ptr(rowptr), r0, r1,
                                   ptr(col), ptr(val)), "gen_synth_rows")
    return col[:cnt], val[:cnt]


def gen_stencil3d(nx: int, ny: int, nz: int, points: int = 27, seed: int = 49):
    """3-D 7/27-point stencil CSR (int64 rowptr, int32 col, float64 val): the
    structured SuiteSparse kind (sblas_gen_stencil3d)."""
    n = nx * ny * nz
    rp = np.zeros(n + 1, np.int64)
    check(lib.sblas_gen_stencil3d(nx, ny, nz, points, seed, ptr(rp), None, None), "gen_stencil3d")
    nnz = int(rp[-1])
    col = np.zeros(max(nnz, 1), np.int32)
    val = np.zeros(max(nnz, 1), np.float64)
    check(lib.sblas_gen_stencil3d(nx, ny, nz, points, seed, ptr(rp), ptr(col), ptr(val)), "gen_stencil3d")
    return rp, col[:nnz], val[:nnz]


def gen_rmat(scale: int, edge_factor: int = 16, seed: int = 50):
    """R-MAT power-law graph CSR, 2^scale vertices (sblas_gen_rmat)."""
    n = 1 << scale
    cap = edge_factor * n
    rp = np.zeros(n + 1, np.int64)
    col = np.zeros(cap, np.int32)
    val = np.zeros(cap, np.float64)
    check(lib.sblas_gen_rmat(scale, edge_factor, seed, ptr(rp), ptr(col), ptr(val), cap), "gen_rmat")
    nnz = int(rp[-1])
    return rp, col[:nnz].copy(), val[:nnz].copy()


def gen_lower_banded(n: int, offd: int, band: int, seed: int = 47):
    """Unit-lower CSC (colptr, rowidx, val), diagonal first per column."""
    cp = np.zeros(n + 1, np.int32)
    check(lib.sblas_gen_lower_banded(n, offd, band, seed, ptr(cp), None, None), "gen_lower_banded")
    nnz = int(cp[-1])
    ri = np.zeros(max(nnz, 1), np.int32)
    v = np.zeros(max(nnz, 1), np.float64)
    check(lib.sblas_gen_lower_banded(n, offd, band, seed, ptr(cp), ptr(ri), ptr(v)),
          "gen_lower_banded")
    return cp, ri[:nnz], v[:nnz]


def trsv_mgpu_solve(colptr, rowidx, val, n: int, b, ngpu: int, substitution: int = 0,
                    rhs: int = 1):
    """Multi-device sync-free solve from host CSC (sblas_trsv_mgpu_solve);
    b is n x rhs row-major (or length n for rhs 1).  Returns (x, kernel ms)."""
    cp = np.ascontiguousarray(colptr, np.int32)
    ri = np.ascontiguousarray(rowidx, np.int32)
    v = np.ascontiguousarray(val, np.float64)
    bb = np.ascontiguousarray(b, np.float64)
    x = np.zeros(max(n, 1) * rhs, np.float64)
    ms = C.c_double(0.0)
    check(lib.sblas_trsv_mgpu_solve(ptr(cp), ptr(ri), ptr(v), n, substitution, rhs, ptr(bb),
                                    ptr(x), ngpu, C.byref(ms)), "trsv_mgpu_solve")
    x = x[:n * rhs]
    return (x if rhs == 1 else x.reshape(n, rhs)), ms.value


class TrsvMgpu:
    """Persistent multi-GPU sync-free solve (sblas_trsv_mgpu_create/run/
    destroy): the blocks are built and uploaded once; each run uploads b and
    solves."""

    def __init__(self, colptr, rowidx, val, n: int, ngpu: int, substitution: int = 0, rhs: int = 1,
                 tasks: int = 1, balance: int = 0):
        self.h = C.c_void_p()
        self.n, self.rhs = n, rhs
        cp = np.ascontiguousarray(colptr, np.int32)
        ri = np.ascontiguousarray(rowidx, np.int32)
        v = np.ascontiguousarray(val, np.float64)
        check(lib.sblas_trsv_mgpu_create(C.byref(self.h), ptr(cp), ptr(ri), ptr(v), n, substitution, rhs,
                                         ngpu, tasks, balance), "trsv_mgpu_create")

    def run(self, b):
        """Returns (x, kernel ms)."""
        bb = np.ascontiguousarray(b, np.float64)
        x = np.zeros(max(self.n, 1) * self.rhs, np.float64)
        ms = C.c_double(0.0)
        check(lib.sblas_trsv_mgpu_run(self.h, ptr(bb), ptr(x), C.byref(ms)), "trsv_mgpu_run")
        x = x[:self.n * self.rhs]
        return (x if self.rhs == 1 else x.reshape(self.n, self.rhs)), ms.value

    def info(self):
        """[(device, rows)] per block (sblas_trsv_mgpu_info)."""
        nb = C.c_int()
        check(lib.sblas_trsv_mgpu_info(self.h, C.byref(nb), None, None), "trsv_mgpu_info")
        dv = np.zeros(nb.value, np.int32)
        rw = np.zeros(nb.value, np.int32)
        check(lib.sblas_trsv_mgpu_info(self.h, None, ptr(dv), ptr(rw)), "trsv_mgpu_info")
        return [(int(d), int(r)) for d, r in zip(dv, rw)]

    def close(self):
        if self.h:
            lib.sblas_trsv_mgpu_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def trsv_mgpu_solve_tasks(colptr, rowidx, val, n: int, b, ngpu: int, tasks: int,
                          substitution: int = 0, rhs: int = 1, balance: int = 1):
    """ngpu*tasks concurrently running blocks, block d on device d % ngpu
    (sblas_trsv_mgpu_solve_tasks; balance 1 = sptrsv_v3's equal-row split).
    Returns (x, kernel ms)."""
    cp = np.ascontiguousarray(colptr, np.int32)
    ri = np.ascontiguousarray(rowidx, np.int32)
    v = np.ascontiguousarray(val, np.float64)
    bb = np.ascontiguousarray(b, np.float64)
    x = np.zeros(max(n, 1) * rhs, np.float64)
    ms = C.c_double(0.0)
    check(lib.sblas_trsv_mgpu_solve_tasks(ptr(cp), ptr(ri), ptr(v), n, substitution, rhs, ptr(bb),
                                          ptr(x), ngpu, tasks, balance, C.byref(ms)),
          "trsv_mgpu_solve_tasks")
    x = x[:n * rhs]
    return (x if rhs == 1 else x.reshape(n, rhs)), ms.value


def spmv_ooc(m: int, n: int, rowptr, col, val, x, alpha: float, beta: float, y, ngpu: int = 1,
             chunk_nnz: int = 1 << 24, nstreams: int = 2):
    """Out-of-core y = alpha*A*x + beta*y streaming host CSR through the GPUs
    (sblas_spmv_ooc).  y (host float64) is updated in place.  Returns the
    stats dict."""
    rp = np.ascontiguousarray(rowptr, np.int64)
    ci = np.ascontiguousarray(col, np.int32)
    v = np.ascontiguousarray(val, np.float64)
    xx = np.ascontiguousarray(x, np.float64)
    assert y.dtype == np.float64 and y.flags.c_contiguous
    st = np.zeros(6)
    check(lib.sblas_spmv_ooc(m, n, int(rp[-1]), alpha, ptr(rp), ptr(ci), ptr(v), ptr(xx), beta,
                             ptr(y), ngpu, chunk_nnz, nstreams, ptr(st)), "spmv_ooc")
    return {"seconds": st[0], "h2d_gbps": st[1], "chunks": int(st[2]), "devices": int(st[3]),
            "pin_seconds": st[4], "setup_seconds": st[5]}


def csr2csc_mgpu(m: int, n: int, rowptr, col, val, ngpu: int):
    """Multi-device CSR -> CSC of host arrays (sblas_csr2csc_mgpu).
    Returns (colptr, rowidx, val, ms_transpose, ms_compose)."""
    rp = np.ascontiguousarray(rowptr, np.int32)
    nnz = int(rp[-1])
    ci = np.ascontiguousarray(col, np.int32)
    v = np.ascontiguousarray(val, np.float64)
    cp = np.zeros(n + 1, np.int32)
    ri = np.zeros(max(nnz, 1), np.int32)
    cv = np.zeros(max(nnz, 1), np.float64)
    t1, t2 = C.c_double(), C.c_double()
    check(lib.sblas_csr2csc_mgpu(m, n, nnz, ngpu, ptr(rp), ptr(ci), ptr(v), ptr(cp), ptr(ri),
                                 ptr(cv), C.byref(t1), C.byref(t2)), "csr2csc_mgpu")
    return cp, ri[:nnz], cv[:nnz], t1.value, t2.value


def hbm_probe(mode: int, src_ptr: int, dst_ptr: int, nbytes: int, wg_per_cu: int = 8, stream=None) -> None:
    """Enqueue one HBM stream probe (sblas_hbm_probe): 0 read, 1 non-temporal
    read, 2 copy."""
    check(lib.sblas_hbm_probe(mode, src_ptr, dst_ptr, nbytes, wg_per_cu, stream), "hbm_probe")


def hbm_probe_timed(mode: int, src_ptr: int, dst_ptr: int, nbytes: int, wg_per_cu: int = 8, stream=None) -> float:
    """One HBM stream probe, waited for; returns its device span in ms
    (sblas_hbm_probe_timed: runtime-stamped kernel start / end events)."""
    ms = C.c_float(0.0)
    check(lib.sblas_hbm_probe_timed(mode, src_ptr, dst_ptr, nbytes, wg_per_cu, stream, C.byref(ms)),
          "hbm_probe_timed")
    return ms.value


def gen_vector(n: int, seed: int) -> np.ndarray:
    v = np.zeros(max(n, 1), np.float64)
    check(lib.sblas_gen_vector(n, seed, ptr(v)), "gen_vector")
    return v[:n]


# --------------------------------------------------------------------------
# reference operator API (host arrays)
# --------------------------------------------------------------------------
def spmv_mgpu(version: str, m, n, rowptr, col, val, x, y, alpha, beta, ngpu=1, kernel=1,
              nb=None, q=1) -> int:
    """version in {'baseline','v1','v2'}; y updated in place (numpy)."""
    a = np.array([alpha], np.float64)
    b = np.array([beta], np.float64)
    rp = np.ascontiguousarray(rowptr, np.int64)
    nnz = int(rp[-1])
    args = (m, n, nnz, ptr(a), ptr(val), ptr(rp), ptr(col), ptr(x), ptr(b), ptr(y), ngpu)
    if version == "baseline":
        return lib.sblas_spMV_mgpu_baseline(*args)
    if version == "v1":
        return lib.sblas_spMV_mgpu_v1(*args, kernel)
    if version == "v2":
        return lib.sblas_spMV_mgpu_v2(*args, kernel, nb if nb else max(nnz, 1), q)
    raise ValueError(version)


# --------------------------------------------------------------------------
# persistent device objects
# --------------------------------------------------------------------------
class DeviceCSR:
    """A CSR slice resident on one GPU (sblas_csr handle)."""

    def __init__(self, handle: int):
        self.h = C.c_void_p(handle)

    @classmethod
    def upload_slice(cls, device: int, n: int, rowptr: np.ndarray, col: np.ndarray,
                     val: np.ndarray, r0: int, r1: int, i0: int, i1: int, stream=None):
        h = C.c_void_p()
        rp = np.ascontiguousarray(rowptr, np.int64)
        check(lib.sblas_csr_upload_slice(C.byref(h), device, n, ptr(rp), ptr(col), ptr(val),
                                         r0, r1, i0, i1, stream), "csr_upload_slice")
        return cls(h.value)

    @classmethod
    def upload(cls, device: int, n: int, rowptr, col, val, stream=None):
        m = len(rowptr) - 1
        return cls.upload_slice(device, n, rowptr, col, val, 0, m, 0, int(rowptr[-1]), stream)

    def info(self) -> Tuple[int, int, int]:
        m, n, nnz = C.c_int(), C.c_int(), C.c_longlong()
        check(lib.sblas_csr_info(self.h, C.byref(m), C.byref(n), C.byref(nnz)), "csr_info")
        return m.value, n.value, nnz.value

    def analyse(self, algo: int, stream=None) -> None:
        check(lib.sblas_csr_analyse(self.h, algo, stream), "csr_analyse")

    def spmv(self, algo: int, alpha: float, x_ptr: int, beta: float, y_ptr: int,
             stream=None) -> None:
        check(lib.sblas_spmv(self.h, algo, alpha, x_ptr, beta, y_ptr, stream), "spmv")

    def spmv_timed(self, algo: int, alpha: float, x_ptr: int, beta: float, y_ptr: int,
                   stream=None) -> float:
        """sblas_spmv_timed: runs the SpMV, waits, returns its device span in
        ms (first kernel start .. last kernel end)."""
        ms = C.c_float(0.0)
        check(lib.sblas_spmv_timed(self.h, algo, alpha, x_ptr, beta, y_ptr, stream, C.byref(ms)),
              "spmv_timed")
        return float(ms.value)

    def spmm(self, ncols: int, alpha: float, b_ptr: int, ldb: int, b_layout: int, beta: float,
             c_ptr: int, ldc: int, stream=None) -> None:
        check(lib.sblas_spmm(self.h, ncols, alpha, b_ptr, ldb, b_layout, beta, c_ptr, ldc,
                             stream), "spmm")

    def transpose(self, colptr_ptr: int, rowidx_ptr: int, cval_ptr: int, stream=None) -> None:
        check(lib.sblas_csr_transpose(self.h, colptr_ptr, rowidx_ptr, cval_ptr, stream),
              "csr_transpose")

    def pick(self, stream=None) -> int:
        """The algorithm AUTO runs on this handle (sblas_csr_pick)."""
        a = C.c_int()
        check(lib.sblas_csr_pick(self.h, stream, C.byref(a)), "csr_pick")
        return a.value

    def xsort_info(self) -> dict:
        """The analysed XSORT plan's shape (sblas_csr_xsort_info)."""
        v = np.zeros(8, np.int64)
        check(lib.sblas_csr_xsort_info(self.h, ptr(v)), "csr_xsort_info")
        keys = ("ready", "ranges", "wide", "items", "grid", "solo", "chunks", "max_item_chunks")
        return {k: int(x) for k, x in zip(keys, v)}

    @property
    def deterministic(self) -> bool:
        """Bitwise-repeatable launches (sblas_csr_set_deterministic)."""
        v = C.c_int()
        check(lib.sblas_csr_get_deterministic(self.h, C.byref(v)), "csr_get_deterministic")
        return bool(v.value)

    @deterministic.setter
    def deterministic(self, on: bool) -> None:
        check(lib.sblas_csr_set_deterministic(self.h, int(bool(on))), "csr_set_deterministic")

    def panels(self, algo: int) -> int:
        """XCD column panels the analysed plan of `algo` runs over (0 = plain)."""
        p = C.c_int()
        check(lib.sblas_csr_panels(self.h, algo, C.byref(p)), "csr_panels")
        return p.value

    def plan_bytes(self, algo: int) -> int:
        """Device bytes the algorithm's analysis holds beside the CSR."""
        return int(lib.sblas_csr_plan_bytes(self.h, algo))

    def algorithmic_bytes(self, beta_nonzero: bool) -> int:
        return int(lib.sblas_spmv_algorithmic_bytes(self.h, int(beta_nonzero)))

    def close(self) -> None:
        if self.h:
            lib.sblas_csr_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


CTX_ALLGATHER = 0  # sblas_ctx_exchange
CTX_ALLREDUCE = 1


class DeviceCtx:
    """Single-process multi-GPU SpMV context (sblas_ctx: RCCL communicator
    over `ngpu` distinct devices, resident slices, ncclAllGather or
    ncclAllReduce exchange)."""

    def __init__(self, ngpu: int, devices=None):
        self.h = C.c_void_p()
        dl = None if devices is None else np.ascontiguousarray(devices, np.int32)
        check(lib.sblas_ctx_create(C.byref(self.h), ngpu, ptr(dl)), "ctx_create")
        self.ngpu = ngpu
        self.m = 0

    def upload(self, m: int, n: int, rowptr, col, val, algo: int, partition: int = 0,
               exchange: int = CTX_ALLGATHER) -> None:
        rp = np.ascontiguousarray(rowptr, np.int64)
        ci = np.ascontiguousarray(col, np.int32)
        v = np.ascontiguousarray(val, np.float64)
        check(lib.sblas_ctx_matrix_upload_ex(self.h, m, n, ptr(rp), ptr(ci), ptr(v), algo, partition,
                                             exchange), "ctx_matrix_upload")
        self.m = m

    def upload_parts(self, m: int, n: int, rowptr, col, val, algo: int, parts: int) -> None:
        """Cyclic chunks + all-gather with the exchange overlapped over `parts`
        groups of each device's chunks (sblas_ctx_matrix_upload_parts)."""
        rp = np.ascontiguousarray(rowptr, np.int64)
        ci = np.ascontiguousarray(col, np.int32)
        v = np.ascontiguousarray(val, np.float64)
        check(lib.sblas_ctx_matrix_upload_parts(self.h, m, n, ptr(rp), ptr(ci), ptr(v), algo, parts),
              "ctx_matrix_upload_parts")
        self.m = m

    def parts(self) -> int:
        p = C.c_int()
        check(lib.sblas_ctx_parts(self.h, C.byref(p)), "ctx_parts")
        return p.value

    def slice_info(self, d: int):
        """(rows, nnz, algorithmic bytes with beta != 0) of device d's share."""
        r, z, b = C.c_longlong(), C.c_longlong(), C.c_longlong()
        check(lib.sblas_ctx_slice_info(self.h, d, C.byref(r), C.byref(z), C.byref(b)), "ctx_slice_info")
        return r.value, z.value, b.value

    def comm_info(self):
        """(RCCL rank count, device ordinal per context rank) as the
        communicator reports them (ncclCommCount / ncclCommCuDevice; rank
        count 0 for a loopback context)."""
        nr = C.c_int()
        g = C.c_int()
        check(lib.sblas_ctx_ngpu(self.h, C.byref(g)), "ctx_ngpu")
        dv = np.zeros(g.value, np.int32)
        check(lib.sblas_ctx_comm_info(self.h, C.byref(nr), ptr(dv)), "ctx_comm_info")
        return nr.value, [int(d) for d in dv]

    def slice_algo(self, d: int) -> int:
        """The SpMV algorithm device d's slice runs (resolved when AUTO)."""
        a = C.c_int()
        check(lib.sblas_ctx_slice_algo(self.h, d, C.byref(a)), "ctx_slice_algo")
        return a.value

    def spmv_ex(self, alpha: float, beta: float, delay_us: float = 0.0, wait: bool = True):
        """Timing form (sblas_ctx_spmv_ex).  Returns the 3 + 3g stats (ms) when
        wait, else None (sync() collects them)."""
        st = np.zeros(3 + 3 * self.ngpu)
        check(lib.sblas_ctx_spmv_ex(self.h, alpha, beta, delay_us, int(wait), ptr(st)), "ctx_spmv_ex")
        return st if wait else None

    def sync(self) -> np.ndarray:
        st = np.zeros(3 + 3 * self.ngpu)
        check(lib.sblas_ctx_sync(self.h, ptr(st)), "ctx_sync")
        return st

    def set_x(self, x) -> None:
        check(lib.sblas_ctx_set_x(self.h, ptr(np.ascontiguousarray(x, np.float64))), "ctx_set_x")

    def set_y(self, y) -> None:
        check(lib.sblas_ctx_set_y(self.h, ptr(np.ascontiguousarray(y, np.float64))), "ctx_set_y")

    def spmv(self, alpha: float, beta: float):
        """Returns (kernel ms, exchange ms, step ms), max over devices."""
        st = np.zeros(3)
        check(lib.sblas_ctx_spmv(self.h, alpha, beta, ptr(st)), "ctx_spmv")
        return tuple(st)

    def get_y(self, device_index: int = 0) -> np.ndarray:
        y = np.zeros(max(self.m, 1))
        check(lib.sblas_ctx_get_y(self.h, device_index, ptr(y)), "ctx_get_y")
        return y[:self.m]

    def bind(self) -> None:
        check(lib.sblas_ctx_bind(self.h), "ctx_bind")

    @staticmethod
    def unbind() -> None:
        lib.sblas_ctx_bind(None)

    def close(self) -> None:
        if self.h:
            lib.sblas_ctx_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceTRSV:
    def __init__(self, device, n, nnz, colptr_ptr, rowidx_ptr, val_ptr, substitution=0,
                 stream=None):
        self.h = C.c_void_p()
        check(lib.sblas_trsv_create(C.byref(self.h), device, n, nnz, colptr_ptr, rowidx_ptr,
                                    val_ptr, substitution, stream), "trsv_create")

    def solve(self, algo: int, b_ptr: int, x_ptr: int, stream=None) -> None:
        check(lib.sblas_trsv_solve(self.h, algo, b_ptr, x_ptr, stream), "trsv_solve")

    def pick(self, stream=None) -> int:
        """algo 4 (AUTO)'s ticket order for this handle: 1 natural, 3 level order."""
        a = C.c_int(0)
        check(lib.sblas_trsv_pick(self.h, stream, C.byref(a)), "trsv_pick")
        return a.value

    def solve_rhs(self, rhs: int, b_ptr: int, x_ptr: int, stream=None) -> None:
        """SpTRSM: b, x device n x rhs row-major."""
        check(lib.sblas_trsv_solve_rhs(self.h, rhs, b_ptr, x_ptr, stream), "trsv_solve_rhs")

    def solve_rhs_opt(self, algo: int, opt: int, rhs: int, b_ptr: int, x_ptr: int, stream=None) -> None:
        """algo 0: reference push dataflow with lane mapping opt (1 nnz, 2 rhs, 3 auto);
        algo 1: pull executor; 3: pull, tickets in level order; 4: 1 or 3 as pick() chooses."""
        check(lib.sblas_trsv_solve_rhs_opt(self.h, algo, opt, rhs, b_ptr, x_ptr, stream),
              "trsv_solve_rhs_opt")

    def levels(self) -> int:
        n = C.c_int()
        check(lib.sblas_trsv_levels(self.h, C.byref(n)), "trsv_levels")
        return n.value

    def close(self) -> None:
        if self.h:
            lib.sblas_trsv_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def test_deny_peer_access(on: bool) -> None:
    """Test hook: refuse every peer link (sblas_test_deny_peer_access)."""
    check(lib.sblas_test_deny_peer_access(int(bool(on))), "test_deny_peer_access")


def peer_refs(a: int, b: int) -> int:
    """References the library holds on the a -> b peer link."""
    return int(lib.sblas_peer_refs(a, b))


def set_test_option(name: str, value=None) -> None:
    """Planner override for tests (sblas_test_set_option); value None clears
    it.  Read when a plan is built."""
    check(lib.sblas_test_set_option(name.encode(), float(value or 0.0), int(value is not None)),
          "test_set_option")


class test_options:
    """`with sblas.test_options(xs_cap=50): ...` -- planner overrides for the
    plans built inside the block, cleared on exit."""

    def __init__(self, **opts):
        self.opts = opts

    def __enter__(self):
        for k, v in self.opts.items():
            set_test_option(k, v)
        return self

    def __exit__(self, *exc):
        for k in self.opts:
            set_test_option(k, None)
        return False
