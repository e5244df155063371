"""Multi-GPU SpMV over torch.distributed (one process per GPU, RCCL over xGMI).

SURVEY §8 G1: the matrix is split by nnz (dspmv_mgpu_v1.cu:60-94, with the
Q5 fix), each rank keeps its slice resident, x is replicated, and after the
local kernel the y slices are exchanged with ONE collective:

* ``allgather`` (default): every rank contributes its slice padded to the
  largest slice (all_gather_into_tensor == ncclAllGather); the rank-order
  merge of split rows then runs on the device (sblas_assemble_slices), so
  every rank ends with the full y, bit-identical across ranks;
* ``allreduce`` (BASELINE config 3's literal form): each rank places its
  slice into a zero vector of length m and the vectors are summed.

Torch is plumbing here (device buffers, the process group); the kernels are
libsblas's.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass

import numpy as np

import sblas


@dataclass
class Plan:
    world: int
    m: int
    n: int
    nnz: int
    start_idx: np.ndarray
    end_idx: np.ndarray
    start_row: np.ndarray
    end_row: np.ndarray
    start_flag: np.ndarray

    @property
    def nrows(self) -> np.ndarray:
        return (self.end_row - self.start_row + 1).astype(np.int64)

    @property
    def stride(self) -> int:
        return int(max(1, self.nrows.max()))

    def meta(self) -> np.ndarray:
        """{row0, nrows, cont} per rank, int32, as sblas_assemble_slices wants."""
        return np.stack([self.start_row, self.nrows.astype(np.int32),
                         self.start_flag]).T.astype(np.int32).ravel()

    def local(self, rank: int):
        """(row_begin, row_end_exclusive, idx_begin, idx_end_exclusive, cont)."""
        return (int(self.start_row[rank]), int(self.end_row[rank]) + 1,
                int(self.start_idx[rank]), int(self.end_idx[rank]) + 1,
                bool(self.start_flag[rank]))


def make_plan(rowptr: np.ndarray, n: int, world: int, row_cost=None) -> Plan:
    """spMV_mgpu_v1's nnz split (dspmv_mgpu_v1.cu:60-94), or with row_cost =
    w the cost-weighted whole-row split (sblas_partition_cost: ranges
    balancing sum(nnz_r + w), no split rows)."""
    if row_cost is None:
        si, ei, sr, er, sf = sblas.partition_nnz(rowptr, world)
    else:
        si, ei, sr, er, sf = sblas.partition_cost(rowptr, world, row_cost)
    return Plan(world, len(rowptr) - 1, n, int(rowptr[-1]), si, ei, sr, er, sf)


class DistSpMV:
    """One rank's share of a multi-GPU y = alpha*A*x + beta*y."""

    def __init__(self, plan: Plan, rank: int, device: int, rowptr, col_slice, val_slice,
                 algo: int, torch, dist=None, exchange: str = "allgather"):
        self.plan, self.rank, self.algo = plan, rank, algo
        self.torch, self.dist, self.exchange_mode = torch, dist, exchange
        r0, r1, i0, i1, cont = plan.local(rank)
        self.r0, self.r1, self.cont = r0, r1, cont
        dev = torch.device("cuda", device)
        # upload_slice indexes col/val by GLOBAL element index: shift the bases.
        col_base = col_slice.ctypes.data - i0 * 4
        val_base = val_slice.ctypes.data - i0 * 8
        h = sblas.C.c_void_p()
        rp = np.ascontiguousarray(rowptr, np.int64)
        sblas.check(sblas.lib.sblas_csr_upload_slice(sblas.C.byref(h), device, plan.n, rp.ctypes.data,
                                                     col_base, val_base, r0, r1, i0, i1, None),
                    "csr_upload_slice")
        self.A = sblas.DeviceCSR(h.value)
        t0 = time.perf_counter()
        self.A.analyse(algo)
        if algo == sblas.AUTO:  # the library's choice for this slice (sblas_csr_pick)
            self.algo = algo = self.A.pick()
        self.plan_s = time.perf_counter() - t0
        self.dm = r1 - r0
        stride = plan.stride
        f64 = torch.float64
        self.y_full = torch.zeros(plan.m, dtype=f64, device=dev)
        if exchange == "allreduce":
            # BASELINE configs[2]: the kernel writes its rows in place into a
            # zero-padded full-length send buffer; the exchange copies it into
            # y_full and sums y_full over the ranks (ncclAllReduce), then the
            # rank's own rows of the sum become the next call's input
            # (the C-ABI context's SBLAS_CTX_ALLREDUCE, csrc/ctx.hip)
            self.y_send = torch.zeros(max(plan.m, 1), dtype=f64, device=dev)
            self.y_local = self.y_send[r0:r1]
            self.gathered = None
        else:
            self.y_local = torch.zeros(stride, dtype=f64, device=dev)  # padded slice
            self.gathered = torch.zeros(plan.world * stride, dtype=f64, device=dev)
        self.meta = torch.from_numpy(plan.meta()).to(dev)

    def load_y(self, y_full) -> None:
        """Set y (full vector, device tensor) as the next call's input."""
        self.y_full.copy_(y_full)
        if self.exchange_mode == "allreduce":
            self.y_send.zero_()
        self.y_local[: self.dm].copy_(self.y_full[self.r0:self.r1])
        if self.cont and self.dm > 0:
            self.y_local[0] = 0.0

    def kernel(self, alpha: float, x, beta: float, stream=None) -> None:
        self.A.spmv(self.algo, alpha, x.data_ptr(), beta, self.y_local.data_ptr(), stream)

    def exchange(self, stream=None) -> None:
        if self.plan.world == 1:
            return
        if self.exchange_mode == "allgather":
            if self.dist.get_backend() == "nccl":
                self.dist.all_gather_into_tensor(self.gathered, self.y_local)
            else:  # gloo rehearsal path (CPU staging)
                chunks = [c.cpu() for c in self.gathered.chunk(self.plan.world)]
                self.dist.all_gather(chunks, self.y_local.cpu())
                self.gathered.copy_(self.torch.cat(chunks).to(self.gathered.device))
            sblas.check(sblas.lib.sblas_assemble_slices(
                self.gathered.data_ptr(), self.plan.world, self.plan.stride, self.meta.data_ptr(),
                self.y_full.data_ptr(), self.rank, self.y_local.data_ptr(), stream),
                "assemble_slices")
        else:  # literal allreduce of the zero-padded y (config 3)
            self.y_full.copy_(self.y_send[: self.plan.m])
            if self.dist.get_backend() == "nccl":
                self.dist.all_reduce(self.y_full)
            else:
                h = self.y_full.cpu()
                self.dist.all_reduce(h)
                self.y_full.copy_(h.to(self.y_full.device))
            # re-prime: own rows of the sum; a continuation row restarts from
            # 0 (the previous rank adds beta*y for it)
            self.y_local.copy_(self.y_full[self.r0:self.r1])
            if self.cont and self.dm > 0:
                self.y_local[0] = 0.0

    def result(self):
        """Full y after exchange (world 1: the local slice is the whole y)."""
        if self.plan.world == 1:
            return self.y_local[: self.plan.m]
        return self.y_full

    def close(self):
        self.A.close()


# ---------------------------------------------------------------------------
# Cyclic row-chunk distribution.  The nnz split above keeps one contiguous
# row range per rank, so on config 2 (heavy rows first) the light-row ranks
# hold 2.3x the average row count and the padded allgather moves 37 MB
# instead of 16 MB at N = 8.  Dealing equal-row chunks round-robin (chunk j
# -> rank j % world, ScaLAPACK-style block-cyclic rows) gives every rank the
# same row count and, for any row-length profile that is smooth at chunk
# scale, the same nnz; ranks own whole rows, so no split-row carries.
# ---------------------------------------------------------------------------
@dataclass
class CyclicPlan:
    world: int
    m: int
    n: int
    nnz: int
    chunk_rows: int

    @property
    def nchunks(self) -> int:
        return -(-self.m // self.chunk_rows) if self.m else 0

    @property
    def stride(self) -> int:
        """Rows of one rank's (padded) slice: ceil(nchunks / world) chunks."""
        return max(1, -(-self.nchunks // self.world) * self.chunk_rows)

    def chunks(self, rank: int):
        """[(row_begin, row_end_exclusive)] of the chunks `rank` holds, in
        local order."""
        R = self.chunk_rows
        return [(j * R, min(self.m, (j + 1) * R)) for j in range(rank, self.nchunks, self.world)]

    def local_rows(self, rank: int) -> int:
        return sum(b - a for a, b in self.chunks(rank))


def make_cyclic_plan(rowptr: np.ndarray, n: int, world: int, chunks_per_rank: int = 8) -> CyclicPlan:
    m = len(rowptr) - 1
    R = max(1, -(-m // max(1, world * chunks_per_rank)))
    return CyclicPlan(world, m, n, int(rowptr[-1]), R)


def cyclic_local_csr(rowptr: np.ndarray, plan: CyclicPlan, rank: int, rows_fn):
    """Local CSR of `rank` (its chunks' rows concatenated in local order).
    rows_fn(r0, r1) -> (col, val) of global rows [r0, r1)."""
    rp = np.asarray(rowptr, np.int64)
    parts = plan.chunks(rank)
    lens = [rp[a + 1:b + 1] - rp[a:b] for a, b in parts]
    lrp = np.zeros(sum(len(x) for x in lens) + 1, np.int64)
    if len(lrp) > 1:
        lrp[1:] = np.cumsum(np.concatenate(lens))
    cols, vals = [], []
    for a, b in parts:
        c, v = rows_fn(a, b)
        cols.append(np.asarray(c, np.int32))
        vals.append(np.asarray(v, np.float64))
    col = np.concatenate(cols) if cols else np.zeros(0, np.int32)
    val = np.concatenate(vals) if vals else np.zeros(0, np.float64)
    return lrp, np.ascontiguousarray(col), np.ascontiguousarray(val)


def overlap_halves(plan: CyclicPlan):
    """Two-half split of the cyclic deal for the overlapped exchange.

    Each rank's first hA local chunks (global chunks < hA * world) form half A,
    the rest half B; each half is dealt cyclically on its own, so each is
    placed by one sblas_assemble_cyclic call.  Returns (hA, strideA, strideB,
    rows_a): per-rank slice lengths of the halves and the global rows of
    half A (half B starts at row rows_a)."""
    R, g = plan.chunk_rows, plan.world
    ncmax = -(-plan.nchunks // g)
    hA = (ncmax + 1) // 2
    strideA = hA * R
    strideB = max(1, plan.stride - strideA)
    rows_a = min(plan.m, hA * g * R)
    return hA, strideA, strideB, rows_a


class DistSpMVCyclic:
    """One rank's share of y = alpha*A*x + beta*y under the cyclic row-chunk
    distribution: the rank's rows are uploaded as one local CSR, y_local is
    its (padded) slice, the exchange is one all_gather_into_tensor of equal
    slices (no padding beyond the last chunk) and sblas_assemble_cyclic
    places every chunk at its global rows.  y_local already is the next
    call's y input (whole rows), so nothing is copied back."""

    def __init__(self, plan: CyclicPlan, rank: int, device: int, local_rowptr, col, val,
                 algo: int, torch, dist=None, overlap: bool = False):
        self.plan, self.rank, self.algo = plan, rank, algo
        self.torch, self.dist = torch, dist
        self.dm = len(local_rowptr) - 1
        dev = torch.device("cuda", device)
        lrp64 = np.ascontiguousarray(local_rowptr, np.int64)
        col = np.ascontiguousarray(col, np.int32)
        val = np.ascontiguousarray(val, np.float64)
        self.A = sblas.DeviceCSR.upload(device, plan.n, lrp64, col, val)
        t0 = time.perf_counter()
        self.A.analyse(algo)
        if algo == sblas.AUTO:  # the library's choice for this slice (sblas_csr_pick)
            self.algo = algo = self.A.pick()
        self.plan_s = time.perf_counter() - t0
        f64 = torch.float64
        self.y_local = torch.zeros(plan.stride, dtype=f64, device=dev)
        self.y_full = torch.zeros(plan.m, dtype=f64, device=dev)
        self.gathered = torch.zeros(plan.world * plan.stride, dtype=f64, device=dev)
        # overlap: the rank's chunks in two halves (the first hA local chunks
        # of every rank, then the rest), each its own handle; the all-gather
        # of half A runs while half B's kernel runs
        # (needs two chunks per rank to split)
        # SBLAS_DIST_XCHG_W1=1 (with a process group at world size 1): run the
        # exchange and placement path anyway, so one GPU exercises it over RCCL
        self.xw1 = os.environ.get("SBLAS_DIST_XCHG_W1") == "1" and dist is not None
        self.overlap = bool(overlap) and (plan.world > 1 or self.xw1) and plan.nchunks > plan.world
        self._work = []
        if self.overlap:
            self.hA, self.strideA, self.strideB, self.rows_a = overlap_halves(plan)
            rA = min(self.dm, self.strideA)
            self.halves = []
            for r0, r1 in ((0, rA), (rA, self.dm)):
                H = None
                if r1 > r0:
                    H = sblas.DeviceCSR.upload_slice(device, plan.n, lrp64, col, val, r0, r1,
                                                     int(lrp64[r0]), int(lrp64[r1]))
                    H.analyse(algo)
                self.halves.append((H, r0, r1))
            self.gA = torch.zeros(plan.world * self.strideA, dtype=f64, device=dev)
            self.gB = torch.zeros(plan.world * self.strideB, dtype=f64, device=dev)

    def load_y(self, y_full) -> None:
        self.y_full.copy_(y_full)
        o = 0
        for a, b in self.plan.chunks(self.rank):
            self.y_local[o:o + b - a].copy_(self.y_full[a:b])
            o += b - a

    def kernel(self, alpha: float, x, beta: float, stream=None) -> None:
        if self.overlap:
            (HA, a0, _), (HB, b0, _) = self.halves
            if HA is not None:
                HA.spmv(self.algo, alpha, x.data_ptr(), beta, self.y_local.data_ptr() + 8 * a0, stream)
            if self.dist.get_backend() == "nccl":  # collective stream waits for half A only
                self._work.append(self.dist.all_gather_into_tensor(
                    self.gA, self.y_local[: self.strideA], async_op=True))
            if HB is not None:
                HB.spmv(self.algo, alpha, x.data_ptr(), beta, self.y_local.data_ptr() + 8 * b0, stream)
            return
        if self.dm > 0:
            self.A.spmv(self.algo, alpha, x.data_ptr(), beta, self.y_local.data_ptr(), stream)

    def _gather_gloo(self, out, inp):
        chunks = [c.cpu() for c in out.chunk(self.plan.world)]
        self.dist.all_gather(chunks, inp.cpu())
        out.copy_(self.torch.cat(chunks).to(out.device))

    def exchange(self, stream=None) -> None:
        if self.plan.world == 1 and not self.xw1:
            return
        if self.overlap:
            yB = self.y_local[self.strideA: self.strideA + self.strideB]
            if self.dist.get_backend() == "nccl":
                self._work.append(self.dist.all_gather_into_tensor(self.gB, yB, async_op=True))
                for w in self._work:
                    w.wait()
                self._work = []
            else:  # gloo rehearsal: same data flow, no overlap
                self._gather_gloo(self.gA, self.y_local[: self.strideA])
                self._gather_gloo(self.gB, yB)
            p, R, g, rows_a = self.plan, self.plan.chunk_rows, self.plan.world, self.rows_a
            sblas.check(sblas.lib.sblas_assemble_cyclic(
                self.gA.data_ptr(), g, self.strideA, R, rows_a, self.y_full.data_ptr(), stream),
                "assemble_cyclic")
            if p.m > rows_a:
                sblas.check(sblas.lib.sblas_assemble_cyclic(
                    self.gB.data_ptr(), g, self.strideB, R, p.m - rows_a,
                    self.y_full.data_ptr() + 8 * rows_a, stream), "assemble_cyclic")
            return
        if self.dist.get_backend() == "nccl":
            self.dist.all_gather_into_tensor(self.gathered, self.y_local)
        else:  # gloo rehearsal path (CPU staging)
            chunks = [c.cpu() for c in self.gathered.chunk(self.plan.world)]
            self.dist.all_gather(chunks, self.y_local.cpu())
            self.gathered.copy_(self.torch.cat(chunks).to(self.gathered.device))
        sblas.check(sblas.lib.sblas_assemble_cyclic(
            self.gathered.data_ptr(), self.plan.world, self.plan.stride, self.plan.chunk_rows,
            self.plan.m, self.y_full.data_ptr(), stream), "assemble_cyclic")

    def result(self):
        if self.plan.world == 1 and not self.xw1:
            return self.y_local[: self.plan.m]
        return self.y_full

    def close(self):
        self.A.close()
        for H, _, _ in getattr(self, "halves", []):
            if H is not None:
                H.close()


# ---------------------------------------------------------------------------
# SpMM: rows of A split by nnz into whole-row blocks, B
# replicated on every rank, C row slices disjoint -> one all-gather, no
# split-row fix-up.  (The reference's alternative, B split by columns with A
# replicated, needs no exchange at all; the row split is the one that scales
# A's footprint and bytes with the rank count.)
# ---------------------------------------------------------------------------
def row_blocks_by_nnz(rowptr: np.ndarray, world: int) -> np.ndarray:
    """world+1 row boundaries; block d holds whole rows, ~nnz/world nonzeros
    (first row whose start reaches d*nnz/world)."""
    rp = np.asarray(rowptr, np.int64)
    nnz = int(rp[-1])
    targets = (np.arange(world + 1, dtype=np.int64) * nnz) // max(world, 1)
    rb = np.searchsorted(rp, targets, side="left").astype(np.int64)
    rb[0], rb[-1] = 0, len(rp) - 1
    return np.maximum.accumulate(rb)


def spmm_grid_shape(world: int, ncols: int):
    """(row blocks, column groups) of DistSpMM's split "grid": the most column
    groups that leave every rank a multiple of 16 C columns (the C tile's
    16-column fast path), the rest of the ranks as whole-row blocks by nnz.
    A rank then reads 1/R of A and its 1/Cg of every B row its rows touch;
    on configs[3] (64 columns) N = 2 / 4 / 8 -> (1, 2) / (1, 4) / (2, 4)."""
    for cg in range(world, 0, -1):
        if world % cg == 0 and ncols % cg == 0 and (ncols // cg) % 16 == 0:
            return world // cg, cg
    return world, 1


class DistSpMM:
    """One rank's share of C = alpha*A*B + beta*C (B row-major k x ncols on
    every rank; C column-major m x ncols, kept as a (ncols, m) tensor).

    split "rows" (default, the north star's partition): whole-row blocks of A
    by nnz, C row slices all-gathered.  split "cols" (the reference's own,
    dspmm_mgpu_baseline.cu:147-150): A replicated, rank d owns C/B columns
    [floor(d*n/g), floor((d+1)*n/g)) -- its C slice is a contiguous block of
    the (ncols, m) tensor -- and the column slices are all-gathered.  split
    "grid": both at once (spmm_grid_shape): rank d = (row block d // Cg,
    column group d % Cg) owns that C block; the blocks are all-gathered and
    placed."""

    def __init__(self, rowptr, col, val, k: int, ncols: int, world: int, rank: int, device: int,
                 torch, dist=None, split: str = "rows"):
        self.torch, self.dist, self.world, self.rank = torch, dist, world, rank
        rp = np.ascontiguousarray(rowptr, np.int64)
        self.m, self.ncols = len(rp) - 1, ncols
        self.split = split
        if split == "cols":
            self._init_cols(rp, col, val, k, device)
            return
        if split == "grid":
            self._init_grid(rp, col, val, k, device)
            return
        self.rb = row_blocks_by_nnz(rp, world)
        r0, r1 = int(self.rb[rank]), int(self.rb[rank + 1])
        i0, i1 = int(rp[r0]), int(rp[r1])
        self.r0, self.r1 = r0, r1
        self.A = sblas.DeviceCSR.upload_slice(device, k, rp, np.ascontiguousarray(col, np.int32),
                                              np.ascontiguousarray(val, np.float64), r0, r1, i0, i1)
        self.stride = int(max(1, np.diff(self.rb).max()))
        dev = torch.device("cuda", device)
        f64 = torch.float64
        self.c_local = torch.zeros((ncols, self.stride), dtype=f64, device=dev)  # ld = stride
        self.gathered = torch.zeros((world, ncols, self.stride), dtype=f64, device=dev)
        self.c_full = torch.zeros((ncols, self.m), dtype=f64, device=dev)

    def _init_cols(self, rp, col, val, k, device):
        torch, m, n, g = self.torch, self.m, self.ncols, self.world
        self.cb = [d * n // g for d in range(g + 1)]
        self.c0, self.c1 = self.cb[self.rank], self.cb[self.rank + 1]
        self.A = sblas.DeviceCSR.upload_slice(device, k, rp, np.ascontiguousarray(col, np.int32),
                                              np.ascontiguousarray(val, np.float64), 0, m, 0, int(rp[-1]))
        self.wmax = max(self.cb[d + 1] - self.cb[d] for d in range(g))
        dev = torch.device("cuda", device)
        f64 = torch.float64
        self.c_local = torch.zeros((max(self.wmax, 1), m), dtype=f64, device=dev)
        self.gathered = torch.zeros((g, max(self.wmax, 1), m), dtype=f64, device=dev)
        self.c_full = torch.zeros((n, m), dtype=f64, device=dev)
        self.stride = m

    def _init_grid(self, rp, col, val, k, device):
        torch, n, g = self.torch, self.ncols, self.world
        self.R, self.Cg = spmm_grid_shape(g, n)
        self.rb = row_blocks_by_nnz(rp, self.R)
        self.cb = [c * n // self.Cg for c in range(self.Cg + 1)]
        ri, ci = self.rank // self.Cg, self.rank % self.Cg
        self.r0, self.r1 = int(self.rb[ri]), int(self.rb[ri + 1])
        self.c0, self.c1 = self.cb[ci], self.cb[ci + 1]
        i0, i1 = int(rp[self.r0]), int(rp[self.r1])
        self.A = sblas.DeviceCSR.upload_slice(device, k, rp, np.ascontiguousarray(col, np.int32),
                                              np.ascontiguousarray(val, np.float64), self.r0, self.r1, i0, i1)
        self.stride = int(max(1, np.diff(self.rb).max()))
        self.wc = n // self.Cg
        dev = torch.device("cuda", device)
        f64 = torch.float64
        self.c_local = torch.zeros((self.wc, self.stride), dtype=f64, device=dev)  # ld = stride
        self.gathered = torch.zeros((g, self.wc, self.stride), dtype=f64, device=dev)
        self.c_full = torch.zeros((n, self.m), dtype=f64, device=dev)

    def _grid_block(self, d):
        ri, ci = d // self.Cg, d % self.Cg
        return int(self.rb[ri]), int(self.rb[ri + 1]), self.cb[ci], self.cb[ci + 1]

    def load_c(self, c_full) -> None:
        """Set C (a (ncols, m) device tensor) as the next call's input."""
        self.c_full.copy_(c_full)
        if self.split == "grid":
            self.c_local[:, : self.r1 - self.r0].copy_(self.c_full[self.c0:self.c1, self.r0:self.r1])
            return
        if self.split == "cols":
            self.c_local[: self.c1 - self.c0].copy_(self.c_full[self.c0:self.c1])
            return
        self.c_local[:, : self.r1 - self.r0].copy_(self.c_full[:, self.r0:self.r1])

    def kernel(self, alpha: float, B, beta: float, stream=None) -> None:
        if self.split == "grid":  # rows [r0, r1) x B/C columns [c0, c1), ld = ncols
            if self.r1 > self.r0:
                self.A.spmm(self.wc, alpha, B.data_ptr() + 8 * self.c0, self.ncols, 1, beta,
                            self.c_local.data_ptr(), self.stride, stream)
            return
        if self.split == "cols":
            dn = self.c1 - self.c0
            if dn > 0 and self.m > 0:  # B[:, c0:c1] row-major with ld = ncols
                self.A.spmm(dn, alpha, B.data_ptr() + 8 * self.c0, self.ncols, 1, beta,
                            self.c_local.data_ptr(), self.m, stream)
            return
        if self.r1 > self.r0:
            self.A.spmm(self.ncols, alpha, B.data_ptr(), self.ncols, 1, beta,
                        self.c_local.data_ptr(), self.stride, stream)

    def exchange(self) -> None:
        if self.world == 1:
            return
        if self.split == "grid":
            if self.dist.get_backend() == "nccl":
                self.dist.all_gather_into_tensor(self.gathered.view(-1), self.c_local.reshape(-1))
            else:  # gloo rehearsal (CPU staging)
                parts = [torch_zeros_like_cpu(self.c_local) for _ in range(self.world)]
                self.dist.all_gather(parts, self.c_local.cpu())
                self.gathered.copy_(self.torch.stack(parts).to(self.gathered.device))
            for d in range(self.world):
                r0, r1, c0, c1 = self._grid_block(d)
                if r1 > r0:
                    self.c_full[c0:c1, r0:r1].copy_(self.gathered[d, :, : r1 - r0])
            self.c_local[:, : self.r1 - self.r0].copy_(self.c_full[self.c0:self.c1, self.r0:self.r1])
            return
        if self.split == "cols":
            if self.dist.get_backend() == "nccl":
                self.dist.all_gather_into_tensor(self.gathered.view(-1), self.c_local.reshape(-1))
            else:  # gloo rehearsal (CPU staging)
                parts = [torch_zeros_like_cpu(self.c_local) for _ in range(self.world)]
                self.dist.all_gather(parts, self.c_local.cpu())
                self.gathered.copy_(self.torch.stack(parts).to(self.gathered.device))
            for d in range(self.world):
                a, b = self.cb[d], self.cb[d + 1]
                if b > a:
                    self.c_full[a:b].copy_(self.gathered[d, : b - a])
            self.c_local[: self.c1 - self.c0].copy_(self.c_full[self.c0:self.c1])
            return
        if self.dist.get_backend() == "nccl":
            self.dist.all_gather_into_tensor(self.gathered.view(-1), self.c_local.reshape(-1))
        else:  # gloo rehearsal (CPU staging)
            parts = [torch_zeros_like_cpu(self.c_local) for _ in range(self.world)]
            self.dist.all_gather(parts, self.c_local.cpu())
            self.gathered.copy_(self.torch.stack(parts).to(self.gathered.device))
        for d in range(self.world):
            a, b = int(self.rb[d]), int(self.rb[d + 1])
            if b > a:
                self.c_full[:, a:b].copy_(self.gathered[d, :, : b - a])
        self.c_local[:, : self.r1 - self.r0].copy_(self.c_full[:, self.r0:self.r1])

    def result(self):
        if self.world == 1:
            return self.c_local[: self.ncols] if self.split == "cols" else self.c_local[:, : self.m]
        return self.c_full

    def close(self) -> None:
        self.A.close()


def torch_zeros_like_cpu(t):
    import torch
    return torch.zeros(t.shape, dtype=t.dtype)
