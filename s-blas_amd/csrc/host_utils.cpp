// host_utils.cpp -- host-side pieces of libsblas that need no GPU:
// Matrix-Market reader, partitions, synthetic generators, timers.
//
// Semantics follow the reference (cited per function); the implementation is
// our own: the MM reader slurps the file once and parses in place (the
// reference fscanf's entry by entry, dspmv_test.cu:122-136), and the
// generator is row-parallel (one counter-based stream per row).
#include <sys/stat.h>
#include <sys/time.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sblas.h"

namespace sblas {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

const char *last_error() { return g_err; }

int row_of_index(int m, const long long *rowptr, long long idx)
{
    int lo = 0, hi = m;  // last r in [0, m] with rowptr[r] <= idx
    while (lo < hi) {
        const int mid = lo + (hi - lo + 1) / 2;
        if (rowptr[mid] <= idx) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// ---------------------------------------------------------------------------
// Matrix Market
// ---------------------------------------------------------------------------
namespace {

struct MMFile {
    std::string buf;
    size_t pos = 0;
    int m = 0, n = 0;
    long long nz = 0;
    bool pattern = false, real = false, complex_ = false, integer = false, sym = false;
};

bool ieq(const char *a, const char *b)
{
    for (; *a && *b; ++a, ++b)
        if (std::tolower((unsigned char)*a) != std::tolower((unsigned char)*b)) return false;
    return *a == 0 && *b == 0;
}

// mm_read_banner (mmio.h:254) + mm_read_mtx_crd_size (mmio.h:339) semantics.
bool mm_open(const char *path, MMFile &F)
{
    FILE *f = std::fopen(path, "rb");
    if (!f) {
        set_error("cannot open %s", path);
        return false;
    }
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    F.buf.resize(sz > 0 ? (size_t)sz : 0);
    if (sz > 0 && std::fread(&F.buf[0], 1, (size_t)sz, f) != (size_t)sz) {
        std::fclose(f);
        set_error("short read %s", path);
        return false;
    }
    std::fclose(f);
    F.buf.push_back('\0');
    auto next_line = [&](std::string &line) -> bool {
        if (F.pos >= F.buf.size() - 1) return false;
        const size_t e = F.buf.find('\n', F.pos);
        const size_t end = e == std::string::npos ? F.buf.size() - 1 : e;
        line.assign(F.buf, F.pos, end - F.pos);
        F.pos = end + 1;
        return true;
    };
    std::string line;
    if (!next_line(line)) return false;
    char banner[64] = {0}, obj[64] = {0}, fmt[64] = {0}, field[64] = {0}, symm[64] = {0};
    if (std::sscanf(line.c_str(), "%63s %63s %63s %63s %63s", banner, obj, fmt, field, symm) != 5 ||
        std::strcmp(banner, "%%MatrixMarket") != 0 || !ieq(obj, "matrix") || !ieq(fmt, "coordinate")) {
        set_error("%s: not a Matrix-Market coordinate file", path);
        return false;
    }
    F.pattern = ieq(field, "pattern");
    F.real = ieq(field, "real");
    F.complex_ = ieq(field, "complex");
    F.integer = ieq(field, "integer");
    F.sym = ieq(symm, "symmetric") || ieq(symm, "hermitian");
    do {
        if (!next_line(line)) {
            set_error("%s: missing size line", path);
            return false;
        }
    } while (!line.empty() && line[0] == '%');
    long long a, b, c;
    if (std::sscanf(line.c_str(), "%lld %lld %lld", &a, &b, &c) != 3) {
        set_error("%s: bad size line", path);
        return false;
    }
    F.m = (int)a;
    F.n = (int)b;
    F.nz = c;
    return true;
}

inline const char *skip_ws(const char *p)
{
    while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r') ++p;
    return p;
}
inline const char *parse_int(const char *p, long long &v)
{
    p = skip_ws(p);
    bool neg = false;
    if (*p == '-' || *p == '+') neg = *p++ == '-';
    long long r = 0;
    const char *s = p;
    while (*p >= '0' && *p <= '9') r = r * 10 + (*p++ - '0');
    if (p == s) return nullptr;
    v = neg ? -r : r;
    return p;
}
inline const char *parse_dbl(const char *p, double &v)
{
    p = skip_ws(p);
    char *e = nullptr;
    v = std::strtod(p, &e);
    return e == p ? nullptr : e;
}


// ---- parsed CSR, memo, parallel parse, .csrbin cache ----------------------
struct HostCsr {
    int m = 0, n = 0;
    long long nnz = 0;
    std::vector<long long> rowptr;
    std::vector<int> col;
    std::vector<double> val;
};

struct FileId {
    long long size = -1, mtime = 0;
};

FileId file_id(const char *path)
{
    struct stat st;
    FileId f;
    if (::stat(path, &st) == 0) {
        f.size = (long long)st.st_size;
        f.mtime = (long long)st.st_mtim.tv_sec * 1000000000LL + st.st_mtim.tv_nsec;
    }
    return f;
}

struct Memo {
    std::string path;
    int mode = -1;
    FileId id;
    HostCsr A;
};
thread_local Memo g_memo;

HostCsr *memo_lookup(const char *path, int mode)
{
    if (g_memo.mode != mode || g_memo.path != path) return nullptr;
    const FileId f = file_id(path);
    if (f.size != g_memo.id.size || f.mtime != g_memo.id.mtime) return nullptr;
    return &g_memo.A;
}

HostCsr &memo_slot(const char *path, int mode)
{
    g_memo = Memo();
    g_memo.path = path;
    g_memo.mode = mode;
    g_memo.id = file_id(path);
    return g_memo.A;
}

void memo_clear() { g_memo = Memo(); }

// .csrbin: "SBLASCSR" | u32 version | i32 mode (-1: written by the user) |
// i64 source size | i64 source mtime | i32 m | i32 n | i64 nnz |
// i64 rowptr[m+1] | i32 col[nnz] | f64 val[nnz]
constexpr char kBinMagic[8] = {'S', 'B', 'L', 'A', 'S', 'C', 'S', 'R'};
constexpr uint32_t kBinVersion = 1;

int csrbin_store(const char *path, int mode, long long src_size, long long src_mtime, int m, int n,
                 long long nnz, const long long *rowptr, const int *col, const double *val)
{
    const std::string tmp = std::string(path) + ".tmp";
    FILE *f = std::fopen(tmp.c_str(), "wb");
    if (!f) {
        set_error("cannot write %s", tmp.c_str());
        return SBLAS_ERR_IO;
    }
    const int32_t mode32 = mode, m32 = m, n32 = n;
    const int64_t sz = src_size, mt = src_mtime, nz = nnz;
    bool ok = std::fwrite(kBinMagic, 1, 8, f) == 8 && std::fwrite(&kBinVersion, 4, 1, f) == 1 &&
              std::fwrite(&mode32, 4, 1, f) == 1 && std::fwrite(&sz, 8, 1, f) == 1 &&
              std::fwrite(&mt, 8, 1, f) == 1 && std::fwrite(&m32, 4, 1, f) == 1 &&
              std::fwrite(&n32, 4, 1, f) == 1 && std::fwrite(&nz, 8, 1, f) == 1 &&
              std::fwrite(rowptr, 8, (size_t)m + 1, f) == (size_t)m + 1 &&
              (nnz == 0 || (std::fwrite(col, 4, (size_t)nnz, f) == (size_t)nnz &&
                            std::fwrite(val, 8, (size_t)nnz, f) == (size_t)nnz));
    ok = (std::fclose(f) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), path) != 0) {
        std::remove(tmp.c_str());
        set_error("cannot write %s", path);
        return SBLAS_ERR_IO;
    }
    return SBLAS_OK;
}

// mode >= 0: the file must have been made from a source with this size/mtime
int csrbin_load(const char *path, int mode, long long src_size, long long src_mtime, HostCsr &A)
{
    FILE *f = std::fopen(path, "rb");
    if (!f) {
        set_error("cannot open %s", path);
        return SBLAS_ERR_IO;
    }
    char magic[8];
    uint32_t ver = 0;
    int32_t mode32 = 0, m32 = 0, n32 = 0;
    int64_t sz = 0, mt = 0, nz = 0;
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, kBinMagic, 8) == 0 &&
              std::fread(&ver, 4, 1, f) == 1 && ver == kBinVersion && std::fread(&mode32, 4, 1, f) == 1 &&
              std::fread(&sz, 8, 1, f) == 1 && std::fread(&mt, 8, 1, f) == 1 &&
              std::fread(&m32, 4, 1, f) == 1 && std::fread(&n32, 4, 1, f) == 1 &&
              std::fread(&nz, 8, 1, f) == 1 && m32 >= 0 && n32 >= 0 && nz >= 0;
    if (ok && mode >= 0) ok = mode32 == mode && sz == src_size && mt == src_mtime;
    if (ok) {
        A.m = m32;
        A.n = n32;
        A.nnz = nz;
        A.rowptr.resize((size_t)m32 + 1);
        A.col.resize((size_t)nz);
        A.val.resize((size_t)nz);
        ok = std::fread(A.rowptr.data(), 8, (size_t)m32 + 1, f) == (size_t)m32 + 1 &&
             (nz == 0 || (std::fread(A.col.data(), 4, (size_t)nz, f) == (size_t)nz &&
                          std::fread(A.val.data(), 8, (size_t)nz, f) == (size_t)nz)) &&
             A.rowptr[0] == 0 && A.rowptr[(size_t)m32] == nz;
    }
    std::fclose(f);
    if (!ok) {
        set_error("%s: not a valid .csrbin (or stale for this source)", path);
        return SBLAS_ERR_IO;
    }
    return SBLAS_OK;
}

// Parses the entries of F (from F.pos) in parallel, in file order.
int parse_entries(const MMFile &F, int mode, const char *path, std::vector<int> &ri,
                  std::vector<int> &ci, std::vector<double> &vi)
{
    const char *base = F.buf.c_str();
    const size_t b0 = F.pos, b1 = F.buf.size() - 1;  // trailing '\0'
    const long long nz = F.nz;
    int T = 1;
#ifdef _OPENMP
    T = std::max(1, std::min(omp_get_max_threads(), 64));
#endif
    if ((long long)(b1 - b0) < (1LL << 20)) T = 1;
    std::vector<size_t> cut((size_t)T + 1);
    cut[0] = b0;
    cut[(size_t)T] = b1;
    for (int t = 1; t < T; ++t) {
        size_t c = b0 + (b1 - b0) * (size_t)t / (size_t)T;
        while (c < b1 && base[c - 1] != '\n') ++c;  // start of a line
        cut[(size_t)t] = std::max(c, cut[(size_t)t - 1]);
    }
    struct Part {
        std::vector<int> r, c;
        std::vector<double> v;
        long long bad = -1;  // byte offset of the first malformed entry
    };
    std::vector<Part> parts((size_t)T);
#pragma omp parallel for num_threads(T) schedule(static, 1)
    for (int t = 0; t < T; ++t) {
        Part &P = parts[(size_t)t];
        const size_t guess = (size_t)((double)nz * (double)(cut[(size_t)t + 1] - cut[(size_t)t]) /
                                      (double)std::max<size_t>(b1 - b0, 1)) + 16;
        P.r.reserve(guess);
        P.c.reserve(guess);
        P.v.reserve(guess);
        const char *p = base + cut[(size_t)t];
        const char *end = base + cut[(size_t)t + 1];
        while (true) {
            p = skip_ws(p);
            if (p >= end || *p == 0) break;
            const char *line = p;
            long long r, c;
            double v = 0.0;
            bool ok = (p = parse_int(p, r)) && (p = parse_int(p, c));
            if (ok) {
                if (mode == 0) {
                    if (F.real || F.complex_) {
                        ok = (p = parse_dbl(p, v)) != nullptr;
                        double im;
                        if (ok && F.complex_) ok = (p = parse_dbl(p, im)) != nullptr;
                    } else if (F.integer) {
                        long long iv;
                        ok = (p = parse_int(p, iv)) != nullptr;
                        v = (double)iv;
                    } else {
                        v = 1.0;
                    }
                } else if (mode == 1 || mode == 3) {
                    ok = (p = parse_dbl(p, v)) != nullptr;
                } else {
                    v = 0.00001;
                }
            }
            if (ok && (r < 1 || c < 1 || r > F.m || c > F.n)) ok = false;
            if (!ok) {
                P.bad = (long long)(line - base);
                break;
            }
            P.r.push_back((int)(r - 1));
            P.c.push_back((int)(c - 1));
            P.v.push_back(v);
            while (p < end && *p != '\n') ++p;  // rest of the line
        }
    }
    long long total = 0;
    for (int t = 0; t < T; ++t) {
        const Part &P = parts[(size_t)t];
        if (P.bad >= 0) {
            set_error("%s: entry %lld malformed or out of range (byte %lld)", path,
                      total + (long long)P.r.size(), P.bad);
            return SBLAS_ERR_IO;
        }
        total += (long long)P.r.size();
    }
    if (total < nz) {
        set_error("%s: entry %lld malformed (file has %lld of %lld entries)", path, total, total, nz);
        return SBLAS_ERR_IO;
    }
    ri.resize((size_t)nz);
    ci.resize((size_t)nz);
    vi.resize((size_t)nz);
    long long off = 0;
    for (int t = 0; t < T && off < nz; ++t) {  // entries past nz are ignored, as fscanf does
        const Part &P = parts[(size_t)t];
        const size_t k = (size_t)std::min<long long>((long long)P.r.size(), nz - off);
        std::memcpy(&ri[(size_t)off], P.r.data(), k * sizeof(int));
        std::memcpy(&ci[(size_t)off], P.c.data(), k * sizeof(int));
        std::memcpy(&vi[(size_t)off], P.v.data(), k * sizeof(double));
        off += (long long)k;
    }
    return SBLAS_OK;
}

int mm_to_csr(const MMFile &F, int mode, const char *path, HostCsr &A)
{
    std::vector<int> ri, ci;
    std::vector<double> vi;
    const int st = parse_entries(F, mode, path, ri, ci, vi);
    if (st != SBLAS_OK) return st;
    const long long nz = F.nz;
    const bool expand = mode == 0 && F.sym;
    std::vector<long long> cnt((size_t)F.m + 1, 0);
    for (long long i = 0; i < nz; ++i) {
        cnt[(size_t)ri[(size_t)i] + 1]++;
        if (expand && ri[(size_t)i] != ci[(size_t)i]) cnt[(size_t)ci[(size_t)i] + 1]++;
    }
    for (int i = 0; i < F.m; ++i) cnt[(size_t)i + 1] += cnt[(size_t)i];
    A.m = F.m;
    A.n = F.n;
    A.nnz = cnt[(size_t)F.m];
    A.rowptr = cnt;
    if (mode == 1 || mode == 2) {
        // Q1: col/val keep FILE order; only the row counts build rowptr.
        A.col = std::move(ci);
        A.val = std::move(vi);
        return SBLAS_OK;
    }
    A.col.resize((size_t)A.nnz);
    A.val.resize((size_t)A.nnz);
    std::vector<long long> next(cnt.begin(), cnt.end() - 1);
    for (long long i = 0; i < nz; ++i) {  // stable scatter in file order
        const int r = ri[(size_t)i], c = ci[(size_t)i];
        long long o = next[(size_t)r]++;
        A.col[(size_t)o] = c;
        A.val[(size_t)o] = vi[(size_t)i];
        if (expand && r != c) {
            o = next[(size_t)c]++;
            A.col[(size_t)o] = r;
            A.val[(size_t)o] = vi[(size_t)i];
        }
    }
    return SBLAS_OK;
}

// SBLAS_MM_CACHE: "1" -> <file>.m<mode>.csrbin next to the file; any other
// non-empty value -> that directory.
std::string cache_path(const char *path, int mode)
{
    const char *env = std::getenv("SBLAS_MM_CACHE");
    if (!env || !*env || !std::strcmp(env, "0")) return std::string();
    std::string p = path;
    if (std::strcmp(env, "1") != 0) {
        const size_t sl = p.find_last_of('/');
        p = std::string(env) + "/" + (sl == std::string::npos ? p : p.substr(sl + 1));
    }
    return p + ".m" + std::to_string(mode) + ".csrbin";
}

int load_matrix(const char *path, int mode, HostCsr &A)
{
    const FileId id = file_id(path);
    const std::string cp = cache_path(path, mode);
    if (!cp.empty() && id.size >= 0 && csrbin_load(cp.c_str(), mode, id.size, id.mtime, A) == SBLAS_OK)
        return SBLAS_OK;
    MMFile F;
    if (!mm_open(path, F)) return SBLAS_ERR_IO;
    const int st = mm_to_csr(F, mode, path, A);
    if (st != SBLAS_OK) return st;
    if (!cp.empty())  // best effort: an unwritable cache directory is not an error
        (void)csrbin_store(cp.c_str(), mode, id.size, id.mtime, A.m, A.n, A.nnz, A.rowptr.data(),
                           A.col.data(), A.val.data());
    return SBLAS_OK;
}

}  // namespace
}  // namespace sblas

using namespace sblas;

extern "C" {

const char *sblas_last_error(void) { return sblas::last_error(); }

double sblas_get_time(void)
{
    struct timeval tp;
    gettimeofday(&tp, nullptr);
    return (double)tp.tv_sec + (double)tp.tv_usec * 1e-6;
}

int sblas_get_row_from_index(int n, long long *a, long long idx)
{
    return sblas::row_of_index(n, a, idx);
}

// mode 0: mmio_data (sptrsv_v1/src/mmio_highlevel.h:137-296)
// mode 1/2: test_spmv 'f'/'b' loader (spmv/test/dspmv_test.cu:101-136,217-251)
// mode 3: test_spmm loader (spmm/test/dspmm_baseline_test.cu:420-455), rows
//         bucketed stably (the row order sortbyrow then refines by column)
//
// the entries are parsed in parallel (OpenMP, one chunk of
// whole lines per thread, concatenated in file order, so the result is
// identical to a sequential parse), the two-call size/data protocol parses
// the file once (thread-local memo keyed by path, mode, size and mtime), and
// with SBLAS_MM_CACHE set the CSR is also kept in a binary .csrbin file that
// later loads read directly (see sblas_csrbin_write).
int sblas_mm_read(const char *path, int mode, int *m, int *n, long long *nnz,
                  long long *rowptr, int *col, double *val)
{
    if (!path || !m || !n || !nnz || mode < 0 || mode > 3) return SBLAS_ERR_INVALID;
    HostCsr *A = memo_lookup(path, mode);
    if (!A) {
        const int st = load_matrix(path, mode, memo_slot(path, mode));
        if (st != SBLAS_OK) {
            memo_clear();
            return st;
        }
        A = memo_lookup(path, mode);
    }
    *m = A->m;
    *n = A->n;
    *nnz = A->nnz;
    if (!rowptr) return SBLAS_OK;
    std::memcpy(rowptr, A->rowptr.data(), sizeof(long long) * ((size_t)A->m + 1));
    if (A->nnz) {
        std::memcpy(col, A->col.data(), sizeof(int) * (size_t)A->nnz);
        std::memcpy(val, A->val.data(), sizeof(double) * (size_t)A->nnz);
    }
    memo_clear();  // the data call ends the protocol
    return SBLAS_OK;
}

int sblas_csrbin_write(const char *path, int m, int n, long long nnz, const long long *rowptr,
                       const int *col, const double *val)
{
    if (!path || m < 0 || n < 0 || nnz < 0 || !rowptr || (nnz && (!col || !val)))
        return SBLAS_ERR_INVALID;
    return csrbin_store(path, -1, 0, 0, m, n, nnz, rowptr, col, val);
}

int sblas_csrbin_read(const char *path, int *m, int *n, long long *nnz, long long *rowptr,
                      int *col, double *val)
{
    if (!path || !m || !n || !nnz) return SBLAS_ERR_INVALID;
    HostCsr A;
    const int st = csrbin_load(path, -1, 0, 0, A);
    if (st != SBLAS_OK) return st;
    *m = A.m;
    *n = A.n;
    *nnz = A.nnz;
    if (!rowptr) return SBLAS_OK;
    std::memcpy(rowptr, A.rowptr.data(), sizeof(long long) * ((size_t)A.m + 1));
    if (A.nnz) {
        std::memcpy(col, A.col.data(), sizeof(int) * (size_t)A.nnz);
        std::memcpy(val, A.val.data(), sizeof(double) * (size_t)A.nnz);
    }
    return SBLAS_OK;
}

int sblas_partition_rowblock(int m, int g, int *row_start)
{
    if (g <= 0 || m < 0 || !row_start) return SBLAS_ERR_INVALID;
    for (int d = 0; d <= g; ++d) row_start[d] = (int)((long long)d * m / g);
    return SBLAS_OK;
}

// dspmv_mgpu_v1.cu:60-94 with Q5 fixed: start_row = last row whose first
// element is <= start_idx (so empty rows are never orphaned), rows between two
// partitions belong to the earlier one, partition 0 starts at row 0 and the
// last ends at m-1.
int sblas_partition_nnz(int m, long long nnz, const long long *rowptr, int g,
                        long long *start_idx, long long *end_idx, int *start_row,
                        int *end_row, int *start_flag)
{
    if (g <= 0 || m < 0 || nnz < 0 || !rowptr) return SBLAS_ERR_INVALID;
    for (int d = 0; d < g; ++d) {
        start_idx[d] = (long long)d * nnz / g;
        end_idx[d] = (long long)(d + 1) * nnz / g - 1;
    }
    for (int d = 0; d < g; ++d) {
        if (d == 0) {
            start_row[d] = 0;
            start_flag[d] = 0;
        } else if (start_idx[d] >= nnz) {
            start_row[d] = m;
            start_flag[d] = 0;
        } else {
            start_row[d] = row_of_index(m, rowptr, start_idx[d]);
            start_flag[d] = start_idx[d] > rowptr[start_row[d]] ? 1 : 0;
        }
    }
    for (int d = 0; d < g; ++d) {
        end_row[d] = (d == g - 1) ? m - 1
                   : (start_flag[d + 1] ? start_row[d + 1] : start_row[d + 1] - 1);
        if (end_row[d] < start_row[d] - 1) end_row[d] = start_row[d] - 1;
    }
    return SBLAS_OK;
}

// Cost-weighted row split: contiguous WHOLE-row ranges
// whose cost sum_r (nnz_r + w) is balanced, so a rank of short rows gets
// fewer entries than one of long rows (a row-end costs a segmented-sum kernel
// about w entries' time).  Same outputs as sblas_partition_nnz with every
// start_flag 0 (no row is split, no carries); an empty range has end_row =
// start_row - 1 and end_idx = start_idx - 1.
int sblas_partition_cost(int m, const long long *rowptr, int g, double w, long long *start_idx,
                         long long *end_idx, int *start_row, int *end_row, int *start_flag)
{
    if (g <= 0 || m < 0 || !rowptr || !(w >= 0.0)) return SBLAS_ERR_INVALID;
    auto cost = [&](long long r) { return (double)rowptr[r] + w * (double)r; };
    const double total = cost(m);
    for (int d = 0; d < g; ++d) {
        int r0 = 0;
        if (d > 0) {  // first row whose cost prefix reaches d/g of the total
            const double target = total * d / g;
            long long lo = 0, hi = m;
            while (lo < hi) {
                const long long mid = (lo + hi) / 2;
                if (cost(mid) >= target) hi = mid;
                else lo = mid + 1;
            }
            r0 = (int)std::max<long long>(lo, start_row[d - 1]);
        }
        start_row[d] = r0;
        start_flag[d] = 0;
    }
    for (int d = 0; d < g; ++d) {
        end_row[d] = d == g - 1 ? m - 1 : start_row[d + 1] - 1;
        start_idx[d] = rowptr[start_row[d]];
        end_idx[d] = rowptr[end_row[d] + 1] - 1;
    }
    return SBLAS_OK;
}

// ---------------------------------------------------------------------------
// Synthetic generator (DESIGN.md "Synthetic"): per-row SplitMix64 stream
// started at stream_state(seed, row); columns by 128-bit multiply-high into
// [0,n), redrawn on duplicates, sorted; then one U[0,1) value per sorted
// column.
// ---------------------------------------------------------------------------
static inline unsigned long long mix64(unsigned long long z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline unsigned long long splitmix(unsigned long long &s) { return mix64(s += 0x9E3779B97F4A7C15ULL); }
// Start of row (or column) i's stream.  Rounds 1-4 used seed ^ (i+1)*golden:
// row i+1's start then often equalled row i's state after one draw (the xor
// with a small seed commutes with the +golden step unless it meets a carry),
// so ~1 pair in 8 of consecutive rows shared all but one column and runs of
// rows repeated one column set (config 2's first 20k heavy rows: 8% distinct
// columns instead of 64%; round 5, profiles/r05/gen/).  Hashing the index
// and the seed puts every stream at an independent point of the sequence.
static inline unsigned long long stream_state(unsigned long long seed, unsigned long long i)
{
    return mix64(seed ^ mix64((i + 1) * 0x9E3779B97F4A7C15ULL));
}
static inline double to_u01(unsigned long long r) { return (double)(r >> 11) * 0x1.0p-53; }

int sblas_gen_synth_rowptr(int n, int heavy, int light, long long *rowptr)
{
    if (n < 0 || heavy < 0 || light < 0 || !rowptr) return SBLAS_ERR_INVALID;
    const int nh = n / 8;
    rowptr[0] = 0;
    for (int i = 0; i < n; ++i) rowptr[i + 1] = rowptr[i] + (i < nh ? heavy : light);
    return SBLAS_OK;
}

int sblas_gen_synth_rows(int n, int heavy, int light, int prefix_cols,
                         unsigned long long seed, const long long *rowptr,
                         int row_begin, int row_end, int *col, double *val)
{
    (void)heavy;
    (void)light;
    if (row_begin < 0 || row_end > n || row_begin > row_end || !rowptr) return SBLAS_ERR_INVALID;
    const long long base = rowptr[row_begin];
#pragma omp parallel for schedule(dynamic, 1024)
    for (int i = row_begin; i < row_end; ++i) {
        const long long b = rowptr[i] - base;
        const int d = (int)(rowptr[i + 1] - rowptr[i]);
        unsigned long long s = stream_state(seed, (unsigned long long)i);
        int *c = col + b;
        if (prefix_cols) {
            for (int k = 0; k < d; ++k) c[k] = k;
        } else {
            for (int k = 0; k < d; ++k) {
                for (;;) {
                    const unsigned long long r = splitmix(s);
                    const int v = (int)(((unsigned __int128)r * (unsigned)n) >> 64);
                    bool dup = false;
                    for (int t = 0; t < k; ++t)
                        if (c[t] == v) {
                            dup = true;
                            break;
                        }
                    if (!dup) {
                        c[k] = v;
                        break;
                    }
                }
            }
            std::sort(c, c + d);
        }
        for (int k = 0; k < d; ++k) val[b + k] = to_u01(splitmix(s));
    }
    return SBLAS_OK;
}

// Unit-lower-triangular CSC stand-in for circuit5M-class SpTRSV (SURVEY
// M1-cfg5): column j holds its unit diagonal first, then `offd` distinct rows
// drawn uniformly from (j, min(n-1, j+band)] (fewer near the end), sorted.
// Off-diagonal value = (1 + r%10) / (20 * row_len(i)), r from the column's
// SplitMix64 stream, so every row's off-diagonal sum stays <= 0.5 and the
// forward solve is well conditioned.  Two calls: colptr only (rowidx NULL),
// then the full arrays.
int sblas_gen_lower_banded(int n, int offd, int band, unsigned long long seed, int *colptr,
                           int *rowidx, double *val)
{
    if (n < 0 || offd < 0 || band < 1 || !colptr) return SBLAS_ERR_INVALID;
    colptr[0] = 0;
    for (int j = 0; j < n; ++j) {
        const long long room = std::min<long long>((long long)n - 1 - j, band);
        colptr[j + 1] = colptr[j] + 1 + (int)std::min<long long>(offd, room);
    }
    if (!rowidx) return SBLAS_OK;
    std::vector<int> rowlen((size_t)n, 1);
    std::vector<unsigned char> draw((size_t)colptr[n]);
#pragma omp parallel for schedule(dynamic, 4096)
    for (int j = 0; j < n; ++j) {
        unsigned long long st = stream_state(seed, (unsigned long long)j);
        const int a = colptr[j], b = colptr[j + 1];
        rowidx[a] = j;
        const long long room = std::min<long long>((long long)n - 1 - j, band);
        for (int k = a + 1; k < b; ++k) {
            for (;;) {
                const unsigned long long r = splitmix(st);
                const int v = j + 1 + (int)(((unsigned __int128)r * (unsigned long long)room) >> 64);
                bool dup = false;
                for (int t = a + 1; t < k; ++t)
                    if (rowidx[t] == v) {
                        dup = true;
                        break;
                    }
                if (!dup) {
                    rowidx[k] = v;
                    break;
                }
            }
        }
        std::sort(rowidx + a + 1, rowidx + b);
        for (int k = a + 1; k < b; ++k) draw[(size_t)k] = (unsigned char)(splitmix(st) % 10);
    }
    for (int j = 0; j < n; ++j)
        for (int k = colptr[j] + 1; k < colptr[j + 1]; ++k) rowlen[(size_t)rowidx[k]]++;
#pragma omp parallel for schedule(static)
    for (int j = 0; j < n; ++j) {
        val[colptr[j]] = 1.0;
        for (int k = colptr[j] + 1; k < colptr[j + 1]; ++k)
            val[k] = (1.0 + draw[(size_t)k]) / (20.0 * rowlen[(size_t)rowidx[k]]);
    }
    return SBLAS_OK;
}

// 3-D stencil matrix on an nx x ny x nz grid, natural ordering (row r =
// (k*ny + j)*nx + i): the structured, banded kind of SuiteSparse matrix
// (FEM / finite-difference Laplacians).  points = 7 (faces) or 27 (the full
// 3x3x3 box).  Off-diagonal a_rc = -U[0,1) from a per-entry hash of (seed,
// r, c); the diagonal is 1 + sum |off|, so the matrix is diagonally dominant.
// Columns ascend within a row.  col == NULL: rowptr only.
int sblas_gen_stencil3d(int nx, int ny, int nz, int points, unsigned long long seed, long long *rowptr, int *col,
                        double *val)
{
    if (nx < 1 || ny < 1 || nz < 1 || (points != 7 && points != 27) || !rowptr) return SBLAS_ERR_INVALID;
    const long long n = (long long)nx * ny * nz;
    if (n > 0x7fffffffLL) return SBLAS_ERR_INVALID;
    auto inside = [&](int i, int j, int k) { return i >= 0 && i < nx && j >= 0 && j < ny && k >= 0 && k < nz; };
    auto is_pt = [&](int di, int dj, int dk) {
        return points == 27 || (std::abs(di) + std::abs(dj) + std::abs(dk) <= 1);
    };
    rowptr[0] = 0;
    std::vector<int> len((size_t)n);
#pragma omp parallel for schedule(static)
    for (long long r = 0; r < n; ++r) {
        const int i = (int)(r % nx), j = (int)((r / nx) % ny), k = (int)(r / ((long long)nx * ny));
        int c = 0;
        for (int dk = -1; dk <= 1; ++dk)
            for (int dj = -1; dj <= 1; ++dj)
                for (int di = -1; di <= 1; ++di)
                    c += is_pt(di, dj, dk) && inside(i + di, j + dj, k + dk);
        len[(size_t)r] = c;
    }
    for (long long r = 0; r < n; ++r) rowptr[r + 1] = rowptr[r] + len[(size_t)r];
    if (!col) return SBLAS_OK;
    if (!val) return SBLAS_ERR_INVALID;
#pragma omp parallel for schedule(static)
    for (long long r = 0; r < n; ++r) {
        const int i = (int)(r % nx), j = (int)((r / nx) % ny), k = (int)(r / ((long long)nx * ny));
        long long e = rowptr[r], de = -1;
        double off = 0.0;
        for (int dk = -1; dk <= 1; ++dk)
            for (int dj = -1; dj <= 1; ++dj)
                for (int di = -1; di <= 1; ++di) {
                    if (!is_pt(di, dj, dk) || !inside(i + di, j + dj, k + dk)) continue;
                    const long long c = r + ((long long)dk * ny + dj) * nx + di;
                    col[e] = (int)c;
                    if (c == r) {
                        de = e;
                    } else {
                        unsigned long long h = seed ^ ((unsigned long long)r * 0x9E3779B97F4A7C15ULL) ^
                                               ((unsigned long long)c * 0xC2B2AE3D27D4EB4FULL);
                        val[e] = -to_u01(splitmix(h));
                        off -= val[e];
                    }
                    ++e;
                }
        val[de] = 1.0 + off;
    }
    return SBLAS_OK;
}

// R-MAT power-law graph (Graph500 generator parameters a, b, c = 0.57, 0.19,
// 0.19, no per-level noise) with 2^scale vertices and edge_factor * 2^scale
// edge draws: each draw descends `scale` quadrant levels from its own hashed
// stream, vertex labels are then permuted (seeded Fisher-Yates) so the heavy
// rows spread over the matrix, duplicate (row, col) draws are merged (values
// summed) and columns ascend within a row.  Values U[0,1).  rowptr: 2^scale + 1
// int64 entries; col/val hold cap entries (edge_factor * 2^scale always
// suffices); the nonzero count is rowptr[2^scale].
int sblas_gen_rmat(int scale, int edge_factor, unsigned long long seed, long long *rowptr, int *col, double *val,
                   long long cap)
{
    if (scale < 1 || scale > 30 || edge_factor < 1 || !rowptr || !col || !val) return SBLAS_ERR_INVALID;
    const long long n = 1LL << scale, E = (long long)edge_factor * n;
    if (cap < E) return SBLAS_ERR_INVALID;
    std::vector<int> perm((size_t)n);
    for (long long v = 0; v < n; ++v) perm[(size_t)v] = (int)v;
    {
        unsigned long long st = seed ^ 0xA5A5A5A5DEADBEEFULL;
        for (long long v = n - 1; v > 0; --v) {
            const long long w = (long long)(((unsigned __int128)splitmix(st) * (unsigned long long)(v + 1)) >> 64);
            std::swap(perm[(size_t)v], perm[(size_t)w]);
        }
    }
    std::vector<int> er((size_t)E), ec((size_t)E);
    std::vector<double> ev((size_t)E);
#pragma omp parallel for schedule(static)
    for (long long e = 0; e < E; ++e) {
        unsigned long long st = stream_state(seed, (unsigned long long)e);
        long long r = 0, c = 0;
        for (int l = 0; l < scale; ++l) {
            const double u = to_u01(splitmix(st));
            const int rb = u >= 0.57 + 0.19, cb = (u >= 0.57 && u < 0.57 + 0.19) || u >= 0.57 + 0.19 + 0.19;
            r = (r << 1) | rb;
            c = (c << 1) | cb;
        }
        er[(size_t)e] = perm[(size_t)r];
        ec[(size_t)e] = perm[(size_t)c];
        ev[(size_t)e] = to_u01(splitmix(st));
    }
    // bucket the draws by row (stable in draw order), then sort + merge per row
    std::vector<long long> cnt((size_t)n + 1, 0);
    for (long long e = 0; e < E; ++e) ++cnt[(size_t)er[(size_t)e] + 1];
    for (long long v = 0; v < n; ++v) cnt[(size_t)v + 1] += cnt[(size_t)v];
    std::vector<long long> pos(cnt.begin(), cnt.end() - 1);
    std::vector<std::pair<int, double>> tmp((size_t)E);
    for (long long e = 0; e < E; ++e) tmp[(size_t)pos[(size_t)er[(size_t)e]]++] = {ec[(size_t)e], ev[(size_t)e]};
    std::vector<int> rl((size_t)n);
#pragma omp parallel for schedule(dynamic, 1024)
    for (long long v = 0; v < n; ++v) {
        auto b = tmp.begin() + cnt[(size_t)v], en = tmp.begin() + cnt[(size_t)v + 1];
        std::stable_sort(b, en, [](const std::pair<int, double> &x, const std::pair<int, double> &y) {
            return x.first < y.first;
        });
        long long w = cnt[(size_t)v];
        for (auto it = b; it != en; ++it) {
            if (w > cnt[(size_t)v] && tmp[(size_t)w - 1].first == it->first) tmp[(size_t)w - 1].second += it->second;
            else tmp[(size_t)w++] = *it;
        }
        rl[(size_t)v] = (int)(w - cnt[(size_t)v]);
    }
    rowptr[0] = 0;
    for (long long v = 0; v < n; ++v) rowptr[v + 1] = rowptr[v] + rl[(size_t)v];
#pragma omp parallel for schedule(dynamic, 1024)
    for (long long v = 0; v < n; ++v)
        for (int k = 0; k < rl[(size_t)v]; ++k) {
            col[rowptr[v] + k] = tmp[(size_t)cnt[(size_t)v] + k].first;
            val[rowptr[v] + k] = tmp[(size_t)cnt[(size_t)v] + k].second;
        }
    return SBLAS_OK;
}

int sblas_gen_vector(int n, unsigned long long seed, double *v)
{
    if (n < 0 || !v) return SBLAS_ERR_INVALID;
    unsigned long long s = seed;
    for (int i = 0; i < n; ++i) v[i] = to_u01(splitmix(s));
    return SBLAS_OK;
}

// sortbyrow + CSR build of test_spmm (spmm/test/dspmm_baseline_test.cu:41-55,
// 461-493): COO sorted by (row, col) in place, rowptr[m+1] from row counts.
// The reference's qsort is unstable, so it leaves the order of duplicate
// (row, col) entries unspecified; here it is their input order (stable
// counting sort by row, then a stable sort by column inside each row).
// Rows outside [0, m) are rejected.
int sblas_coo_sortbyrow(int m, long long nnz, int *row, int *col, double *val, int *rowptr)
{
    if (m < 0 || nnz < 0 || (nnz && (!row || !col || !val)) || !rowptr) return SBLAS_ERR_INVALID;
    if (nnz >= (1LL << 31)) return SBLAS_ERR_UNSUPPORTED;
    std::vector<long long> start((size_t)m + 1, 0);
    for (long long i = 0; i < nnz; ++i) {
        if (row[i] < 0 || row[i] >= m) return SBLAS_ERR_INVALID;
        start[(size_t)row[i] + 1]++;
    }
    for (int r = 0; r < m; ++r) start[(size_t)r + 1] += start[(size_t)r];
    std::vector<int> c2((size_t)nnz);
    std::vector<double> v2((size_t)nnz);
    {
        std::vector<long long> pos(start.begin(), start.end() - 1);
        for (long long i = 0; i < nnz; ++i) {
            const long long p = pos[(size_t)row[i]]++;
            c2[(size_t)p] = col[i];
            v2[(size_t)p] = val[i];
        }
    }
#pragma omp parallel
    {
        std::vector<std::pair<int, double>> t;
#pragma omp for schedule(dynamic, 256)
        for (int r = 0; r < m; ++r) {
            const long long a = start[(size_t)r], b = start[(size_t)r + 1];
            t.resize((size_t)(b - a));
            for (long long k = a; k < b; ++k) t[(size_t)(k - a)] = {c2[(size_t)k], v2[(size_t)k]};
            std::stable_sort(t.begin(), t.end(),
                             [](const std::pair<int, double> &u, const std::pair<int, double> &v) {
                                 return u.first < v.first;
                             });
            for (long long k = a; k < b; ++k) {
                row[k] = r;
                col[k] = t[(size_t)(k - a)].first;
                val[k] = t[(size_t)(k - a)].second;
            }
        }
    }
    for (int r = 0; r <= m; ++r) rowptr[r] = (int)start[(size_t)r];
    return SBLAS_OK;
}

}  // extern "C"
