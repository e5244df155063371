// host_utils.cpp -- host-side pieces of libsblas that need no GPU:
// Matrix-Market reader, partitions, synthetic generators, timers.
//
// Semantics follow the reference (cited per function); the implementation is
// our own: the MM reader slurps the file once and parses in place (the
// reference fscanf's entry by entry, dspmv_test.cu:122-136), and the
// generator is row-parallel (one counter-based stream per row).
#include <sys/time.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdarg>
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
int sblas_mm_read(const char *path, int mode, int *m, int *n, long long *nnz,
                  long long *rowptr, int *col, double *val)
{
    MMFile F;
    if (!path || !m || !n || !nnz || mode < 0 || mode > 2) return SBLAS_ERR_INVALID;
    if (!mm_open(path, F)) return SBLAS_ERR_IO;
    const long long nz = F.nz;
    std::vector<int> ri((size_t)nz), ci((size_t)nz);
    std::vector<double> vi((size_t)nz);
    const char *p = F.buf.c_str() + F.pos;
    for (long long i = 0; i < nz; ++i) {
        long long r, c;
        double v = 0.0;
        if (!(p = parse_int(p, r)) || !(p = parse_int(p, c))) {
            set_error("%s: entry %lld malformed", path, i);
            return SBLAS_ERR_IO;
        }
        if (mode == 0) {
            if (F.real || F.complex_) {
                if (!(p = parse_dbl(p, v))) return SBLAS_ERR_IO;
                if (F.complex_) {
                    double im;
                    if (!(p = parse_dbl(p, im))) return SBLAS_ERR_IO;
                }
            } else if (F.integer) {
                long long iv;
                if (!(p = parse_int(p, iv))) return SBLAS_ERR_IO;
                v = (double)iv;
            } else {
                v = 1.0;
            }
        } else if (mode == 1) {
            if (!(p = parse_dbl(p, v))) return SBLAS_ERR_IO;
        } else {
            v = 0.00001;
        }
        if (r < 1 || c < 1 || r > F.m || c > F.n) {
            set_error("%s: entry %lld (%lld,%lld) out of range", path, i, r, c);
            return SBLAS_ERR_IO;
        }
        ri[(size_t)i] = (int)(r - 1);
        ci[(size_t)i] = (int)(c - 1);
        vi[(size_t)i] = v;
        if (mode == 0) {
            // skip the rest of the line (mmio_data reads exactly its fields)
        }
    }
    const bool expand = mode == 0 && F.sym;
    std::vector<long long> cnt((size_t)F.m + 1, 0);
    for (long long i = 0; i < nz; ++i) {
        cnt[(size_t)ri[(size_t)i] + 1]++;
        if (expand && ri[(size_t)i] != ci[(size_t)i]) cnt[(size_t)ci[(size_t)i] + 1]++;
    }
    for (int i = 0; i < F.m; ++i) cnt[(size_t)i + 1] += cnt[(size_t)i];
    *m = F.m;
    *n = F.n;
    *nnz = cnt[(size_t)F.m];
    if (!rowptr) return SBLAS_OK;
    std::memcpy(rowptr, cnt.data(), sizeof(long long) * ((size_t)F.m + 1));
    if (mode != 0) {
        // Q1: col/val keep FILE order; only the row counts build rowptr.
        std::memcpy(col, ci.data(), sizeof(int) * (size_t)nz);
        std::memcpy(val, vi.data(), sizeof(double) * (size_t)nz);
        return SBLAS_OK;
    }
    std::vector<long long> next(cnt.begin(), cnt.end() - 1);
    for (long long i = 0; i < nz; ++i) {
        const int r = ri[(size_t)i], c = ci[(size_t)i];
        long long o = next[(size_t)r]++;
        col[o] = c;
        val[o] = vi[(size_t)i];
        if (expand && r != c) {
            o = next[(size_t)c]++;
            col[o] = r;
            val[o] = vi[(size_t)i];
        }
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

// ---------------------------------------------------------------------------
// Synthetic generator (DESIGN.md "Synthetic"): per-row SplitMix64 stream,
// state = seed ^ (row+1)*0x9E3779B97F4A7C15; columns by 128-bit
// multiply-high into [0,n), redrawn on duplicates, sorted; then one U[0,1)
// value per sorted column.
// ---------------------------------------------------------------------------
static inline unsigned long long splitmix(unsigned long long &s)
{
    unsigned long long z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
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
        unsigned long long s = seed ^ ((unsigned long long)(i + 1) * 0x9E3779B97F4A7C15ULL);
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
        unsigned long long st = seed ^ ((unsigned long long)(j + 1) * 0x9E3779B97F4A7C15ULL);
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

int sblas_gen_vector(int n, unsigned long long seed, double *v)
{
    if (n < 0 || !v) return SBLAS_ERR_INVALID;
    unsigned long long s = seed;
    for (int i = 0; i < n; ++i) v[i] = to_u01(splitmix(s));
    return SBLAS_OK;
}

}  // extern "C"
