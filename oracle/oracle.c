/*
 * oracle.c -- CPU restatement of pnnl/s-blas's hot-path algorithms.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Written from the reference's
 * behaviour, not copied: every function names the reference lines it follows.
 */
#include "oracle.h"

#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
void orc_ref_alpha_beta(long long skip, double *alpha, double *beta)
{
    srand(1); /* glibc's default state == srand(1) */
    for (long long i = 0; i < skip; ++i) (void)rand();
    *alpha = (double)rand() / (RAND_MAX);
    *beta = (double)rand() / (RAND_MAX);
}

/* ------------------------------------------------------------------------ */
/* Matrix-Market header: banner (mmio.h:254 mm_read_banner), comment lines,
 * size line (mmio.h:339 mm_read_mtx_crd_size). */
static int lower_eq(const char *a, const char *b)
{
    for (; *a && *b; ++a, ++b)
        if (tolower((unsigned char)*a) != tolower((unsigned char)*b)) return 0;
    return *a == 0 && *b == 0;
}

static FILE *mm_open_header(const char *path, int *m, int *n, long long *nz,
                            int *flags)
{
    FILE *f = fopen(path, "r");
    if (!f) return NULL;
    char line[1100], banner[64], obj[64], fmt[64], field[64], sym[64];
    if (!fgets(line, sizeof line, f) ||
        sscanf(line, "%63s %63s %63s %63s %63s", banner, obj, fmt, field, sym) != 5 ||
        strcmp(banner, "%%MatrixMarket") != 0 || !lower_eq(obj, "matrix") ||
        !lower_eq(fmt, "coordinate")) {
        fclose(f);
        return NULL;
    }
    int fl = 0;
    if (lower_eq(field, "pattern")) fl |= 1;
    else if (lower_eq(field, "real")) fl |= 2;
    else if (lower_eq(field, "complex")) fl |= 4;
    else if (lower_eq(field, "integer")) fl |= 8;
    if (lower_eq(sym, "symmetric") || lower_eq(sym, "hermitian")) fl |= 16;
    do {
        if (!fgets(line, sizeof line, f)) { fclose(f); return NULL; }
    } while (line[0] == '%');
    long long a, b, c;
    if (sscanf(line, "%lld %lld %lld", &a, &b, &c) != 3) { fclose(f); return NULL; }
    *m = (int)a; *n = (int)b; *nz = c; *flags = fl;
    return f;
}

int orc_mm_info(const char *path, int *m, int *n, long long *nnz_file, int *flags)
{
    FILE *f = mm_open_header(path, m, n, nnz_file, flags);
    if (!f) return -1;
    fclose(f);
    return 0;
}

/* dspmv_test.cu:101-136 + :217-251.  The reference reads every entry with
 * "%d %d %lg" ('f') or "%d %d" ('b' -> 1e-5) whatever the banner says, keeps
 * col/val in file order and only counts rows into rowptr. */
int orc_mm_load_testspmv(const char *path, char data_type, long long *rowptr,
                         int *col, double *val)
{
    int m, n, fl;
    long long nz;
    FILE *f = mm_open_header(path, &m, &n, &nz, &fl);
    if (!f) return -1;
    int *row = (int *)malloc(sizeof(int) * (size_t)(nz > 0 ? nz : 1));
    for (long long i = 0; i < nz; ++i) {
        int r = 0, c = 0;
        double v = 0.0;
        if (data_type == 'b') {
            if (fscanf(f, "%d %d\n", &r, &c) != 2) { free(row); fclose(f); return -2; }
            v = 0.00001;
        } else {
            if (fscanf(f, "%d %d %lg\n", &r, &c, &v) != 3) { free(row); fclose(f); return -2; }
        }
        row[i] = r - 1;
        col[i] = c - 1;
        val[i] = v;
    }
    fclose(f);
    for (int i = 0; i <= m; ++i) rowptr[i] = 0;
    for (long long i = 0; i < nz; ++i) rowptr[row[i] + 1]++;
    for (int i = 0; i < m; ++i) rowptr[i + 1] += rowptr[i];
    free(row);
    return 0;
}

/* mmio_highlevel.h:137-296 (mmio_data).  Counting pass (with symmetric
 * mirror), exclusive scan, then in file order each entry is appended to its
 * row (and, if symmetric and off-diagonal, the mirror to the column's row). */
int orc_mm_load_mmio(const char *path, int *m_out, int *n_out, int *nnz_out,
                     int *is_sym, int *rowptr, int *col, double *val)
{
    int m, n, fl;
    long long nz;
    FILE *f = mm_open_header(path, &m, &n, &nz, &fl);
    if (!f) return -1;
    int *ri = (int *)malloc(sizeof(int) * (size_t)(nz ? nz : 1));
    int *ci = (int *)malloc(sizeof(int) * (size_t)(nz ? nz : 1));
    double *vi = (double *)malloc(sizeof(double) * (size_t)(nz ? nz : 1));
    int *cnt = (int *)calloc((size_t)m + 1, sizeof(int));
    for (long long i = 0; i < nz; ++i) {
        int r = 0, c = 0, iv = 0;
        double v = 0.0, vim = 0.0;
        int ok;
        if (fl & 2) ok = fscanf(f, "%d %d %lg\n", &r, &c, &v) == 3;
        else if (fl & 4) ok = fscanf(f, "%d %d %lg %lg\n", &r, &c, &v, &vim) == 4;
        else if (fl & 8) { ok = fscanf(f, "%d %d %d\n", &r, &c, &iv) == 3; v = iv; }
        else { ok = fscanf(f, "%d %d\n", &r, &c) == 2; v = 1.0; }
        if (!ok) { free(ri); free(ci); free(vi); free(cnt); fclose(f); return -2; }
        ri[i] = r - 1; ci[i] = c - 1; vi[i] = v;
        cnt[ri[i]]++;
    }
    fclose(f);
    int sym = (fl & 16) != 0;
    if (sym)
        for (long long i = 0; i < nz; ++i)
            if (ri[i] != ci[i]) cnt[ci[i]]++;
    /* exclusive scan into rowptr-shaped array */
    int *ptr = (int *)malloc(sizeof(int) * ((size_t)m + 1));
    ptr[0] = 0;
    for (int i = 0; i < m; ++i) ptr[i + 1] = ptr[i] + cnt[i];
    *m_out = m; *n_out = n; *nnz_out = ptr[m]; *is_sym = sym;
    if (rowptr) {
        memcpy(rowptr, ptr, sizeof(int) * ((size_t)m + 1));
        memset(cnt, 0, sizeof(int) * ((size_t)m + 1));
        for (long long i = 0; i < nz; ++i) {
            int r = ri[i], c = ci[i];
            int o = ptr[r] + cnt[r]++;
            col[o] = c; val[o] = vi[i];
            if (sym && r != c) {
                o = ptr[c] + cnt[c]++;
                col[o] = r; val[o] = vi[i];
            }
        }
    }
    free(ptr); free(ri); free(ci); free(vi); free(cnt);
    return 0;
}

/* ------------------------------------------------------------------------ */
void orc_csr_spmv(int m, const long long *rowptr, const int *col,
                  const double *val, const double *x, double alpha, double beta,
                  double *y)
{
    for (int i = 0; i < m; ++i) {
        double s = 0.0;
        for (long long j = rowptr[i]; j < rowptr[i + 1]; ++j) s += val[j] * x[col[j]];
        y[i] = (beta == 0.0) ? alpha * s : alpha * s + beta * y[i];
    }
}

void orc_csr_spmv_omp(int m, const long long *rowptr, const int *col,
                      const double *val, const double *x, double alpha,
                      double beta, double *y, int nthreads)
{
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4096)
#endif
    for (int i = 0; i < m; ++i) {
        double s = 0.0;
        for (long long j = rowptr[i]; j < rowptr[i + 1]; ++j) s += val[j] * x[col[j]];
        y[i] = (beta == 0.0) ? alpha * s : alpha * s + beta * y[i];
    }
}

void orc_spmv_bound(int m, const long long *rowptr, const int *col, const double *val,
                    const double *x, double alpha, double beta, const double *y0,
                    double *bound)
{
    const double u = 0x1p-53;
#pragma omp parallel for schedule(dynamic, 4096)
    for (int i = 0; i < m; ++i) {
        double s = 0.0;
        for (long long j = rowptr[i]; j < rowptr[i + 1]; ++j) s += fabs(alpha * val[j] * x[col[j]]);
        const double k = (double)(rowptr[i + 1] - rowptr[i]);
        const double gam = k * u / (1.0 - k * u);
        bound[i] = 4.0 * gam * s + 4.0 * u * fabs(beta * y0[i]) + 1e-300;
    }
}

int orc_get_row_from_index_ref(int n, const long long *a, long long idx)
{
    /* spmv_helper.cu:16-39: bisection that returns on the first equal key */
    int l = 0, r = n;
    while (l < r - 1) {
        int mid = l + (r - l) / 2;
        if (idx < a[mid]) r = mid;
        else if (idx > a[mid]) l = mid;
        else return mid;
    }
    if (idx == a[l]) return l;
    if (idx == a[r]) return r;
    return l;
}

int orc_row_of_index(int m, const long long *rowptr, long long idx)
{
    int lo = 0, hi = m; /* find last r in [0,m] with rowptr[r] <= idx */
    while (lo < hi) {
        int mid = lo + (hi - lo + 1) / 2;
        if (rowptr[mid] <= idx) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

void orc_partition_rowblock(int m, int g, int *row_start)
{
    for (int d = 0; d <= g; ++d) row_start[d] = (int)((long long)d * m / g);
}

void orc_partition_nnz(int m, long long nnz, const long long *rowptr, int g,
                       long long *start_idx, long long *end_idx, int *start_row,
                       int *end_row, int *start_flag)
{
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
            start_row[d] = orc_row_of_index(m, rowptr, start_idx[d]);
            start_flag[d] = start_idx[d] > rowptr[start_row[d]];
        }
    }
    for (int d = 0; d < g; ++d) {
        if (d == g - 1) end_row[d] = m - 1;
        else end_row[d] = start_flag[d + 1] ? start_row[d + 1] : start_row[d + 1] - 1;
        if (end_row[d] < start_row[d] - 1) end_row[d] = start_row[d] - 1;
    }
}

static void local_csrmv(int dev_m, const int *lptr, const int *col,
                        const double *val, const double *x, double alpha,
                        double beta, double *y)
{
    for (int i = 0; i < dev_m; ++i) {
        double s = 0.0;
        for (int j = lptr[i]; j < lptr[i + 1]; ++j) s += val[j] * x[col[j]];
        y[i] = (beta == 0.0) ? alpha * s : alpha * s + beta * y[i];
    }
}

void orc_spmv_mgpu_v1(int m, int n, long long nnz, double alpha,
                      const double *val, const long long *rowptr,
                      const int *col, const double *x, double beta, double *y,
                      int g)
{
    (void)n;
    long long *si = (long long *)malloc(sizeof(long long) * g);
    long long *ei = (long long *)malloc(sizeof(long long) * g);
    int *sr = (int *)malloc(sizeof(int) * g), *er = (int *)malloc(sizeof(int) * g);
    int *sf = (int *)malloc(sizeof(int) * g);
    double *y0 = (double *)malloc(sizeof(double) * g);
    orc_partition_nnz(m, nnz, rowptr, g, si, ei, sr, er, sf);
    for (int d = 0; d < g; ++d) y0[d] = (sf[d] && sr[d] < m) ? y[sr[d]] : 0.0;
    double **part = (double **)malloc(sizeof(double *) * g);
    for (int d = 0; d < g; ++d) {
        int dm = er[d] - sr[d] + 1;
        int dn = (int)(ei[d] - si[d] + 1);
        part[d] = (double *)malloc(sizeof(double) * (dm > 0 ? dm : 1));
        if (dm <= 0) continue;
        int *lp = (int *)malloc(sizeof(int) * (dm + 1));
        lp[0] = 0;
        lp[dm] = dn;
        for (int j = 1; j < dm; ++j) lp[j] = (int)(rowptr[sr[d] + j] - si[d]);
        memcpy(part[d], y + sr[d], sizeof(double) * dm); /* H2D of y slice */
        local_csrmv(dm, lp, col + si[d], val + si[d], x, alpha, beta, part[d]);
        free(lp);
    }
    /* host fix-up in device order (dspmv_mgpu_v1.cu:235-248) */
    for (int d = 0; d < g; ++d) {
        int dm = er[d] - sr[d] + 1;
        if (dm <= 0) continue;
        double tmp = sf[d] ? y[sr[d]] : 0.0;
        memcpy(y + sr[d], part[d], sizeof(double) * dm);
        if (sf[d]) {
            y[sr[d]] += tmp;
            y[sr[d]] -= y0[d] * beta;
        }
    }
    for (int d = 0; d < g; ++d) free(part[d]);
    free(part); free(si); free(ei); free(sr); free(er); free(sf); free(y0);
}

void orc_spmv_mgpu_baseline(int m, int n, long long nnz, double alpha,
                            const double *val, const long long *rowptr,
                            const int *col, const double *x, double beta,
                            double *y, int g)
{
    (void)n; (void)nnz;
    int *rs = (int *)malloc(sizeof(int) * (g + 1));
    orc_partition_rowblock(m, g, rs);
    for (int d = 0; d < g; ++d) {
        int dm = rs[d + 1] - rs[d];
        if (dm <= 0) continue;
        int *lp = (int *)malloc(sizeof(int) * (dm + 1));
        for (int i = 0; i <= dm; ++i) lp[i] = (int)(rowptr[rs[d] + i] - rowptr[rs[d]]);
        local_csrmv(dm, lp, col + rowptr[rs[d]], val + rowptr[rs[d]], x, alpha, beta, y + rs[d]);
        free(lp);
    }
    free(rs);
}

/* ------------------------------------------------------------------------ */
/* dspmv_test.cu:137-208 with the row loop clamped to m (Q3). */
long long orc_gen_ref_nnz(int n)
{
    int m = n, nb = m / 8;
    if (nb <= 0) nb = 1;
    long long p = 0;
    for (int i = 0; i < m; i += nb) {
        double r = (i == 0) ? 0.9 : 0.01;
        int hi = i + nb < m ? i + nb : m;
        for (int ii = i; ii < hi; ++ii)
            for (int j = 0; j < n * r; ++j) p++;
    }
    return p;
}

void orc_gen_ref(int n, int *coo_row, int *coo_col, double *coo_val)
{
    int m = n, nb = m / 8;
    if (nb <= 0) nb = 1;
    long long p = 0;
    srand(1);
    for (int i = 0; i < m; i += nb) {
        double r = (i == 0) ? 0.9 : 0.01;
        int hi = i + nb < m ? i + nb : m;
        for (int ii = i; ii < hi; ++ii)
            for (int j = 0; j < n * r; ++j) {
                coo_row[p] = ii;
                coo_col[p] = j;
                coo_val[p] = (double)rand() / (RAND_MAX);
                p++;
            }
    }
}

/* Synthetic generator (our own definition; DESIGN.md "Synthetic").  One
 * SplitMix64 stream per row, started at mix(seed ^ mix((row+1)*golden)) so
 * that rows draw independent columns.  Columns drawn by 128-bit multiply-high
 * into [0,n), redrawn on a duplicate within the row, then sorted; values
 * drawn afterwards, one per sorted column. */
static unsigned long long mix64(unsigned long long z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static unsigned long long sm64(unsigned long long *s) { return mix64(*s += 0x9E3779B97F4A7C15ULL); }
static double u01(unsigned long long r) { return (double)(r >> 11) * (1.0 / 9007199254740992.0); }

static int cmp_int(const void *a, const void *b)
{
    int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

void orc_gen_synth_rowptr(int n, int heavy, int light, long long *rowptr)
{
    int nh = n / 8;
    rowptr[0] = 0;
    for (int i = 0; i < n; ++i) rowptr[i + 1] = rowptr[i] + (i < nh ? heavy : light);
}

void orc_gen_synth(int n, int heavy, int light, int prefix_cols,
                   unsigned long long seed, const long long *rowptr, int *col,
                   double *val)
{
    (void)heavy; (void)light;
    for (int i = 0; i < n; ++i) {
        long long b = rowptr[i];
        int d = (int)(rowptr[i + 1] - b);
        unsigned long long s = mix64(seed ^ mix64((unsigned long long)(i + 1) * 0x9E3779B97F4A7C15ULL));
        int *c = col + b;
        if (prefix_cols) {
            for (int k = 0; k < d; ++k) c[k] = k;
        } else {
            for (int k = 0; k < d; ++k) {
                for (;;) {
                    unsigned long long r = sm64(&s);
                    int v = (int)(((unsigned __int128)r * (unsigned)n) >> 64);
                    int dup = 0;
                    for (int t = 0; t < k; ++t) if (c[t] == v) { dup = 1; break; }
                    if (!dup) { c[k] = v; break; }
                }
            }
            qsort(c, (size_t)d, sizeof(int), cmp_int);
        }
        for (int k = 0; k < d; ++k) val[b + k] = u01(sm64(&s));
    }
}

void orc_gen_vector(int n, unsigned long long seed, double *v)
{
    unsigned long long s = seed;
    for (int i = 0; i < n; ++i) v[i] = u01(sm64(&s));
}

/* ------------------------------------------------------------------------ */
void orc_transpose(int m, int n, int nnz, const int *rowptr, const int *col,
                   const double *val, int *colptr, int *rowidx, double *cval)
{
    memset(colptr, 0, sizeof(int) * ((size_t)n + 1));
    for (int i = 0; i < nnz; ++i) colptr[col[i] + 1]++;
    for (int i = 0; i < n; ++i) colptr[i + 1] += colptr[i];
    int *next = (int *)malloc(sizeof(int) * ((size_t)n + 1));
    memcpy(next, colptr, sizeof(int) * ((size_t)n + 1));
    for (int r = 0; r < m; ++r)
        for (int j = rowptr[r]; j < rowptr[r + 1]; ++j) {
            int o = next[col[j]]++;
            rowidx[o] = r;
            cval[o] = val[j];
        }
    free(next);
}

int orc_build_tri(int m, const int *rowptr, const int *col, int substitution,
                  unsigned seed, int *trowptr, int *tcol, double *tval)
{
    int p = 0;
    if (trowptr) { srand(seed); trowptr[0] = 0; }
    for (int i = 0; i < m; ++i) {
        for (int j = rowptr[i]; j < rowptr[i + 1]; ++j) {
            int c = col[j];
            int keep = substitution == 0 ? c < i : c > i;
            if (!keep) continue;
            if (trowptr) { tcol[p] = c; tval[p] = (double)(rand() % 10 + 1); }
            p++;
        }
        if (trowptr) { tcol[p] = i; tval[p] = 1.0; trowptr[i + 1] = p + 1; }
        p++;
    }
    return p;
}

void orc_tri_rhs(int n, const int *colptr, const int *rowidx, const double *val,
                 double *x_ref, double *b)
{
    for (int i = 0; i < n; ++i) x_ref[i] = (double)(rand() % 10 + 1);
    for (int i = 0; i < n; ++i) b[i] = 0.0;
    for (int i = 0; i < n; ++i)
        for (int j = colptr[i]; j < colptr[i + 1]; ++j) b[rowidx[j]] += val[j] * x_ref[i];
}

/* sptrsv_syncfree_serialref.h:6-108: in-degree histogram, then columns in
 * order (forward) or reverse (backward); x = (b - left_sum)/diag; scatter. */
int orc_sptrsv_serial(const int *colptr, const int *rowidx, const double *val,
                      int n, int substitution, int rhs, const double *b,
                      double *x)
{
    double *left = (double *)calloc((size_t)n * rhs, sizeof(double));
    if (substitution == 0) {
        for (int i = 0; i < n; ++i) {
            for (int k = 0; k < rhs; ++k)
                x[i * rhs + k] = (b[i * rhs + k] - left[i * rhs + k]) / val[colptr[i]];
            for (int j = colptr[i] + 1; j < colptr[i + 1]; ++j)
                for (int k = 0; k < rhs; ++k)
                    left[rowidx[j] * rhs + k] += x[i * rhs + k] * val[j];
        }
    } else {
        for (int i = n - 1; i >= 0; --i) {
            for (int k = 0; k < rhs; ++k)
                x[i * rhs + k] = (b[i * rhs + k] - left[i * rhs + k]) / val[colptr[i + 1] - 1];
            for (int j = colptr[i]; j < colptr[i + 1] - 1; ++j)
                for (int k = 0; k < rhs; ++k)
                    left[rowidx[j] * rhs + k] += x[i * rhs + k] * val[j];
        }
    }
    free(left);
    return 0;
}

/* findlevel.h:71-147 computes level sets by repeated in-degree peeling; the
 * level of column i equals 1 + max level of the columns it depends on. */
int orc_levels_lower(int n, const int *colptr, const int *rowidx, int *level_of)
{
    int nlev = 0;
    for (int i = 0; i < n; ++i) level_of[i] = 0;
    for (int i = 0; i < n; ++i) {
        int li = level_of[i];
        if (li + 1 > nlev) nlev = li + 1;
        for (int j = colptr[i]; j < colptr[i + 1]; ++j) {
            int r = rowidx[j];
            if (r != i && level_of[r] < li + 1) level_of[r] = li + 1;
        }
    }
    return nlev;
}

/* ------------------------------------------------------------------------ */
void orc_spmm(int m, int n, int k, double alpha, const int *rowptr,
              const int *col, const double *val, const double *B, int ldb,
              double beta, double *C, int ldc)
{
    (void)k;
    for (int c = 0; c < n; ++c)
        for (int i = 0; i < m; ++i) {
            double s = 0.0;
            for (int j = rowptr[i]; j < rowptr[i + 1]; ++j)
                s += val[j] * B[(long long)c * ldb + col[j]];
            double *o = C + (long long)c * ldc + i;
            *o = (beta == 0.0) ? alpha * s : alpha * s + beta * *o;
        }
}

void orc_spmm_omp(int m, int n, double alpha, const int *rowptr, const int *col,
                  const double *val, const double *B, int ldb, int b_rowmajor, double beta,
                  double *C, int ldc, double *bound, int nthreads)
{
    const double u = 0x1p-53;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
    {
        /* per (row, column of C) the sum runs over the row's entries in
         * storage order, as orc_spmm; the column loop is inside so B rows
         * are read contiguously when B is row-major */
        double *s = (double *)malloc(sizeof(double) * 2 * (size_t)(n > 0 ? n : 1));
        double *a = s + n;
#pragma omp for schedule(dynamic, 4)
        for (int i = 0; i < m; ++i) {
            const double k = (double)(rowptr[i + 1] - rowptr[i]);
            const double gam = k * u / (1.0 - k * u);
            for (int c = 0; c < n; ++c) s[c] = a[c] = 0.0;
            for (int j = rowptr[i]; j < rowptr[i + 1]; ++j) {
                const double v = val[j];
                for (int c = 0; c < n; ++c) {
                    const double b = b_rowmajor ? B[(long long)col[j] * ldb + c]
                                                : B[(long long)c * ldb + col[j]];
                    s[c] += v * b;
                    a[c] += fabs(alpha * v * b);
                }
            }
            for (int c = 0; c < n; ++c) {
                double *o = C + (long long)c * ldc + i;
                if (bound) bound[(long long)c * ldc + i] = 4.0 * gam * a[c] + 4.0 * u * fabs(beta * *o) + 1e-300;
                *o = (beta == 0.0) ? alpha * s[c] : alpha * s[c] + beta * *o;
            }
        }
        free(s);
    }
}

typedef struct { int r, c; double v; } coo_t;
static int cmp_coo(const void *a, const void *b)
{
    const coo_t *x = (const coo_t *)a, *y = (const coo_t *)b;
    if (x->r != y->r) return (x->r > y->r) - (x->r < y->r);
    return (x->c > y->c) - (x->c < y->c);
}

void orc_coo_sort_to_csr(int m, int nnz, int *coo_row, int *coo_col,
                         double *coo_val, int *rowptr)
{
    coo_t *t = (coo_t *)malloc(sizeof(coo_t) * (size_t)(nnz ? nnz : 1));
    for (int i = 0; i < nnz; ++i) { t[i].r = coo_row[i]; t[i].c = coo_col[i]; t[i].v = coo_val[i]; }
    qsort(t, (size_t)nnz, sizeof(coo_t), cmp_coo);
    for (int i = 0; i <= m; ++i) rowptr[i] = 0;
    for (int i = 0; i < nnz; ++i) {
        coo_row[i] = t[i].r; coo_col[i] = t[i].c; coo_val[i] = t[i].v;
        rowptr[t[i].r + 1]++;
    }
    for (int i = 0; i < m; ++i) rowptr[i + 1] += rowptr[i];
    free(t);
}
