// test_sptrsv -- CLI clone of sptrsv/sptrsv_v1/src/main.cu:
//
//   test_sptrsv -n <ngpu> -rhs <k> -forward|-backward -mtx <A.mtx> [-seed s] [-opt 1|3]
//
// L (U) = strict lower (upper) pattern of A with values rand()%10+1 plus a
// unit diagonal (main.cu:150-186), CSC by a stable transpose (tranpose.h),
// x_ref = rand()%10+1, b = L*x_ref (main.cu:329-355).  The reference seeds
// rand() with time(NULL) (quirk Q8); this tool uses -seed (default 1) so runs
// are reproducible.  Prints the reference's lines, including the one
// run_test.py parses ("cuda syncfree SpTRSV solve used X ms").
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/sblas.h"
#include "../../include/sblas_refapi.h"

using namespace std;

int main(int argc, char **argv)
{
    if (argc < 8) {
        printf("Usage: ./test_sptrsv -n [number of GPU(s)] -rhs 1 -forward -mtx [input sparse matrix A file] "
               "[-k tasks per GPU (sptrsv_v3)]\n");
        return -1;
    }
    int ngpu = 1, rhs = 1, substitution = 0, opt = 3, task = 0;
    unsigned seed = 1;
    const char *filename = nullptr;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "-n") && i + 1 < argc) ngpu = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-rhs") && i + 1 < argc) rhs = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-forward")) substitution = 0;
        else if (!strcmp(argv[i], "-backward")) substitution = 1;
        else if (!strcmp(argv[i], "-mtx") && i + 1 < argc) filename = argv[++i];
        else if (!strcmp(argv[i], "-seed") && i + 1 < argc) seed = (unsigned)atoi(argv[++i]);
        else if (!strcmp(argv[i], "-opt") && i + 1 < argc) opt = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-k") && i + 1 < argc) task = atoi(argv[++i]);  // v3: tasks per GPU
    }
    printf("---------------------------------------------------------------------------------------------\n");
    printf("PRECISION = 64-bit Double Precision\n");
    printf("Benchmark REPEAT = 1\n");
    printf("---------------------------------------------------------------------------------------------\n");
    int count = 0;
    sblas_device_count(&count);
    if (count <= 0 || ngpu <= 0) {
        printf("Error: Number of GPU(s) needs to be greater than 0.\n");
        return -1;
    }
    printf("Using %i GPU(s).\n", ngpu);
    printf("rhs = %i\n", rhs);
    printf("substitution = %i\n", substitution);
    if (!filename || rhs <= 0) {
        printf("usage: -rhs <k >= 1> with -mtx <file>\n");
        return -1;
    }
    printf("-------------- %s --------------\n", filename);
    srand(seed);
    int m = 0, n = 0;
    long long nnz = 0;
    if (sblas_mm_read(filename, 0, &m, &n, &nnz, nullptr, nullptr, nullptr) != SBLAS_OK) {
        printf("%s\n", sblas_last_error());
        return -1;
    }
    vector<long long> rp((size_t)m + 1);
    vector<int> col((size_t)max(nnz, 1LL));
    vector<double> val((size_t)max(nnz, 1LL));
    sblas_mm_read(filename, 0, &m, &n, &nnz, rp.data(), col.data(), val.data());
    printf("input matrix A: ( %i, %i ) nnz = %lld\n", m, n, nnz);
    if (m != n) {
        printf("This is not a square matrix, return.\n");
        return -1;
    }
    // triangular part + unit diagonal, in row order
    vector<int> trp((size_t)m + 1, 0), tcol;
    vector<double> tval;
    tcol.reserve((size_t)(nnz + m));
    tval.reserve((size_t)(nnz + m));
    for (int i = 0; i < m; ++i) {
        for (long long j = rp[(size_t)i]; j < rp[(size_t)i + 1]; ++j) {
            const int c = col[(size_t)j];
            if (substitution == 0 ? c < i : c > i) {
                tcol.push_back(c);
                tval.push_back((double)(rand() % 10 + 1));
            }
        }
        tcol.push_back(i);
        tval.push_back(1.0);
        trp[(size_t)i + 1] = (int)tcol.size();
    }
    const int nnzTR = (int)tcol.size();
    printf(substitution == 0 ? "A's unit-lower triangular L: ( %i, %i ) nnz = %i\n"
                             : "A's unit-upper triangular U: ( %i, %i ) nnz = %i\n", m, n, nnzTR);
    // stable CSR -> CSC (row indices ascend within a column)
    vector<int> cp((size_t)n + 1, 0), ri((size_t)nnzTR);
    vector<double> cv((size_t)nnzTR);
    for (int e = 0; e < nnzTR; ++e) cp[(size_t)tcol[(size_t)e] + 1]++;
    for (int c = 0; c < n; ++c) cp[(size_t)c + 1] += cp[(size_t)c];
    vector<int> next(cp.begin(), cp.end() - 1);
    for (int r = 0; r < m; ++r)
        for (int e = trp[(size_t)r]; e < trp[(size_t)r + 1]; ++e) {
            const int o = next[(size_t)tcol[(size_t)e]]++;
            ri[(size_t)o] = r;
            cv[(size_t)o] = tval[(size_t)e];
        }
    // level sets (stats only, findlevel.h:71-147)
    vector<int> lev((size_t)n, 0);
    int nlevel = 0;
    for (int t = 0; t < n; ++t) {
        const int i = substitution == 0 ? t : n - 1 - t;
        nlevel = max(nlevel, lev[(size_t)i] + 1);
        for (int j = cp[(size_t)i]; j < cp[(size_t)i + 1]; ++j)
            if (ri[(size_t)j] != i) lev[(size_t)ri[(size_t)j]] = max(lev[(size_t)ri[(size_t)j]], lev[(size_t)i] + 1);
    }
    vector<int> hist((size_t)max(nlevel, 1), 0);
    for (int i = 0; i < n; ++i) hist[(size_t)lev[(size_t)i]]++;
    const int pmin = nlevel ? *min_element(hist.begin(), hist.end()) : 0;
    const int pmax = nlevel ? *max_element(hist.begin(), hist.end()) : 0;
    printf("This matrix/graph has %i levels, its parallelism is %4.2f (min: %i ; avg: %i ; max: %i )\n",
           nlevel, nlevel ? (double)m / nlevel : 0.0, pmin, nlevel ? m / nlevel : 0, pmax);
    // x_ref / b / x are n x rhs row-major (main.cu:330-352)
    const size_t R = (size_t)rhs;
    vector<double> x_ref((size_t)n * R), b((size_t)m * R, 0.0), x((size_t)n * R, 0.0);
    for (size_t i = 0; i < (size_t)n * R; ++i) x_ref[i] = (double)(rand() % 10 + 1);
    for (int c = 0; c < n; ++c)
        for (int j = cp[(size_t)c]; j < cp[(size_t)c + 1]; ++j)
            for (size_t k = 0; k < R; ++k)
                b[(size_t)ri[(size_t)j] * R + k] += cv[(size_t)j] * x_ref[(size_t)c * R + k];
    printf("----------------------------start-----------------------------------------------------\n");
    double gflops = 0;
    // -k <task>: sptrsv_v3's overload (ngpu*task round-robin tasks)
    const int rc = task > 0
        ? sptrsv_syncfree_cuda(cp.data(), ri.data(), cv.data(), m, n, nnzTR, substitution, rhs, opt,
                               x.data(), b.data(), x_ref.data(), &gflops, ngpu, task)
        : sptrsv_syncfree_cuda(cp.data(), ri.data(), cv.data(), m, n, nnzTR, substitution, rhs, opt,
                               x.data(), b.data(), x_ref.data(), &gflops, ngpu);
    if (rc != 0) printf("sptrsv failed: %s\n", sblas_last_error());
    printf("----------------------------done------------------------------------------------------------\n");
    return rc == 0 ? 0 : 1;
}
