// test_spmv -- CLI clone of the reference's spmv/test/dspmv_test.cu (same argv,
// same stdout lines, so run_test.py-style harnesses parse it unchanged):
//
//   test_spmv f <matrix.mtx> <ngpu> <repeat> <kernel 1-3> <f|b> [--ref-loader]
//   test_spmv g <n>          <ngpu> <repeat> <kernel 1-3>
//
// Differences by design:
//   * default loader builds a true CSR (mmio_data semantics, symmetric
//     expansion); --ref-loader reproduces the reference's file-order loader
//     (quirks Q1/Q2) for bit-comparable runs;
//   * the 'g' generator clamps its last row block to m (Q3);
//   * ngpu may exceed the visible GPU count: ordinals wrap (d % count).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <limits>
#include <vector>

#include "../../include/sblas.h"
#include "../../include/sblas_refapi.h"

using namespace std;

int main(int argc, char *argv[])
{
    bool ref_loader = false;
    vector<char *> av;
    for (int i = 0; i < argc; ++i) {
        if (strcmp(argv[i], "--ref-loader") == 0) ref_loader = true;
        else av.push_back(argv[i]);
    }
    argc = (int)av.size();
    if (argc < 6) {
        cout << "Incorrect number of arguments!" << endl;
        cout << "Usage ./spmv [input matrix file] [number of GPU(s)] [number of test(s)] "
                "[kernel version (1-3)] [data type ('f' or 'b')]"
             << endl;
        return -1;
    }
    const char input_type = av[1][0];
    char *filename = av[2];
    const int ngpu = atoi(av[3]);
    const int repeat_test = atoi(av[4]);
    const int kernel_version = atoi(av[5]);

    int deviceCount = 0;
    sblas_device_count(&deviceCount);
    if (deviceCount <= 0) {
        cout << "Error: Not enough number of GPUs. Only " << deviceCount << "available." << endl;
        return -1;
    }
    if (ngpu <= 0) {
        cout << "Error: Number of GPU(s) needs to be greater than 0." << endl;
        return -1;
    }
    if (kernel_version != 1 && kernel_version != 2 && kernel_version != 3) {
        cout << "Error: The kernel version can only be: 1, 2, or 3." << endl;
        return -1;
    }
    cout << "Using " << ngpu << " GPU(s)." << endl;
    cout << "Kernel #" << kernel_version << " is selected." << endl;

    int m = 0, n = 0;
    long long nnz = 0;
    vector<long long> rowptr;
    vector<int> col;
    vector<double> val;
    if (input_type == 'f') {
        const char data_type = argc > 6 ? av[6][0] : 'f';
        cout << "Loading input matrix from " << filename << endl;
        const int mode = ref_loader ? (data_type == 'b' ? 2 : 1) : 0;
        if (sblas_mm_read(filename, mode, &m, &n, &nnz, nullptr, nullptr, nullptr) != SBLAS_OK) {
            printf("Could not process Matrix Market banner.\n");
            exit(1);
        }
        rowptr.resize((size_t)m + 1);
        col.resize((size_t)max(nnz, 1LL));
        val.resize((size_t)max(nnz, 1LL));
        if (sblas_mm_read(filename, mode, &m, &n, &nnz, rowptr.data(), col.data(), val.data()) != SBLAS_OK) {
            printf("%s\n", sblas_last_error());
            exit(1);
        }
        if (data_type == 'b')
            for (auto &v : val) v = 0.00001;
        cout << "m: " << m << " n: " << n << " nnz: " << nnz << endl;
    } else if (input_type == 'g') {
        // dspmv_test.cu:137-208, last block clamped (Q3)
        n = atoi(filename);
        m = n;
        int nb = m / 8;
        if (nb <= 0) nb = 1;
        long long p = 0;
        for (int i = 0; i < m; i += nb) {
            const double r = i == 0 ? 0.9 : 0.01;
            for (int ii = i; ii < min(i + nb, m); ++ii)
                for (int j = 0; j < n * r; ++j) p++;
        }
        nnz = p;
        cout << "m: " << m << " n: " << n << " nnz: " << nnz << endl;
        rowptr.assign((size_t)m + 1, 0);
        col.resize((size_t)max(nnz, 1LL));
        val.resize((size_t)max(nnz, 1LL));
        cout << "Start generating data " << std::flush;
        p = 0;
        for (int i = 0; i < m; i += nb) {
            cout << "." << std::flush;
            const double r = i == 0 ? 0.9 : 0.01;
            for (int ii = i; ii < min(i + nb, m); ++ii) {
                for (int j = 0; j < n * r; ++j) {
                    col[(size_t)p] = j;
                    val[(size_t)p] = (double)rand() / (RAND_MAX);
                    p++;
                }
                rowptr[(size_t)ii + 1] = p;
            }
        }
        cout << endl << "Done generating data." << endl;
    } else {
        cout << "Error: input type must be 'f' or 'g'." << endl;
        return -1;
    }
    const long long matrix_data_space = nnz * (long long)sizeof(double) +
                                        nnz * (long long)sizeof(int) + (m + 1) * (long long)sizeof(int);
    cout << "Matrix space size: " << (double)matrix_data_space / 1e9 << " GB." << endl;

    vector<double> x((size_t)n, 1.0), y1((size_t)m, 0.0), y2((size_t)m, 0.0), y3((size_t)m, 0.0);
    double ALPHA = (double)rand() / (RAND_MAX);
    double BETA = (double)rand() / (RAND_MAX);

    cout << "Warming up GPU(s)..." << endl;
    spMV_mgpu_v1(m, n, nnz, &ALPHA, val.data(), rowptr.data(), col.data(), x.data(), &BETA,
                 y2.data(), ngpu, kernel_version);

    double min_profile_time = numeric_limits<double>::max();
    int best_dev_count = 1, best_copy = 1;
    for (int d = 1; d <= ngpu; d *= 2) {
        for (int c = 1; c <= 8; c *= 2) {
            const double t0 = get_time();
            spMV_mgpu_v2(m, n, nnz, &ALPHA, val.data(), rowptr.data(), col.data(), x.data(), &BETA,
                         y3.data(), d, kernel_version, max(nnz / (d * c), 1LL), c);
            const double t = get_time() - t0;
            if (t < min_profile_time) {
                min_profile_time = t;
                best_dev_count = d;
                best_copy = c;
            }
        }
    }

    int ret1 = 0, ret2 = 0, ret3 = 0;
    double avg_b = 0, avg_1 = 0, avg_2 = 0;
    cout << "Starting tests..." << endl;
    cout << "  Test No.   Baseline    Version 1     Pass     Version 2     Pass" << endl;
    cout << "              Time(s)      Time(s)                Time(s)         " << endl;
    cout << "=======================================================================" << endl;
    for (int it = 0; it < repeat_test; ++it) {
        std::fill(y1.begin(), y1.end(), 0.0);
        std::fill(y2.begin(), y2.end(), 0.0);
        std::fill(y3.begin(), y3.end(), 0.0);
        double t0 = get_time();
        ret1 = spMV_mgpu_baseline(m, n, nnz, &ALPHA, val.data(), rowptr.data(), col.data(),
                                  x.data(), &BETA, y1.data(), ngpu);
        const double tb = get_time() - t0;
        t0 = get_time();
        ret2 = spMV_mgpu_v1(m, n, nnz, &ALPHA, val.data(), rowptr.data(), col.data(), x.data(),
                            &BETA, y2.data(), ngpu, kernel_version);
        const double t1 = get_time() - t0;
        t0 = get_time();
        ret3 = spMV_mgpu_v2(m, n, nnz, &ALPHA, val.data(), rowptr.data(), col.data(), x.data(),
                            &BETA, y3.data(), best_dev_count, kernel_version,
                            max(nnz / ((long long)best_dev_count * best_copy), 1LL), best_copy);
        const double t2 = get_time() - t0;
        avg_b += tb;
        avg_1 += t1;
        avg_2 += t2;
        bool correct1 = true, correct2 = true;
        for (int i = 0; i < m; ++i) {
            if (std::fabs(y1[(size_t)i] - y2[(size_t)i]) > 1e-3) correct1 = false;
            if (std::fabs(y1[(size_t)i] - y3[(size_t)i]) > 1e-3) correct2 = false;
        }
        cout << setw(10) << it + 1;
        if (ret1 == 0) cout << setw(11) << tb; else cout << setw(11) << "Failed";
        if (ret2 == 0) cout << setw(13) << t1; else cout << setw(13) << "Failed";
        if (ret1 == 0) cout << setw(9) << (correct1 ? "Y" : "N"); else cout << setw(9) << "N/A";
        if (ret3 == 0) cout << setw(14) << t2; else cout << setw(14) << "Failed.";
        if (ret1 == 0) cout << setw(9) << (correct2 ? "Y" : "N"); else cout << setw(9) << "N/A";
        cout << endl;
    }
    if (repeat_test > 0) {
        avg_b /= repeat_test;
        avg_1 /= repeat_test;
        avg_2 /= repeat_test;
    }
    cout << "......................................................................." << endl;
    cout << setw(10) << "Average" << " ";
    if (ret1 == 0) cout << setw(11) << avg_b; else cout << setw(11) << "Failed";
    if (ret2 == 0) cout << setw(13) << avg_1; else cout << setw(13) << "Failed";
    if (ret3 == 0) cout << setw(23) << avg_2; else cout << setw(23) << "Failed";
    cout << endl;
    return 0;
}
