// spmv_ctx -- C++ driver of the single-process multi-GPU context (sblas_ctx:
// ncclCommInitAll, resident slices, ncclBroadcast of x, one ncclAllGather of
// the y slices, device placement).  No Python anywhere on this path.
//
//   spmv_ctx <ngpu> <n> [algo 1|2|4|5] [partition 0=cyclic|1=nnz] [reps]
//            [exchange 0=allgather|1=allreduce (needs partition 1)]
//            [parts K: cyclic + allgather with the exchange overlapped over K
//             parts of each device's chunks, sblas_ctx_matrix_upload_parts]
//
// `spmv_ctx 8 2000000 2 1 20 1` is BASELINE configs[2] from C++: the CSR5
// kernel on spMV_mgpu_v1's nnz split over 8 GPUs, y merged by ncclAllReduce.
//
// Matrix: the config-2 synthetic (rows < n/8: 96 nnz, others 9, uniform
// random sorted columns, seed 42), x U[0,1) seed 43, y0 U[0,1) seed 44,
// alpha/beta = test_spmv's constants.  Checks: every device holds the same y,
// bit for bit; y equals spMV_mgpu_v1 run without the context (host merge)
// within test_spmv's abs 1e-3 and 1e-12 relative; spMV_mgpu_v1 with the
// context bound (RCCL exchange) gives the same y.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/sblas.h"
#include "../../include/sblas_refapi.h"

int main(int argc, char **argv)
{
    if (argc < 3) {
        printf("Usage: ./spmv_ctx <ngpu> <n> [algo 1|2|4|5] [partition 0|1] [reps] [exchange 0|1] [parts]\n");
        return -1;
    }
    const int ngpu = atoi(argv[1]);
    const int n = atoi(argv[2]);
    const int algo = argc > 3 ? atoi(argv[3]) : SBLAS_SPMV_XSORT;
    const int part = argc > 4 ? atoi(argv[4]) : 0;
    const int reps = argc > 5 ? atoi(argv[5]) : 10;
    const int xchg = argc > 6 ? atoi(argv[6]) : SBLAS_CTX_ALLGATHER;
    const int parts = argc > 7 ? atoi(argv[7]) : 1;
    std::vector<long long> rp((size_t)n + 1);
    sblas_gen_synth_rowptr(n, 96, 9, rp.data());
    const long long nnz = rp[(size_t)n];
    std::vector<int> col((size_t)nnz);
    std::vector<double> val((size_t)nnz), x((size_t)n), y0((size_t)n);
    sblas_gen_synth_rows(n, 96, 9, 0, 42, rp.data(), 0, n, col.data(), val.data());
    sblas_gen_vector(n, 43, x.data());
    sblas_gen_vector(n, 44, y0.data());
    double alpha = 0.8401877171547095, beta = 0.39438292681909304;
    printf("m: %d n: %d nnz: %lld, %d GPU(s), algo %d, partition %s, exchange %s\n", n, n, nnz, ngpu, algo,
           part ? "nnz" : "cyclic", xchg ? "allreduce" : "allgather");

    sblas_ctx ctx = nullptr;
    int st = sblas_ctx_create(&ctx, ngpu, nullptr);
    if (st != SBLAS_OK) {
        printf("sblas_ctx_create failed: %s (%s)\n", sblas_status_string(st), sblas_last_error());
        return 1;
    }
    const double t0 = sblas_get_time();
    if (parts > 1 && part == 0 && xchg == SBLAS_CTX_ALLGATHER)
        st = sblas_ctx_matrix_upload_parts(ctx, n, n, rp.data(), col.data(), val.data(), algo, parts);
    else
        st = sblas_ctx_matrix_upload_ex(ctx, n, n, rp.data(), col.data(), val.data(), algo, part, xchg);
    const double t_up = sblas_get_time() - t0;
    if (st == SBLAS_OK) st = sblas_ctx_set_x(ctx, x.data());
    if (st != SBLAS_OK) {
        printf("upload failed: %s (%s)\n", sblas_status_string(st), sblas_last_error());
        return 1;
    }
    printf("upload + analysis: %.3f s\n", t_up);
    // timed steps (y keeps being updated: y <- alpha*A*x + beta*y)
    double sk = 0, sx = 0, stt = 0, stats[3];
    sblas_ctx_set_y(ctx, y0.data());
    sblas_ctx_spmv(ctx, alpha, beta, stats);  // warm-up
    for (int r = 0; r < reps; ++r) {
        if ((st = sblas_ctx_spmv(ctx, alpha, beta, stats)) != SBLAS_OK) break;
        sk += stats[0];
        sx += stats[1];
        stt += stats[2];
    }
    if (st != SBLAS_OK) {
        printf("spmv failed: %s (%s)\n", sblas_status_string(st), sblas_last_error());
        return 1;
    }
    if (reps > 0)
        printf("ctx spmv: kernel %.4f ms, exchange %.4f ms, step %.4f ms = %.1f GFLOP/s\n", sk / reps,
               sx / reps, stt / reps, 2.0 * nnz / (stt / reps * 1e-3) / 1e9);
    // the timing protocol (device-side hold + aligning all-reduce) once
    std::vector<double> tst((size_t)3 + 3 * ngpu);
    if ((st = sblas_ctx_spmv_ex(ctx, alpha, beta, 500.0, 1, tst.data())) != SBLAS_OK) {
        printf("spmv_ex failed: %s (%s)\n", sblas_status_string(st), sblas_last_error());
        return 1;
    }
    printf("ctx aligned step: kernel max %.4f ms, step max %.4f ms\n", tst[0], tst[2]);
    // one checked step from y0
    sblas_ctx_set_y(ctx, y0.data());
    sblas_ctx_spmv(ctx, alpha, beta, nullptr);
    std::vector<double> yc((size_t)n), yd((size_t)n);
    sblas_ctx_get_y(ctx, 0, yc.data());
    bool same = true;
    for (int d = 1; d < ngpu; ++d) {
        sblas_ctx_get_y(ctx, d, yd.data());
        same = same && std::memcmp(yc.data(), yd.data(), sizeof(double) * n) == 0;
    }
    printf("ctx devices agree: %s\n", same ? "PASS" : "FAILED");
    // reference API without the context (host merge), then bound (RCCL)
    std::vector<double> yh(y0), yb(y0);
    sblas_ctx_bind(nullptr);
    int rc1 = spMV_mgpu_v1(n, n, nnz, &alpha, val.data(), rp.data(), col.data(), x.data(), &beta, yh.data(),
                           ngpu, 1);
    sblas_ctx_bind(ctx);
    int rc2 = spMV_mgpu_v1(n, n, nnz, &alpha, val.data(), rp.data(), col.data(), x.data(), &beta, yb.data(),
                           ngpu, 1);
    sblas_ctx_bind(nullptr);
    bool ok = same && rc1 == 0 && rc2 == 0;
    double worst = 0;
    for (int i = 0; i < n && ok; ++i) {
        const double e1 = std::fabs(yc[(size_t)i] - yh[(size_t)i]), e2 = std::fabs(yb[(size_t)i] - yh[(size_t)i]);
        const double tol = 1e-12 * std::max(1.0, std::fabs(yh[(size_t)i]));
        worst = std::max(worst, std::max(e1, e2) / std::max(1.0, std::fabs(yh[(size_t)i])));
        if (e1 > 1e-3 || e2 > 1e-3 || e1 > tol || e2 > tol) ok = false;
    }
    printf("ctx vs spMV_mgpu_v1 (host merge) and bound spMV_mgpu_v1 (RCCL): %s (max rel %.3e)\n",
           ok ? "PASS" : "FAILED", worst);
    sblas_ctx_destroy(ctx);
    return ok ? 0 : 1;
}
