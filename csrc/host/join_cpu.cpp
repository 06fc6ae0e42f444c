// CPU engine of the fused join-predict reductions (sql/fused.py, ops/join_predict.py): the
// per-exploded-row values of the FFM scoring query, computed in parallel; the per-group sums are
// formed by the caller (np.bincount, fp64).  Same rule as csrc/kernels/join_predict.hip
// join_ffm_kernel: <V1[ti], V2[tj]> xi xj when both V rows exist, else W1[ti] xi (NaN W = NULL).
#include <cmath>
#include <cstdint>

#define HM_API extern "C" __attribute__((visibility("default")))

HM_API void hm_join_ffm_rows_cpu(const int32_t* ti, const int32_t* tj, const float* xi, const float* xj,
                                 const float* W1, const float* V1, const uint8_t* m1, const float* V2,
                                 const uint8_t* m2, int64_t n, int k, double* out) {
#pragma omp parallel for schedule(static) if (n > 65536)
    for (int64_t i = 0; i < n; ++i) {
        const int a = ti[i];
        double v = 0.0;
        if (a >= 0) {
            const int b = tj[i];
            if (b >= 0 && m1[a] && m2[b]) {
                const float* p = V1 + (int64_t)a * k;
                const float* q = V2 + (int64_t)b * k;
                double d = 0.0;
                for (int f = 0; f < k; ++f) d += (double)p[f] * (double)q[f];
                v = d * (double)xi[i] * (double)xj[i];
            } else if (!std::isnan(W1[a])) {
                v = (double)W1[a] * (double)xi[i];
            }
        }
        out[i] = v;
    }
}
