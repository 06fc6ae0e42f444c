// Column forms of the scalar math UDFs the SQL executor calls once per row otherwise
// (tools/functions.py sigmoid).  Same libm calls and branch order as the per-row Python
// (math.exp is the C library's exp), so the column result is bit-identical to it.
#include <cmath>
#include <cstdint>

#define HM_API extern "C" __attribute__((visibility("default")))

HM_API void hm_sigmoid_f64(const double* x, int64_t n, double* out) {
#pragma omp parallel for schedule(static) if (n > 65536)
    for (int64_t i = 0; i < n; ++i) {
        const double v = x[i];
        out[i] = v >= 0.0 ? 1.0 / (1.0 + std::exp(-v)) : std::exp(v) / (1.0 + std::exp(v));
    }
}
