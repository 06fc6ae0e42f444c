// CPU engine for train_fm: the rule of csrc/kernels/fm.hip applied strictly row by row
// (Hivemall's per-mapper online SGD).  V is fp32 here (the GPU default is bf16 with
// stochastic rounding); used for CPU runs and as the sequential oracle of the kernel.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#define HM_API extern "C" __attribute__((visibility("default")))

namespace {
inline float log1pexp(float x) { return x > 0.f ? x + std::log1p(std::exp(-x)) : std::log1p(std::exp(x)); }
}

// ip: dims, k, KP, classification, train, eta_kind, use_w0, bf16(ignored), grid(ignored), seed
// hp: eta0, power_t, total_steps, lambda0, lambda_w, lambda_v, min_target, max_target
HM_API int hm_fm_step_cpu(const int32_t* ip, const float* hp, int64_t n_rows, int64_t t0,
                          const int64_t* indptr, const int32_t* idx, const float* val,
                          const float* y, float* w, float* V, float* w0, float* pred, float* loss) {
    const int dims = ip[0], k = ip[1], KP = ip[2], cls = ip[3], train = ip[4], eta_kind = ip[5];
    const int use_w0 = ip[6];
    const float eta0 = hp[0], power_t = hp[1], total = hp[2], l0 = hp[3], lw = hp[4], lv = hp[5];
    const float mn = hp[6], mx = hp[7];
    std::vector<float> S(KP);
    constexpr int64_t PF = 2;      // rows ahead whose w / V lines are requested (a hint only)
    for (int64_t row = 0; row < n_rows; ++row) {
        const int64_t s = indptr[row], e = indptr[row + 1];
        if (row + PF < n_rows)
            for (int64_t q = indptr[row + PF]; q < indptr[row + PF + 1]; ++q) {
                const uint32_t i = (uint32_t)idx[q];
                if (i < (uint32_t)dims) {
                    __builtin_prefetch(w + i, 1, 3);
                    __builtin_prefetch(V + (size_t)i * KP, 1, 3);
                }
            }
        std::fill(S.begin(), S.end(), 0.f);
        float lin = 0.f, sq = 0.f;
        for (int64_t q = s; q < e; ++q) {
            const int i = idx[q];
            if (i < 0 || i >= dims) continue;
            const float x = val ? val[q] : 1.f;
            lin += w[i] * x;
            const float* v = V + (size_t)i * KP;
            for (int f = 0; f < KP; ++f) {
                const float vx = v[f] * x;
                S[f] += vx;
                sq += vx * vx;
            }
        }
        float pair = 0.f;
        for (int f = 0; f < KP; ++f) pair += S[f] * S[f];
        float p = lin + 0.5f * (pair - sq);
        if (use_w0) p += *w0;
        const float yy = y ? y[row] : 0.f;
        float d;
        if (cls) {
            const float z = yy * p;
            d = -yy / (1.f + std::exp(z));
            if (pred) pred[row] = p;
            if (loss) loss[row] = log1pexp(-z);
        } else {
            const float pc = std::min(std::max(p, mn), mx);
            d = pc - yy;
            if (pred) pred[row] = pc;
            if (loss) loss[row] = 0.5f * d * d;
        }
        if (!train) continue;
        const float t = (float)(t0 + row + 1);
        float eta = eta0;
        if (eta_kind == 1) eta = total > 0.f ? eta0 / (1.f + t / total) : eta0;
        else if (eta_kind == 2) eta = eta0 / std::pow(t > 1.f ? t : 1.f, power_t);
        for (int64_t q = s; q < e; ++q) {
            const int i = idx[q];
            if (i < 0 || i >= dims) continue;
            const float x = val ? val[q] : 1.f;
            w[i] -= eta * (d * x + 2.f * lw * w[i]);
            float* v = V + (size_t)i * KP;
            for (int f = 0; f < k; ++f) {
                const float g = d * x * (S[f] - v[f] * x) + 2.f * lv * v[f];
                v[f] -= eta * g;
            }
        }
        if (use_w0) *w0 -= eta * (d + 2.f * l0 * *w0);
    }
    return 0;
}
