// CPU engines for train_mf_sgd / train_mf_adagrad / train_bprmf: the rules of
// csrc/kernels/mf.hip applied one rating (triple) at a time, in order (Hivemall's per-mapper
// online semantics).  Used for CPU runs and as the sequential oracle of the kernels.
#include <cmath>
#include <cstdint>
#include <random>

#define HM_API extern "C" __attribute__((visibility("default")))

namespace {
struct P_ {
    int k, kp, n_users, n_items, adagrad, use_bias, update_mean, eta_kind, loss;
    uint32_t seed;
    int max_tries;
    float eta0, power_t, total, lu, li, lj, lb, eps;
};
P_ unpack(const int32_t* ip, const float* hp) {
    P_ P;
    P.k = ip[0]; P.kp = ip[1]; P.n_users = ip[2]; P.n_items = ip[3]; P.adagrad = ip[4];
    P.use_bias = ip[5]; P.update_mean = ip[6]; P.eta_kind = ip[7]; P.loss = ip[8];
    P.seed = (uint32_t)ip[9]; P.max_tries = ip[10] > 0 ? ip[10] : 16;
    P.eta0 = hp[0]; P.power_t = hp[1]; P.total = hp[2]; P.lu = hp[3]; P.li = hp[4];
    P.lj = hp[5]; P.lb = hp[6]; P.eps = hp[7];
    return P;
}
inline float eta_t(const P_& P, float t) {
    if (P.eta_kind == 0) return P.eta0;
    if (P.eta_kind == 1) return P.total > 0.f ? P.eta0 / (1.f + t / P.total) : P.eta0;
    return P.eta0 / std::pow(t > 1.f ? t : 1.f, P.power_t);
}
inline float log1pexp(float x) { return x > 0.f ? x + std::log1p(std::exp(-x)) : std::log1p(std::exp(x)); }
}  // namespace

HM_API int hm_mf_step_cpu(const int32_t* ip, const float* hp, const int32_t* users,
                          const int32_t* items, const float* ratings, int64_t n, int64_t t0,
                          float* Pu, float* Qi, float* Bu, float* Bi, float* mu, float* GPu,
                          float* GQi, float* GBu, float* GBi, int train, float* pred, float* loss) {
    const P_ P = unpack(ip, hp);
    for (int64_t r = 0; r < n; ++r) {
        const int u = users[r], i = items[r];
        if (u < 0 || u >= P.n_users || i < 0 || i >= P.n_items) continue;
        float* pu = Pu + (size_t)u * P.kp;
        float* qi = Qi + (size_t)i * P.kp;
        float dot = 0.f;
        for (int f = 0; f < P.k; ++f) dot += pu[f] * qi[f];
        const float bu = P.use_bias ? Bu[u] : 0.f, bi = P.use_bias ? Bi[i] : 0.f;
        const float rhat = *mu + bu + bi + dot;
        const float e = ratings[r] - rhat;
        if (pred) pred[r] = rhat;
        if (loss) loss[r] = e * e;
        if (!train) continue;
        const float t = (float)(t0 + r + 1);
        if (!P.adagrad) {
            const float eta = eta_t(P, t);
            for (int f = 0; f < P.k; ++f) {
                const float a = pu[f], b = qi[f];
                pu[f] = a + eta * (e * b - P.lu * a);
                qi[f] = b + eta * (e * a - P.li * b);
            }
            if (P.use_bias) {
                Bu[u] = bu + eta * (e - P.lb * bu);
                Bi[i] = bi + eta * (e - P.lb * bi);
            }
        } else {
            float* gpu = GPu + (size_t)u * P.kp;
            float* gqi = GQi + (size_t)i * P.kp;
            for (int f = 0; f < P.k; ++f) {
                const float a = pu[f], b = qi[f];
                const float gp = e * b - P.lu * a, gq = e * a - P.li * b;
                gpu[f] += gp * gp;
                gqi[f] += gq * gq;
                pu[f] = a + P.eta0 * gp / std::sqrt(P.eps + gpu[f]);
                qi[f] = b + P.eta0 * gq / std::sqrt(P.eps + gqi[f]);
            }
            if (P.use_bias) {
                const float gbu = e - P.lb * bu, gbi = e - P.lb * bi;
                GBu[u] += gbu * gbu;
                GBi[i] += gbi * gbi;
                Bu[u] = bu + P.eta0 * gbu / std::sqrt(P.eps + GBu[u]);
                Bi[i] = bi + P.eta0 * gbi / std::sqrt(P.eps + GBi[i]);
            }
        }
    }
    return 0;
}

static bool is_pos(const int64_t* ptr, const int32_t* items, int u, int j) {
    int64_t lo = ptr[u], hi = ptr[u + 1] - 1;
    while (lo <= hi) {
        const int64_t m = (lo + hi) >> 1;
        if (items[m] == j) return true;
        if (items[m] < j) lo = m + 1; else hi = m - 1;
    }
    return false;
}

HM_API int hm_bpr_step_cpu(const int32_t* ip, const float* hp, const int32_t* tu,
                           const int32_t* ti, const int32_t* tj, int64_t n, const int64_t* uptr,
                           const int32_t* uitems, const int32_t* pos_user, int64_t n_pos,
                           int64_t t0, float* Pu, float* Qi, float* Bi, double* loss_sum) {
    const P_ P = unpack(ip, hp);
    std::mt19937_64 rng((uint64_t)P.seed * 0x9E3779B97F4A7C15ull + (uint64_t)t0);
    double lacc = 0.0;
    for (int64_t r = 0; r < n; ++r) {
        int u, i, j = -1;
        if (tu) {
            u = tu[r]; i = ti[r]; j = tj[r];
        } else {
            const int64_t p = (int64_t)(rng() % (uint64_t)n_pos);
            u = pos_user[p];
            i = uitems[p];
            for (int tries = 0; tries < P.max_tries; ++tries) {
                j = (int)(rng() % (uint64_t)P.n_items);
                if (!is_pos(uptr, uitems, u, j)) break;
                j = -1;
            }
        }
        if (u < 0 || u >= P.n_users || i < 0 || i >= P.n_items || j < 0 || j >= P.n_items || i == j)
            continue;
        float* pu = Pu + (size_t)u * P.kp;
        float* qi = Qi + (size_t)i * P.kp;
        float* qj = Qi + (size_t)j * P.kp;
        float d = 0.f;
        for (int f = 0; f < P.k; ++f) d += pu[f] * (qi[f] - qj[f]);
        const float bi = P.use_bias ? Bi[i] : 0.f, bj = P.use_bias ? Bi[j] : 0.f;
        const float x = bi - bj + d;
        float z;
        if (P.loss == 2) { const float s = 1.f / (1.f + std::exp(-x)); z = s * (1.f - s); }
        else z = 1.f / (1.f + std::exp(x));
        lacc += log1pexp(-x);
        const float eta = eta_t(P, (float)(t0 + r + 1));
        for (int f = 0; f < P.k; ++f) {
            const float a = pu[f], b = qi[f], c = qj[f];
            pu[f] = a + eta * (z * (b - c) - P.lu * a);
            qi[f] = b + eta * (z * a - P.li * b);
            qj[f] = c + eta * (-z * a - P.lj * c);
        }
        if (P.use_bias) {
            Bi[i] = bi + eta * (z - P.lb * bi);
            Bi[j] = bj + eta * (-z - P.lb * bj);
        }
    }
    if (loss_sum) *loss_sum += lacc;
    return 0;
}
