// Matrix factorization kernels for gfx950: biased MF with SGD / AdaGrad (train_mf_sgd,
// train_mf_adagrad) and BPR-MF (train_bprmf) with optional fused device-side negative
// sampling.
//
// Semantics (upstream core/src/main/java/hivemall/mf/
// {OnlineMatrixFactorizationUDTF,MatrixFactorizationSGDUDTF,MatrixFactorizationAdaGradUDTF,
// BPRMatrixFactorizationUDTF}.java):
//   MF : r̂ = μ + b_u + b_i + p_u·q_i,  e = r − r̂
//        p_u += η(e q_i − λ p_u);  q_i += η(e p_u − λ q_i);  b_u += η(e − λ b_u); b_i likewise
//        AdaGrad: η_x = η0 / sqrt(eps + G_x) per parameter, G_x += g²
//   BPR: x = b_i − b_j + p_u·(q_i − q_j);  z = dloss  (lnLogistic: σ(−x))
//        p_u += η(z (q_i − q_j) − λu p_u); q_i += η(z p_u − λi q_i); q_j += η(−z p_u − λj q_j)
//        b_i += η(z − λb b_i);  b_j += η(−z − λb b_j)
//
// MI355X mapping: a "group" of G = next_pow2(k) <= 64 lanes owns one rating/triple (lane f
// holds factor f), so k = 10 packs 4 ratings per wave64 (16-lane groups) and k = 64 one.  The
// dot product is a width-G butterfly (__shfl_xor inside the group).  Factor rows are gathered
// as contiguous k-float segments.  Hogwild across groups, like every GPU MF-SGD.
#include "common.h"

namespace {

struct MFParams {
    int k, kp;                 // factors, row stride
    int n_users, n_items;
    int adagrad;               // 0 SGD, 1 AdaGrad
    int use_bias, update_mean;
    int eta_kind;              // 0 fixed, 1 simple, 2 inverse
    float eta0, power_t, total_steps;
    float lambda_u, lambda_i, lambda_j, lambda_b;
    float eps;
    int loss;                  // BPR: 0 lnLogistic, 1 logistic, 2 sigmoid
    uint32_t seed;
    int max_tries;             // negative-sampling rejection tries
    int coherent;              // 1: factor/bias/state loads bypass L1 (hm::ld_coherent)
    int atomic;                // MF: 0 = read-modify-write stores, 1 = atomic delta adds on users
                               // and items, 2 = atomic adds on items only (the skewed side)
    int bstride;               // MF: element stride of Bu / Bi / GBu / GBi (16: one 64-B line each)
    int bm_words;              // BPR: 32-bit words per user in the positive-item bitmap
};

// Shared-model load: L1-bypassing unless disabled for an A/B (HM_MF_PLAIN_LOADS=1).
__device__ __forceinline__ float ldm(const MFParams& P, const float* p) {
    return P.coherent ? hm::ld_coherent(p) : *p;
}

__device__ __forceinline__ float eta_t(const MFParams& P, float t) {
    if (P.eta_kind == 0) return P.eta0;
    if (P.eta_kind == 1) return P.total_steps > 0.f ? P.eta0 / (1.f + t / P.total_steps) : P.eta0;
    return P.eta0 / powf(t > 1.f ? t : 1.f, P.power_t);
}

template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ---------------------------------------------------------------- biased MF (ratings)
template <int G>
__global__ __launch_bounds__(256) void mf_kernel(MFParams P, const int32_t* __restrict__ users,
                                                 const int32_t* __restrict__ items,
                                                 const float* __restrict__ ratings, int64_t n,
                                                 int64_t t0, float* __restrict__ Pu,
                                                 float* __restrict__ Qi, float* __restrict__ Bu,
                                                 float* __restrict__ Bi, float* __restrict__ mu,
                                                 float* __restrict__ GPu, float* __restrict__ GQi,
                                                 float* __restrict__ GBu, float* __restrict__ GBi,
                                                 int train, float* __restrict__ pred,
                                                 float* __restrict__ loss) {
    constexpr int PER = 64 / G;                       // ratings per wave
    const int lane = hm::lane_id();
    const int sub = lane / G, f = lane % G;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + hm::wave_id();
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t base = wave * PER; base < n; base += nwaves * PER) {
        const int64_t r = base + sub;
        const bool act = r < n;
        int u = act ? users[r] : -1, i = act ? items[r] : -1;
        const bool ok = act && u >= 0 && u < P.n_users && i >= 0 && i < P.n_items;
        const bool fa = ok && f < P.k;
        float pu = 0.f, qi = 0.f;
        const size_t ou = (size_t)(ok ? u : 0) * P.kp + f, oi = (size_t)(ok ? i : 0) * P.kp + f;
        if (fa) { pu = ldm(P, Pu + ou); qi = ldm(P, Qi + oi); }
        float dot = group_sum<G>(pu * qi);
        float bu = 0.f, bi = 0.f;
        const size_t bu_o = (size_t)(ok ? u : 0) * P.bstride, bi_o = (size_t)(ok ? i : 0) * P.bstride;
        if (ok && P.use_bias) { bu = ldm(P, Bu + bu_o); bi = ldm(P, Bi + bi_o); }
        const float m = ldm(P, mu);
        const float rhat = m + bu + bi + dot;
        const float rr = act ? ratings[r] : 0.f;
        const float e = rr - rhat;
        if (ok && f == 0) {
            if (pred) pred[r] = rhat;
            if (loss) loss[r] = e * e;
        }
        if (!train || !ok) continue;
        const float t = (float)(t0 + r + 1);
        if (!P.adagrad) {
            const float eta = eta_t(P, t);
            const float dp = eta * (e * qi - P.lambda_u * pu), dq = eta * (e * pu - P.lambda_i * qi);
            const float dbu = eta * (e - P.lambda_b * bu), dbi = eta * (e - P.lambda_b * bi);
            if (P.atomic) {
                // Hogwild as analysed (Niu et al.): component-wise atomic increments, so
                // concurrent ratings of one popular item/user all land (reads stay stale)
                if (fa) {
                    if (P.atomic == 1) atomicAdd(Pu + ou, dp);
                    else Pu[ou] = pu + dp;
                    atomicAdd(Qi + oi, dq);
                }
                if (P.use_bias && f == 0) {
                    if (P.atomic == 1) atomicAdd(Bu + bu_o, dbu);
                    else Bu[bu_o] = bu + dbu;
                    atomicAdd(Bi + bi_o, dbi);
                }
            } else {
                if (fa) {
                    Pu[ou] = pu + dp;
                    Qi[oi] = qi + dq;
                }
                if (P.use_bias && f == 0) {
                    Bu[bu_o] = bu + dbu;
                    Bi[bi_o] = bi + dbi;
                }
            }
        } else if (P.atomic) {
            if (fa) {
                const float gp = e * qi - P.lambda_u * pu, gq = e * pu - P.lambda_i * qi;
                const float Gp = atomicAdd(GPu + ou, gp * gp) + gp * gp;
                const float Gq = atomicAdd(GQi + oi, gq * gq) + gq * gq;
                atomicAdd(Pu + ou, P.eta0 * gp * rsqrtf(P.eps + Gp));
                atomicAdd(Qi + oi, P.eta0 * gq * rsqrtf(P.eps + Gq));
            }
            if (P.use_bias && f == 0) {
                const float gbu = e - P.lambda_b * bu, gbi = e - P.lambda_b * bi;
                const float Gu = atomicAdd(GBu + bu_o, gbu * gbu) + gbu * gbu;
                const float Gi = atomicAdd(GBi + bi_o, gbi * gbi) + gbi * gbi;
                atomicAdd(Bu + bu_o, P.eta0 * gbu * rsqrtf(P.eps + Gu));
                atomicAdd(Bi + bi_o, P.eta0 * gbi * rsqrtf(P.eps + Gi));
            }
        } else {
            if (fa) {
                const float gp = e * qi - P.lambda_u * pu, gq = e * pu - P.lambda_i * qi;
                const float Gp = ldm(P, GPu + ou) + gp * gp, Gq = ldm(P, GQi + oi) + gq * gq;
                GPu[ou] = Gp;
                GQi[oi] = Gq;
                Pu[ou] = pu + P.eta0 * gp * rsqrtf(P.eps + Gp);
                Qi[oi] = qi + P.eta0 * gq * rsqrtf(P.eps + Gq);
            }
            if (P.use_bias && f == 0) {
                const float gbu = e - P.lambda_b * bu, gbi = e - P.lambda_b * bi;
                const float Gu = ldm(P, GBu + bu_o) + gbu * gbu, Gi = ldm(P, GBi + bi_o) + gbi * gbi;
                GBu[bu_o] = Gu;
                GBi[bi_o] = Gi;
                Bu[bu_o] = bu + P.eta0 * gbu * rsqrtf(P.eps + Gu);
                Bi[bi_o] = bi + P.eta0 * gbi * rsqrtf(P.eps + Gi);
            }
        }
    }
}

// ---------------------------------------------------------------- BPR-MF
__device__ __forceinline__ uint32_t pcg(uint64_t& s) {
    const uint64_t old = s;
    s = old * 6364136223846793005ull + 1442695040888963407ull;
    const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    const uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((-rot) & 31));
}

// Is item j in the sorted positive list of user u?  (CSR: ptr[u]..ptr[u+1])
__device__ __forceinline__ bool is_positive(const int64_t* ptr, const int32_t* items, int u, int j) {
    int64_t lo = ptr[u], hi = ptr[u + 1] - 1;
    while (lo <= hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int v = items[mid];
        if (v == j) return true;
        if (v < j) lo = mid + 1; else hi = mid - 1;
    }
    return false;
}

// Triples either given explicitly (tu/ti/tj) or sampled on the device: a uniformly random
// positive (u, i) from the user->items CSR and a uniformly random negative j (rejection
// against u's sorted positives).
template <int G>
__global__ __launch_bounds__(256) void bpr_kernel(MFParams P, const int32_t* __restrict__ tu,
                                                  const int32_t* __restrict__ ti,
                                                  const int32_t* __restrict__ tj, int64_t n,
                                                  const int64_t* __restrict__ uptr,
                                                  const int32_t* __restrict__ uitems,
                                                  const int32_t* __restrict__ pos_user,
                                                  int64_t n_pos, int64_t t0,
                                                  float* __restrict__ Pu, float* __restrict__ Qi,
                                                  float* __restrict__ Bi, double* __restrict__ loss_sum) {
    constexpr int PER = 64 / G;
    const int lane = hm::lane_id();
    const int sub = lane / G, f = lane % G;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + hm::wave_id();
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
    double lacc = 0.0;
    for (int64_t base = wave * PER; base < n; base += nwaves * PER) {
        const int64_t r = base + sub;
        const bool act = r < n;
        int u = -1, i = -1, j = -1;
        if (act) {
            if (tu) {
                u = tu[r]; i = ti[r]; j = tj[r];
            } else {
                uint64_t s = ((uint64_t)P.seed << 32) ^ (uint64_t)(t0 + r) * 0x9E3779B97F4A7C15ull;
                pcg(s);
                const uint64_t pidx = ((uint64_t)pcg(s) << 32 | pcg(s)) % (uint64_t)n_pos;
                u = pos_user[pidx];
                i = uitems[pidx];
                for (int tries = 0; tries < P.max_tries; ++tries) {
                    j = (int)(pcg(s) % (uint32_t)P.n_items);
                    if (!is_positive(uptr, uitems, u, j)) break;
                    j = -1;
                }
            }
        }
        const bool ok = act && u >= 0 && u < P.n_users && i >= 0 && i < P.n_items && j >= 0 &&
                        j < P.n_items && i != j;
        const bool fa = ok && f < P.k;
        const size_t ou = (size_t)(ok ? u : 0) * P.kp + f;
        const size_t oi = (size_t)(ok ? i : 0) * P.kp + f, oj = (size_t)(ok ? j : 0) * P.kp + f;
        float pu = 0.f, qi = 0.f, qj = 0.f;
        if (fa) { pu = ldm(P, Pu + ou); qi = ldm(P, Qi + oi); qj = ldm(P, Qi + oj); }
        const float d = group_sum<G>(pu * (qi - qj));
        float bi = 0.f, bj = 0.f;
        if (ok && P.use_bias) { bi = ldm(P, Bi + i); bj = ldm(P, Bi + j); }
        const float x = bi - bj + d;
        float z;
        if (P.loss == 2) { const float s = hm::sigmoidf_(x); z = s * (1.f - s); }   // sigmoid
        else z = 1.f / (1.f + __expf(x));                                          // σ(−x)
        if (ok && f == 0) lacc += (double)hm::log1pexp(-x);
        if (!ok) continue;
        const float eta = eta_t(P, (float)(t0 + r + 1));
        if (fa) {
            Pu[ou] = pu + eta * (z * (qi - qj) - P.lambda_u * pu);
            Qi[oi] = qi + eta * (z * pu - P.lambda_i * qi);
            Qi[oj] = qj + eta * (-z * pu - P.lambda_j * qj);
        }
        if (P.use_bias && f == 0) {
            Bi[i] = bi + eta * (z - P.lambda_b * bi);
            Bi[j] = bj + eta * (-z - P.lambda_b * bj);
        }
    }
    if (loss_sum) {
        lacc = hm::wave_sum(lacc);
        if (lane == 0 && lacc != 0.0) atomicAdd(loss_sum, lacc);
    }
}

// Pipelined BPR (default; HM_BPR_VARIANT=1 selects bpr_kernel): the sampling of the NEXT triple
// (random positive -> negative rejection) is issued right behind the current triple's factor
// gathers, so its dependent loads overlap the gather / update of the current one instead of
// preceding it; and the rejection test is one load of a per-user item bitmap (built once per
// positive set, n_users x ceil(n_items / 32) words: 472 MB at ML-20M) instead of a binary
// search over the user's sorted items (~8 dependent loads).  The triples drawn are exactly
// bpr_kernel's (same PCG stream, same rejection order).
struct Trip { int u, i, j; };

__device__ __forceinline__ Trip bpr_draw(const MFParams& P, int64_t r, int64_t n, int64_t t0,
                                         const int32_t* __restrict__ tu, const int32_t* __restrict__ ti,
                                         const int32_t* __restrict__ tj, const int64_t* __restrict__ uptr,
                                         const int32_t* __restrict__ uitems,
                                         const int32_t* __restrict__ pos_user, int64_t n_pos,
                                         const uint32_t* __restrict__ bitmap) {
    Trip t{-1, -1, -1};
    if (r >= n) return t;
    if (tu) { t.u = tu[r]; t.i = ti[r]; t.j = tj[r]; return t; }
    uint64_t s = ((uint64_t)P.seed << 32) ^ (uint64_t)(t0 + r) * 0x9E3779B97F4A7C15ull;
    pcg(s);
    const uint64_t pidx = ((uint64_t)pcg(s) << 32 | pcg(s)) % (uint64_t)n_pos;
    t.u = pos_user[pidx];
    t.i = uitems[pidx];
    for (int tries = 0; tries < P.max_tries; ++tries) {
        const int j = (int)(pcg(s) % (uint32_t)P.n_items);
        const bool pos = bitmap ? ((bitmap[(size_t)t.u * P.bm_words + (j >> 5)] >> (j & 31)) & 1u) != 0u
                                : is_positive(uptr, uitems, t.u, j);
        if (!pos) { t.j = j; break; }
    }
    return t;
}

template <int G>
__global__ __launch_bounds__(256) void bpr_pf_kernel(MFParams P, const int32_t* __restrict__ tu,
                                                     const int32_t* __restrict__ ti,
                                                     const int32_t* __restrict__ tj, int64_t n,
                                                     const int64_t* __restrict__ uptr,
                                                     const int32_t* __restrict__ uitems,
                                                     const int32_t* __restrict__ pos_user,
                                                     int64_t n_pos, int64_t t0,
                                                     const uint32_t* __restrict__ bitmap,
                                                     float* __restrict__ Pu, float* __restrict__ Qi,
                                                     float* __restrict__ Bi, double* __restrict__ loss_sum) {
    constexpr int PER = 64 / G;
    const int lane = hm::lane_id();
    const int sub = lane / G, f = lane % G;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + hm::wave_id();
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
    const int64_t stride = nwaves * PER;
    double lacc = 0.0;
    int64_t base = wave * PER;
    Trip cur = bpr_draw(P, base + sub, n, t0, tu, ti, tj, uptr, uitems, pos_user, n_pos, bitmap);
    for (; base < n; base += stride) {
        const int64_t r = base + sub;
        const int u = cur.u, i = cur.i, j = cur.j;
        const bool ok = r < n && u >= 0 && u < P.n_users && i >= 0 && i < P.n_items && j >= 0 &&
                        j < P.n_items && i != j;
        const bool fa = ok && f < P.k;
        const size_t ou = (size_t)(ok ? u : 0) * P.kp + f;
        const size_t oi = (size_t)(ok ? i : 0) * P.kp + f, oj = (size_t)(ok ? j : 0) * P.kp + f;
        float pu = 0.f, qi = 0.f, qj = 0.f, bi = 0.f, bj = 0.f;
        if (fa) { pu = ldm(P, Pu + ou); qi = ldm(P, Qi + oi); qj = ldm(P, Qi + oj); }
        if (ok && P.use_bias) { bi = ldm(P, Bi + i); bj = ldm(P, Bi + j); }
        // the next triple's draw: its loads go out behind this triple's gathers
        cur = bpr_draw(P, r + stride, n, t0, tu, ti, tj, uptr, uitems, pos_user, n_pos, bitmap);
        const float d = group_sum<G>(pu * (qi - qj));
        const float x = bi - bj + d;
        float z;
        if (P.loss == 2) { const float s = hm::sigmoidf_(x); z = s * (1.f - s); }
        else z = 1.f / (1.f + __expf(x));
        if (ok && f == 0) lacc += (double)hm::log1pexp(-x);
        if (!ok) continue;
        const float eta = eta_t(P, (float)(t0 + r + 1));
        if (fa) {
            Pu[ou] = pu + eta * (z * (qi - qj) - P.lambda_u * pu);
            Qi[oi] = qi + eta * (z * pu - P.lambda_i * qi);
            Qi[oj] = qj + eta * (-z * pu - P.lambda_j * qj);
        }
        if (P.use_bias && f == 0) {
            Bi[i] = bi + eta * (z - P.lambda_b * bi);
            Bi[j] = bj + eta * (-z - P.lambda_b * bj);
        }
    }
    if (loss_sum) {
        lacc = hm::wave_sum(lacc);
        if (lane == 0 && lacc != 0.0) atomicAdd(loss_sum, lacc);
    }
}

// Three-stage software pipeline (default with device sampling and the bitmap).
// bpr_pf_kernel still waits per triple on the next draw's dependent rejection load (u from
// pos_user, then the bitmap word of (u, j)) and on its own factor gathers.  Here every triple's
// work is split across three loop iterations of its wave:
//   D1 (iteration q - 3 ... issued): the PCG draw (pure arithmetic: positive index, first negative
//      candidate j0) and the loads of u, i;
//   D2 (q - 2): the bitmap word of (u, j0);
//   G  (q - 1): the rejection test (a positive j0 falls back to bpr_draw's serial loop over the
//      following candidates: same PCG stream, so the triples are exactly bpr_kernel's) and the
//      factor / bias gathers;
//   C  (q):     dot product, loss, SGD stores.
// Each iteration issues D1 of triple q + 3, D2 of q + 2, G of q + 1 in that order and then
// computes q, so every wait is on loads issued one iteration earlier.  The gathers of q + 1 are
// issued before q's stores: if the two triples share a user or item row (a wave's consecutive
// triples are a whole grid's stride apart in the stream), q + 1 reads it one update stale.
struct Draw { uint64_t s; int u, i, j0; };

__device__ __forceinline__ Draw bpr_d1(const MFParams& P, int64_t r, int64_t n, int64_t t0,
                                       const int32_t* __restrict__ tu, const int32_t* __restrict__ ti,
                                       const int32_t* __restrict__ tj, const int32_t* __restrict__ uitems,
                                       const int32_t* __restrict__ pos_user, int64_t n_pos) {
    Draw d{0ull, -1, -1, -1};
    if (r >= n) return d;
    if (tu) { d.u = tu[r]; d.i = ti[r]; d.j0 = tj[r]; return d; }
    uint64_t s = ((uint64_t)P.seed << 32) ^ (uint64_t)(t0 + r) * 0x9E3779B97F4A7C15ull;
    pcg(s);
    const uint64_t pidx = ((uint64_t)pcg(s) << 32 | pcg(s)) % (uint64_t)n_pos;
    d.u = pos_user[pidx];
    d.i = uitems[pidx];
    d.j0 = P.max_tries > 0 ? (int)(pcg(s) % (uint32_t)P.n_items) : -1;
    d.s = s;
    return d;
}

__device__ __forceinline__ uint32_t bpr_d2(const MFParams& P, const Draw& d, const uint32_t* __restrict__ bitmap,
                                           bool sampled) {
    if (!sampled || d.u < 0 || d.u >= P.n_users || d.j0 < 0) return 0u;
    return bitmap[(size_t)d.u * P.bm_words + (d.j0 >> 5)];
}

__device__ __forceinline__ Trip bpr_resolve(const MFParams& P, Draw d, uint32_t word,
                                            const uint32_t* __restrict__ bitmap, bool sampled) {
    Trip t{d.u, d.i, d.j0};
    if (!sampled || d.u < 0) return t;
    if (d.u >= P.n_users) { t.j = -1; return t; }
    if (d.j0 >= 0 && !((word >> (d.j0 & 31)) & 1u)) return t;
    t.j = -1;                                   // j0 is a positive: the serial rejection loop
    uint64_t s = d.s;
    for (int tries = 1; tries < P.max_tries; ++tries) {
        const int j = (int)(pcg(s) % (uint32_t)P.n_items);
        if (!((bitmap[(size_t)d.u * P.bm_words + (j >> 5)] >> (j & 31)) & 1u)) { t.j = j; break; }
    }
    return t;
}

template <int V>
struct Gath { float pu[V], qi[V], qj[V]; float bi, bj; };

// V factors per lane (V = 4: 16-B loads and stores, G = 16 lanes per triple at k = 64, so a wave
// instruction moves four triples' rows instead of one)
template <int V>
__device__ __forceinline__ void ldv(const MFParams& P, const float* p, float (&o)[V]) {
    if constexpr (V == 4) {
        // P.coherent: a non-temporal 16-B load, which also bypasses the CU's L1 (MI355X_MICROARCH.md)
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v v = P.coherent ? __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p))
                                 : *reinterpret_cast<const f4v*>(p);
        o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    } else {
#pragma unroll
        for (int q = 0; q < V; ++q) o[q] = ldm(P, p + q);
    }
}
template <int V>
__device__ __forceinline__ void stv(float* p, const float (&o)[V]) {
    if constexpr (V == 4) {
        *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
        for (int q = 0; q < V; ++q) p[q] = o[q];
    }
}

template <int G, int V = 1>
__global__ __launch_bounds__(256) void bpr_pf3_kernel(MFParams P, const int32_t* __restrict__ tu,
                                                      const int32_t* __restrict__ ti,
                                                      const int32_t* __restrict__ tj, int64_t n,
                                                      const int32_t* __restrict__ uitems,
                                                      const int32_t* __restrict__ pos_user,
                                                      int64_t n_pos, int64_t t0,
                                                      const uint32_t* __restrict__ bitmap,
                                                      float* __restrict__ Pu, float* __restrict__ Qi,
                                                      float* __restrict__ Bi, double* __restrict__ loss_sum) {
    constexpr int PER = 64 / G;
    const int lane = hm::lane_id();
    const int sub = lane / G, f = lane % G;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + hm::wave_id();
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
    const int64_t stride = nwaves * PER;
    const bool sampled = tu == nullptr;
    double lacc = 0.0;
    auto valid = [&](int64_t r, const Trip& t) {
        return r < n && t.u >= 0 && t.u < P.n_users && t.i >= 0 && t.i < P.n_items && t.j >= 0 &&
               t.j < P.n_items && t.i != t.j;
    };
    auto gather = [&](int64_t r, const Trip& t) -> Gath<V> {
        Gath<V> g;
#pragma unroll
        for (int q = 0; q < V; ++q) g.pu[q] = g.qi[q] = g.qj[q] = 0.f;
        g.bi = g.bj = 0.f;
        const bool ok = valid(r, t);
        if (ok && f * V < P.k) {
            ldv<V>(P, Pu + (size_t)t.u * P.kp + f * V, g.pu);
            ldv<V>(P, Qi + (size_t)t.i * P.kp + f * V, g.qi);
            ldv<V>(P, Qi + (size_t)t.j * P.kp + f * V, g.qj);
        }
        if (ok && P.use_bias) { g.bi = ldm(P, Bi + t.i); g.bj = ldm(P, Bi + t.j); }
        return g;
    };
    const int64_t r0 = wave * PER + sub;
    // prologue: triple r0 resolved and gathered, r0 + stride's bitmap word and r0 + 2 stride's u / i in flight
    Draw da = bpr_d1(P, r0, n, t0, tu, ti, tj, uitems, pos_user, n_pos);
    Draw db = bpr_d1(P, r0 + stride, n, t0, tu, ti, tj, uitems, pos_user, n_pos);
    Trip ta = bpr_resolve(P, da, bpr_d2(P, da, bitmap, sampled), bitmap, sampled);
    Gath<V> ga = gather(r0, ta);
    uint32_t wb = bpr_d2(P, db, bitmap, sampled);
    Draw dc = bpr_d1(P, r0 + 2 * stride, n, t0, tu, ti, tj, uitems, pos_user, n_pos);
    for (int64_t base = wave * PER; base < n; base += stride) {
        const int64_t r = base + sub;
        // ---- issue: D1 of r + 3 stride, D2 of r + 2 stride, G of r + stride ----
        const Draw dn = bpr_d1(P, r + 3 * stride, n, t0, tu, ti, tj, uitems, pos_user, n_pos);
        const uint32_t wc = bpr_d2(P, dc, bitmap, sampled);
        const Trip tb = bpr_resolve(P, db, wb, bitmap, sampled);
        const Gath<V> gb = gather(r + stride, tb);
        // ---- compute triple r ----
        const bool ok = valid(r, ta);
        float part = 0.f;
#pragma unroll
        for (int q = 0; q < V; ++q) part += ga.pu[q] * (ga.qi[q] - ga.qj[q]);
        const float d = group_sum<G>(part);
        const float x = ga.bi - ga.bj + d;
        float z;
        if (P.loss == 2) { const float sg = hm::sigmoidf_(x); z = sg * (1.f - sg); }
        else z = 1.f / (1.f + __expf(x));
        if (ok && f == 0) lacc += (double)hm::log1pexp(-x);
        if (ok) {
            const float eta = eta_t(P, (float)(t0 + r + 1));
            if (f * V < P.k) {
                float nu[V], ni[V], nj[V];
#pragma unroll
                for (int q = 0; q < V; ++q) {
                    nu[q] = ga.pu[q] + eta * (z * (ga.qi[q] - ga.qj[q]) - P.lambda_u * ga.pu[q]);
                    ni[q] = ga.qi[q] + eta * (z * ga.pu[q] - P.lambda_i * ga.qi[q]);
                    nj[q] = ga.qj[q] + eta * (-z * ga.pu[q] - P.lambda_j * ga.qj[q]);
                }
                stv<V>(Pu + (size_t)ta.u * P.kp + f * V, nu);
                stv<V>(Qi + (size_t)ta.i * P.kp + f * V, ni);
                stv<V>(Qi + (size_t)ta.j * P.kp + f * V, nj);
            }
            if (P.use_bias && f == 0) {
                Bi[ta.i] = ga.bi + eta * (z - P.lambda_b * ga.bi);
                Bi[ta.j] = ga.bj + eta * (-z - P.lambda_b * ga.bj);
            }
        }
        ta = tb; ga = gb; db = dc; wb = wc; dc = dn;
    }
    if (loss_sum) {
        lacc = hm::wave_sum(lacc);
        if (lane == 0 && lacc != 0.0) atomicAdd(loss_sum, lacc);
    }
}

// bitmap[u * words + (i >> 5)] |= 1 << (i & 31) for every positive pair (user-sorted CSR)
__global__ void bpr_bitmap_kernel(const int32_t* __restrict__ users, const int32_t* __restrict__ items,
                                  int64_t n, int words, uint32_t* __restrict__ bitmap) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
        const int it = items[q];
        atomicOr(bitmap + (size_t)users[q] * words + (it >> 5), 1u << (it & 31));
    }
}

MFParams unpack(const int32_t* ip, const float* hp) {
    MFParams P;
    P.k = ip[0]; P.kp = ip[1]; P.n_users = ip[2]; P.n_items = ip[3]; P.adagrad = ip[4];
    P.use_bias = ip[5]; P.update_mean = ip[6]; P.eta_kind = ip[7]; P.loss = ip[8];
    P.seed = (uint32_t)ip[9]; P.max_tries = ip[10] > 0 ? ip[10] : 16;
    P.coherent = ip[12] == 0;  // ip[12] = 1: plain (L1-cached) loads, A/B only
    P.atomic = ip[13];         // MF: atomic delta updates
    P.bstride = ip[14] > 0 ? ip[14] : 1;
    P.bm_words = (P.n_items + 31) / 32;
    P.eta0 = hp[0]; P.power_t = hp[1]; P.total_steps = hp[2]; P.lambda_u = hp[3];
    P.lambda_i = hp[4]; P.lambda_j = hp[5]; P.lambda_b = hp[6]; P.eps = hp[7];
    return P;
}

int g_grid_override = 0;

int grid_for(int64_t n, int per) {
    if (g_grid_override > 0) {
        const int64_t need = ((n + per - 1) / per + 3) / 4;
        return (int)(g_grid_override < need ? g_grid_override : (need < 1 ? 1 : need));
    }
    int64_t waves = (n + per - 1) / per;
    int64_t blocks = (waves + 3) / 4;
    if (blocks > 256 * 16) blocks = 256 * 16;
    return blocks < 1 ? 1 : (int)blocks;
}

}  // namespace

// ip: k, kp, n_users, n_items, adagrad, use_bias, update_mean, eta_kind, loss, seed, max_tries,
//     grid, plain_loads, atomic, bias_stride
// hp: eta0, power_t, total_steps, lambda_u, lambda_i, lambda_j, lambda_b, eps
HM_API int hm_mf_step(const int32_t* ip, const float* hp, const int32_t* users,
                      const int32_t* items, const float* ratings, int64_t n, int64_t t0, float* Pu,
                      float* Qi, float* Bu, float* Bi, float* mu, float* GPu, float* GQi,
                      float* GBu, float* GBi, int train, float* pred, float* loss,
                      hipStream_t stream) {
    const MFParams P = unpack(ip, hp);
    g_grid_override = ip[11];  // concurrency cap chosen by the host (Hogwild contention policy)
    if (n <= 0) return 0;
    if (P.k <= 0 || P.k > 64 || P.kp < P.k) return (int)hipErrorInvalidValue;
    if (P.adagrad && (!GPu || !GQi || !GBu || !GBi)) return (int)hipErrorInvalidValue;
#define HM_MF(GG)                                                                                  \
    hipLaunchKernelGGL((mf_kernel<GG>), dim3(grid_for(n, 64 / GG)), dim3(256), 0, stream, P, users,  \
                       items, ratings, n, t0, Pu, Qi, Bu, Bi, mu, GPu, GQi, GBu, GBi, train, pred,   \
                       loss)
    if (P.k <= 8) HM_MF(8);
    else if (P.k <= 16) HM_MF(16);
    else if (P.k <= 32) HM_MF(32);
    else HM_MF(64);
#undef HM_MF
    HM_LAUNCH_RET();
}

// ip[15]: 1 = bpr_kernel (the binary-search sampler, no lookahead), 2 = bpr_pf_kernel, else
// bpr_pf3_kernel (bpr_pf_kernel when sampling without the bitmap).
// bitmap: the positive-item bitmap of hm_bpr_bitmap (device sampling), or null.
HM_API int hm_bpr_step(const int32_t* ip, const float* hp, const int32_t* tu, const int32_t* ti,
                       const int32_t* tj, int64_t n, const int64_t* uptr, const int32_t* uitems,
                       const int32_t* pos_user, int64_t n_pos, int64_t t0, float* Pu, float* Qi,
                       float* Bi, double* loss_sum, const uint32_t* bitmap, hipStream_t stream) {
    const MFParams P = unpack(ip, hp);
    g_grid_override = ip[11];  // concurrency cap chosen by the host (Hogwild contention policy)
    const int variant = ip[15];
    if (n <= 0) return 0;
    if (P.k <= 0 || P.k > 64 || P.kp < P.k) return (int)hipErrorInvalidValue;
    if (!tu && (!uptr || !uitems || !pos_user || n_pos <= 0)) return (int)hipErrorInvalidValue;
#define HM_BPR(GG)                                                                                 \
    if (variant == 1)                                                                              \
        hipLaunchKernelGGL((bpr_kernel<GG>), dim3(grid_for(n, 64 / GG)), dim3(256), 0, stream, P, tu, \
                           ti, tj, n, uptr, uitems, pos_user, n_pos, t0, Pu, Qi, Bi, loss_sum);      \
    else if (variant == 2 || (!tu && !bitmap))                                                     \
        hipLaunchKernelGGL((bpr_pf_kernel<GG>), dim3(grid_for(n, 64 / GG)), dim3(256), 0, stream, P, \
                           tu, ti, tj, n, uptr, uitems, pos_user, n_pos, t0, tu ? nullptr : bitmap,  \
                           Pu, Qi, Bi, loss_sum);                                                    \
    else                                                                                           \
        hipLaunchKernelGGL((bpr_pf3_kernel<GG>), dim3(grid_for(n, 64 / GG)), dim3(256), 0, stream, P, \
                           tu, ti, tj, n, uitems, pos_user, n_pos, t0, tu ? nullptr : bitmap,        \
                           Pu, Qi, Bi, loss_sum)
    // k in (16, 64] on 16-B-aligned rows: 4 factors per lane, k / 4 lanes per triple, so one wave
    // instruction moves 64 / G triples' rows (the default).  Measured (profiles/r6/bpr_v4/): k = 64
    // 3.31 vs 1.48-1.59 G triples/s, k = 32 4.99 vs 2.84 G; k = 16 4.18 vs 4.44 G and k = 10 4.35 vs
    // 4.36 G keep the one-factor-per-lane forms (also variant 5, A/B)
    const bool v4 = P.k > 16 && (P.kp & 3) == 0 && variant != 1 && variant != 2 && variant != 5 && (tu || bitmap);
    if (v4) {
        if (P.k <= 32)
            hipLaunchKernelGGL((bpr_pf3_kernel<8, 4>), dim3(grid_for(n, 8)), dim3(256), 0, stream, P, tu, ti, tj, n,
                               uitems, pos_user, n_pos, t0, tu ? nullptr : bitmap, Pu, Qi, Bi, loss_sum);
        else
            hipLaunchKernelGGL((bpr_pf3_kernel<16, 4>), dim3(grid_for(n, 4)), dim3(256), 0, stream, P, tu, ti, tj, n,
                               uitems, pos_user, n_pos, t0, tu ? nullptr : bitmap, Pu, Qi, Bi, loss_sum);
        HM_LAUNCH_RET();
    }
    if (P.k <= 8) HM_BPR(8);
    else if (P.k <= 16) HM_BPR(16);
    else if (P.k <= 32) HM_BPR(32);
    else HM_BPR(64);
#undef HM_BPR
    HM_LAUNCH_RET();
}

// Positive-item bitmap of a user-sorted positive set (bpr_pf_kernel's rejection test); the
// caller zeroes ``bitmap`` (n_users x ceil(n_items / 32) words).
HM_API int hm_bpr_bitmap(const int32_t* users, const int32_t* items, int64_t n, int n_items,
                         uint32_t* bitmap, hipStream_t stream) {
    if (n <= 0) return 0;
    const int words = (n_items + 31) / 32;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 256 * 64) blocks = 256 * 64;
    hipLaunchKernelGGL(bpr_bitmap_kernel, dim3((int)blocks), dim3(256), 0, stream, users, items, n, words, bitmap);
    HM_LAUNCH_RET();
}
