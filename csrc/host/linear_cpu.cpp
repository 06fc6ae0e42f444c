// CPU engine of the online linear family: same replica / shard / row-order semantics as
// csrc/kernels/linear.hip (replica r = one sequential Hivemall mapper over its shard),
// replicas run in parallel with OpenMP.  With R = 1 this is exactly upstream's
// single-mapper per-example learner and serves as the numerical oracle of the kernel.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../kernels/linear_rules.h"

#define HM_API extern "C" __attribute__((visibility("default")))

using namespace hm_lin;

namespace {

inline F4 ld4(const float* p) { return F4{p[0], p[1], p[2], p[3]}; }
inline void st4(float* p, const F4& s) { p[0] = s.w; p[1] = s.s1; p[2] = s.s2; p[3] = s.s3; }

void train_replica(const Params& P, int r, int R, int dims, int L, int64_t n_rows, int mini_batch,
                   const int64_t* indptr, const int32_t* idx, const float* val, const float* y,
                   const int32_t* order, float* S, uint8_t* touched, float* RS, double* loss_out) {
    const size_t msize = (size_t)L * dims;
    float* M = S + (size_t)r * msize * 4;
    uint8_t* T = touched + (size_t)r * dims;
    float* rs = RS + (size_t)r * HM_REP_SCALARS;
    double loss_acc = 0.0;
    const int64_t r0 = n_rows * r / R, r1 = n_rows * (r + 1) / R;
    const bool mc = L > 1;
    const bool minib = mini_batch > 1 && P.algo == A_GENERAL && !mc;
    std::vector<float> gacc;
    std::vector<uint8_t> gmark;
    std::vector<int> tlist;
    if (minib) {
        gacc.assign(dims, 0.f);
        gmark.assign(dims, 0);
    }
    int in_batch = 0;
    // Rows are sequential (row q+1 reads what row q wrote), but the state lines a later row needs
    // can be requested early: at Hivemall's 2^24 hashed dims the 256-MB table misses every
    // cache, and touching row q+PF's lines now overlaps their misses with row q's math.  A pure
    // hint: the arithmetic and its order are unchanged.
    constexpr int64_t PF = 2;
    for (int64_t q = r0; q < r1; ++q) {
        const int64_t row = order ? (int64_t)order[q] : q;
        const int64_t s = indptr[row], e = indptr[row + 1];
        if (!mc && q + PF < r1) {
            const int64_t pr = order ? (int64_t)order[q + PF] : q + PF;
            for (int64_t k = indptr[pr], ke = indptr[pr + 1]; k < ke; ++k) {
                const uint32_t i = (uint32_t)idx[k];
                if (i < (uint32_t)dims) __builtin_prefetch(M + (size_t)i * 4, 1, 3);
            }
        }
        const float yy = y[row];
        rs[RS_T] += 1.f;
        const float t = rs[RS_T];
        const StepK sk = step_consts(P, t);
        if (!mc) {
            float p = 0.f, var = 0.f, sq = 0.f;
            for (int64_t k = s; k < e; ++k) {
                const int i = idx[k];
                if (i < 0 || i >= dims) continue;
                const float x = val ? val[k] : 1.f;
                T[i] = 1;
                const F4 st = ld4(M + (size_t)i * 4);
                p += st.w * x;
                var += st.s1 * x * x;
                sq += x * x;
            }
            const RowCoef c = row_rule(P, p, yy, var, sq, rs);
            loss_acc += c.loss;
            if (minib) {
                if (c.update) {
                    for (int64_t k = s; k < e; ++k) {
                        const int i = idx[k];
                        if (i < 0 || i >= dims) continue;
                        const float x = val ? val[k] : 1.f;
                        if (!gmark[i]) { gmark[i] = 1; tlist.push_back(i); }
                        gacc[i] += c.dloss * x;
                    }
                }
                ++in_batch;
                if (in_batch == mini_batch || q + 1 == r1) {
                    const float inv = 1.f / (float)in_batch;
                    for (int i : tlist) {
                        F4 st = ld4(M + (size_t)i * 4);
                        optimizer_update(P, st, gacc[i] * inv, sk, rs[RS_EVE_D]);
                        st4(M + (size_t)i * 4, st);
                        gacc[i] = 0.f;
                        gmark[i] = 0;
                    }
                    tlist.clear();
                    in_batch = 0;
                }
                continue;
            }
            if (!c.update) continue;
            for (int64_t k = s; k < e; ++k) {
                const int i = idx[k];
                if (i < 0 || i >= dims) continue;
                const float x = val ? val[k] : 1.f;
                F4 st = ld4(M + (size_t)i * 4);
                feature_update(P, c, st, x, sk, rs[RS_EVE_D]);
                st4(M + (size_t)i * 4, st);
            }
        } else {
            const int act = (int)yy;
            float sa = 0.f, va = 0.f, sm = -INFINITY, vm = 0.f, sq = 0.f;
            int miss = -1;
            for (int64_t k = s; k < e; ++k) {
                const int i = idx[k];
                if (i < 0 || i >= dims) continue;
                const float x = val ? val[k] : 1.f;
                T[i] = 1;
                sq += x * x;
            }
            for (int l = 0; l < L; ++l) {
                float pl = 0.f, vl = 0.f;
                for (int64_t k = s; k < e; ++k) {
                    const int i = idx[k];
                    if (i < 0 || i >= dims) continue;
                    const float x = val ? val[k] : 1.f;
                    const F4 st = ld4(M + ((size_t)l * dims + i) * 4);
                    pl += st.w * x;
                    vl += st.s1 * x * x;
                }
                if (l == act) { sa = pl; va = vl; }
                else if (pl > sm) { sm = pl; vm = vl; miss = l; }
            }
            if (miss < 0 || act < 0 || act >= L) continue;
            const MCCoef c = mc_rule(P, sa, sm, va, vm, sq);
            loss_acc += c.loss;
            if (!c.update) continue;
            for (int64_t k = s; k < e; ++k) {
                const int i = idx[k];
                if (i < 0 || i >= dims) continue;
                const float x = val ? val[k] : 1.f;
                float* pa = M + ((size_t)act * dims + i) * 4;
                float* pm = M + ((size_t)miss * dims + i) * 4;
                F4 a = ld4(pa), m = ld4(pm);
                mc_feature_update(P, c.a_act, c.b, a, x);
                mc_feature_update(P, c.a_miss, c.b, m, x);
                st4(pa, a);
                st4(pm, m);
            }
        }
    }
    loss_out[r] = loss_acc;
}

}  // namespace

HM_API int hm_linear_train_cpu(const Params* P, const int32_t* ip, int64_t n_rows,
                               const int64_t* indptr, const int32_t* idx, const float* val,
                               const float* y, const int32_t* order, float* S, uint8_t* touched,
                               float* RS, double* loss_out) {
    const int R = ip[0], dims = ip[1], L = ip[2], mini_batch = ip[3];
    if (R <= 0 || dims <= 0 || L <= 0) return 1;
    // one replica (Hivemall's single mapper): no parallel region — waking the OpenMP team for
    // one worker cost more than the a9a epoch itself
#pragma omp parallel for schedule(dynamic, 1) if (R > 1)
    for (int r = 0; r < R; ++r)
        train_replica(*P, r, R, dims, L, n_rows, mini_batch, indptr, idx, val, y, order, S, touched,
                      RS, loss_out);
    return 0;
}

// Batched scoring (CPU twin of hm_linear_predict).
HM_API int hm_linear_predict_cpu(const float* w, int dims, int L, const int64_t* indptr,
                                 const int32_t* idx, const float* val, int64_t n_rows, float* out,
                                 const float* cov, float* var_out) {
#pragma omp parallel for schedule(static)
    for (int64_t row = 0; row < n_rows; ++row) {
        for (int l = 0; l < L; ++l) {
            const float* wl = w + (size_t)l * dims;
            float p = 0.f, v = 0.f;
            for (int64_t k = indptr[row]; k < indptr[row + 1]; ++k) {
                const int i = idx[k];
                if (i < 0 || i >= dims) continue;
                const float x = val ? val[k] : 1.f;
                p += wl[i] * x;
                if (cov) v += cov[(size_t)l * dims + i] * x * x;
            }
            out[row * L + l] = p;
            if (var_out) var_out[row * L + l] = v;
        }
    }
    return 0;
}
