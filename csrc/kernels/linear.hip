// Online linear learner family on gfx950 ("mapper-in-a-wave").
//
// Hivemall's linear learners are strictly sequential per example (the PA / CW / AROW / SCW
// updates depend on the current weights *and* covariance), and Hivemall scales them by
// running one independent learner per mapper and averaging (GROUP BY feature avg(weight)
// or argmin_kld) — SURVEY.md §2.4 DP-1/DP-2, §7.4 hard part 1.  This kernel moves that
// design from nodes to waves:
//
//   * replica r = one 64-lane workgroup that runs Hivemall's exact per-row update over its
//     shard of rows, in order, against its own private model replica (no atomics, no
//     Hogwild, bitwise deterministic);
//   * lanes span the non-zeros of a row: one 16-B float4 {w, s1, s2, s3} gather per feature,
//     xᵀw / xᵀΣx / ‖x‖² reduced with DPP/shuffles, the row rule evaluated wave-uniformly,
//     then one float4 store per feature;
//   * small models (a9a: 124 features = 2 KB) are staged in LDS for the whole shard, so the
//     per-row dependent-load latency is an LDS round trip instead of an L2/HBM one;
//   * replicas are mixed (average over the replicas that touched the feature, or
//     argmin-KLD for covariance learners) by ``hm_linear_mix`` and, across GPUs, by an RCCL
//     all-reduce of the compact sums.
//
// Rules live in linear_rules.h (shared with the CPU engine csrc/host/linear_cpu.cpp).
#include "common.h"
#include "linear_rules.h"

using namespace hm_lin;

namespace {

struct LinLaunch {
    int R, dims, L;
    int64_t n_rows;
    int mini_batch;
    int lds_model;       // model replica staged in LDS
    int touched_cap;     // capacity of the per-replica touched list (mini-batch)
};

__device__ __forceinline__ F4 ld4(const float4* p) {
    float4 v = *p;
    return F4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ void st4(float4* p, const F4& s) { *p = make_float4(s.w, s.s1, s.s2, s.s3); }

template <bool LDS>
__global__ __launch_bounds__(64) void linear_train_kernel(
    Params P, LinLaunch G, const int64_t* __restrict__ indptr, const int32_t* __restrict__ idx,
    const float* __restrict__ val, const float* __restrict__ y, const int32_t* __restrict__ order,
    float4* __restrict__ S, uint8_t* __restrict__ touched, float* __restrict__ RS,
    double* __restrict__ loss_out, float2* __restrict__ gacc, int32_t* __restrict__ tlist) {
    extern __shared__ __attribute__((aligned(16))) float4 s_model[];
    const int r = blockIdx.x;
    const int lane = threadIdx.x;
    const int dims = G.dims, L = G.L;
    const size_t msize = (size_t)L * dims;
    float4* M = S + (size_t)r * msize;
    uint8_t* T = touched + (size_t)r * dims;
    if (LDS) {
        for (size_t i = lane; i < msize; i += 64) s_model[i] = M[i];
        __syncthreads();
        M = s_model;
    }
    float rs[HM_REP_SCALARS];
#pragma unroll
    for (int k = 0; k < HM_REP_SCALARS; ++k) rs[k] = RS[r * HM_REP_SCALARS + k];
    double loss_acc = 0.0;

    const int64_t r0 = G.n_rows * r / G.R, r1 = G.n_rows * (r + 1) / G.R;
    const bool mc = L > 1;
    const bool cov = has_covar(P.algo);
    const bool minib = G.mini_batch > 1 && P.algo == A_GENERAL && !mc;
    float2* GA = minib ? gacc + (size_t)r * dims : nullptr;
    int32_t* TL = minib ? tlist + (size_t)r * G.touched_cap : nullptr;
    int n_touched = 0, in_batch = 0;

    // Row pipeline: the replica's rows are strictly sequential (each row reads the state the
    // previous one wrote), but their CSR bounds, first-chunk indices / values and labels do not
    // depend on the state: row q + 1's are loaded while row q computes and row q + 2's bounds one
    // row earlier, so a row waits on one dependent round trip (the state gather) instead of three.
    auto row_of = [&](int64_t q) -> int64_t { return order ? (int64_t)order[q] : q; };
    int64_t cs = 0, ce = 0;              // bounds of row q
    int64_t pb_s = 0, pb_e = 0;          // bounds of row q + 1
    int pci = -1;                        // first-chunk index / value / label of row q
    float pcx = 0.f, pyy = 0.f;
    if (r0 < r1) {
        const int64_t row0 = row_of(r0);
        cs = indptr[row0];
        ce = indptr[row0 + 1];
        if (lane < (int)(ce - cs)) {
            pci = idx[cs + lane];
            pcx = val ? val[cs + lane] : 1.f;
        }
        pyy = y[row0];
        if (r0 + 1 < r1) {
            const int64_t row1 = row_of(r0 + 1);
            pb_s = indptr[row1];
            pb_e = indptr[row1 + 1];
        }
    }

    for (int64_t q = r0; q < r1; ++q) {
        const int64_t s = cs, e = ce;
        const int nnz = (int)(e - s);
        const float yy = pyy;
        rs[RS_T] += 1.f;
        const float t = rs[RS_T];
        const StepK sk = step_consts(P, t);
        // ---- cached first chunk (prefetched one row ahead) ----
        int ci = pci;
        float cx = pcx;
        if (lane < nnz) {
            if (ci < 0 || ci >= dims) ci = -1;
            if (ci >= 0) T[ci] = 1;
        } else {
            ci = -1;
            cx = 0.f;
        }
        // ---- prefetch: row q + 1's first chunk and label (its bounds are in pb_*), row q + 2's
        //      bounds ----
        cs = pb_s;
        ce = pb_e;
        pci = -1;
        pcx = 0.f;
        if (q + 1 < r1) {
            const int n1 = (int)(ce - cs);
            if (lane < n1) {
                pci = idx[cs + lane];
                pcx = val ? val[cs + lane] : 1.f;
            }
            pyy = y[row_of(q + 1)];
            if (q + 2 < r1) {
                const int64_t row2 = row_of(q + 2);
                pb_s = indptr[row2];
                pb_e = indptr[row2 + 1];
            }
        }
        if (!mc) {
            F4 cst = {0.f, 0.f, 0.f, 0.f};
            float p = 0.f, var = 0.f, sq = 0.f;
            if (ci >= 0) {
                cst = ld4(M + ci);
                p = cst.w * cx;
                var = cst.s1 * cx * cx;
                sq = cx * cx;
            }
            for (int64_t k = s + 64 + lane; k < e; k += 64) {
                int i = idx[k];
                const float x = val ? val[k] : 1.f;
                if (i < 0 || i >= dims) continue;
                T[i] = 1;
                const F4 st = ld4(M + i);
                p += st.w * x;
                var += st.s1 * x * x;
                sq += x * x;
            }
            p = hm::wave_sum(p);
            if (cov) var = hm::wave_sum(var);
            sq = hm::wave_sum(sq);
            const RowCoef c = row_rule(P, p, yy, var, sq, rs);
            loss_acc += c.loss;
            if (minib) {
                // accumulate dloss * x into the replica's dense gradient buffer
                if (c.update) {
                    for (int64_t base = s; base < e; base += 64) {  // wave-uniform trip count
                        const int64_t k = base + lane;
                        const int i = k < e ? idx[k] : -1;
                        const float x = k < e ? (val ? val[k] : 1.f) : 0.f;
                        bool first = false;
                        if (i >= 0 && i < dims) {
                            float2 a = GA[i];
                            first = a.y == 0.f;
                            a.x += c.dloss * x;
                            a.y = 1.f;
                            GA[i] = a;
                        }
                        const uint64_t m = __ballot(first);
                        const int pos = n_touched + __popcll(m & ((1ull << lane) - 1ull));
                        if (first && pos < G.touched_cap) TL[pos] = i;
                        n_touched += __popcll(m);
                    }
                }
                ++in_batch;
                if (in_batch == G.mini_batch || q + 1 == r1 || n_touched + 64 * 4 > G.touched_cap) {
                    const float inv = 1.f / (float)in_batch;
                    const int nt = n_touched < G.touched_cap ? n_touched : G.touched_cap;
                    for (int k = lane; k < nt; k += 64) {
                        const int i = TL[k];
                        F4 st = ld4(M + i);
                        float2 a = GA[i];
                        optimizer_update(P, st, a.x * inv, sk, rs[RS_EVE_D]);
                        st4(M + i, st);
                        GA[i] = make_float2(0.f, 0.f);
                    }
                    n_touched = 0;
                    in_batch = 0;
                }
                continue;
            }
            if (!c.update) continue;
            if (ci >= 0) {
                feature_update(P, c, cst, cx, sk, rs[RS_EVE_D]);
                st4(M + ci, cst);
            }
            for (int64_t k = s + 64 + lane; k < e; k += 64) {
                const int i = idx[k];
                const float x = val ? val[k] : 1.f;
                if (i < 0 || i >= dims) continue;
                F4 st = ld4(M + i);
                feature_update(P, c, st, x, sk, rs[RS_EVE_D]);
                st4(M + i, st);
            }
        } else {
            // ---- multiclass: scores of every label, actual vs best wrong ----
            const int act = (int)yy;
            float sa = 0.f, va = 0.f, sm = -INFINITY, vm = 0.f, sq = 0.f;
            int miss = -1;
            float sqp = 0.f;
            for (int64_t k = s + lane; k < e; k += 64) {
                const float x = val ? val[k] : 1.f;
                const int i = idx[k];
                if (i >= 0 && i < dims) sqp += x * x;
            }
            sq = hm::wave_sum(sqp);
            for (int l = 0; l < L; ++l) {
                float pl = 0.f, vl = 0.f;
                for (int64_t k = s + lane; k < e; k += 64) {
                    const int i = idx[k];
                    const float x = val ? val[k] : 1.f;
                    if (i < 0 || i >= dims) continue;
                    const F4 st = ld4(M + (size_t)l * dims + i);
                    pl += st.w * x;
                    vl += st.s1 * x * x;
                }
                pl = hm::wave_sum(pl);
                if (cov) vl = hm::wave_sum(vl);
                if (l == act) { sa = pl; va = vl; }
                else if (pl > sm) { sm = pl; vm = vl; miss = l; }
            }
            if (miss < 0 || act < 0 || act >= L) continue;
            const MCCoef c = mc_rule(P, sa, sm, va, vm, sq);
            loss_acc += c.loss;
            if (!c.update) continue;
            for (int64_t k = s + lane; k < e; k += 64) {
                const int i = idx[k];
                const float x = val ? val[k] : 1.f;
                if (i < 0 || i >= dims) continue;
                float4* pa = M + (size_t)act * dims + i;
                float4* pm = M + (size_t)miss * dims + i;
                F4 a = ld4(pa), m = ld4(pm);
                mc_feature_update(P, c.a_act, c.b, a, x);
                mc_feature_update(P, c.a_miss, c.b, m, x);
                st4(pa, a);
                st4(pm, m);
            }
        }
    }
    if (LDS) {
        __syncthreads();
        float4* Mg = S + (size_t)r * msize;
        for (size_t i = lane; i < msize; i += 64) Mg[i] = s_model[i];
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < HM_REP_SCALARS; ++k) RS[r * HM_REP_SCALARS + k] = rs[k];
        loss_out[r] = loss_acc;
    }
}

// Replica reduction: per (label, feature) element, over the replicas whose touched byte
// is set.  Outputs compact sums so several GPUs can add theirs with one all-reduce:
//   num = Σ w_r            (plain)       or Σ w_r / σ_r   (argmin-KLD)
//   den = Σ 1              (plain)       or Σ 1 / σ_r
//   cnt = Σ 1 (touching replicas)
__global__ __launch_bounds__(256) void linear_mix_reduce_kernel(
    const float4* __restrict__ S, const uint8_t* __restrict__ touched, int R, int dims, int L,
    int kld, float* __restrict__ num, float* __restrict__ den, float* __restrict__ cnt) {
    const size_t n = (size_t)L * dims;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
         e += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(e % dims);
        float a = 0.f, b = 0.f, c = 0.f;
        for (int r = 0; r < R; ++r) {
            if (!touched[(size_t)r * dims + i]) continue;
            const float4 v = S[(size_t)r * n + e];
            if (kld) {
                const float inv = 1.f / fmaxf(v.y, 1e-12f);
                a += v.x * inv;
                b += inv;
            } else {
                a += v.x;
                b += 1.f;
            }
            c += 1.f;
        }
        num[e] = a;
        den[e] = b;
        cnt[e] = c;
    }
}

// Write the mixed model back into every replica (optimizer state stays local, as upstream
// mixes only weights and covariance).  Elements no replica touched are left unchanged.
__global__ __launch_bounds__(256) void linear_mix_apply_kernel(
    float4* __restrict__ S, int R, int dims, int L, int kld, const float* __restrict__ num,
    const float* __restrict__ den, const float* __restrict__ cnt, float* __restrict__ w_out,
    float* __restrict__ cov_out) {
    const size_t n = (size_t)L * dims;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
         e += (size_t)gridDim.x * blockDim.x) {
        const float c = cnt[e];
        if (c <= 0.f) {
            if (w_out) w_out[e] = S[e].x;
            if (cov_out) cov_out[e] = S[e].y;
            continue;
        }
        const float w = num[e] / den[e];
        const float cv = kld ? c / den[e] : 0.f;
        for (int r = 0; r < R; ++r) {
            float4* p = S + (size_t)r * n + e;
            float4 v = *p;
            v.x = w;
            if (kld) v.y = cv;
            *p = v;
        }
        if (w_out) w_out[e] = w;
        if (cov_out) cov_out[e] = kld ? cv : S[e].y;
    }
}

// Batched scoring: out[row * L + l] = Σ_k w[l][idx[k]] * val[k].  One lane per (row, label).
__global__ __launch_bounds__(256) void linear_predict_kernel(
    const float* __restrict__ w, int dims, int L, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ idx, const float* __restrict__ val, int64_t n_rows,
    float* __restrict__ out, const float* __restrict__ cov, float* __restrict__ var_out) {
    const int64_t total = n_rows * L;
    for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = g / L;
        const int l = (int)(g - row * L);
        const float* wl = w + (size_t)l * dims;
        float p = 0.f, v = 0.f;
        for (int64_t k = indptr[row]; k < indptr[row + 1]; ++k) {
            const int i = idx[k];
            if (i < 0 || i >= dims) continue;
            const float x = val ? val[k] : 1.f;
            p += wl[i] * x;
            if (cov) v += cov[(size_t)l * dims + i] * x * x;
        }
        out[g] = p;
        if (var_out) var_out[g] = v;
    }
}

// Shared-table Hogwild engine for large hashed models (upstream
// GeneralLearnerBaseUDTF / the binary & regression learners at -dims 2^24, where a private
// replica per 64-lane wave no longer fits or fills the chip: 2^24 x 16 B = 256 MB each).
//
// R model tables S [R][dims] {w, s1, s2, s3} in HBM, each shared by W / R waves (Hogwild, no
// atomics): wave g takes rows g, g + W, ... (the rows in flight are a contiguous window of the
// stream) and applies the row rule with the global step t = t0 + row + 1, the sequential
// learner's step.  The replica of a workgroup is chosen XCD-aware: blocks are dealt to the 8
// XCDs round-robin (block b runs on XCD b % 8), the L2s of different XCDs are not coherent with
// each other, so every replica lives on ONE XCD — its waves see each other's writes through
// their shared L2 instead of overwriting each other's hot lines at write-back.  Replicas are
// averaged after each pass (hm_linear_mix_*), as Hivemall averages its mappers.
// Measured (profiles/linear_shared_r2.log): one table for the whole chip keeps ~1/concurrency of
// the updates of the hot features of a Zipf stream (held-out logloss 0.665 vs the sequential
// 0.479 at 8192 waves); float-atomic deltas lose nothing but serialise on the hot addresses
// (1.7 M rows/s) and diverge from stale AdaGrad state.
// RELOAD re-reads a feature's state right before updating it (shorter read-modify-write window).
// NT reads the model with non-temporal loads, which bypass the CU's L1: a CU's L1 is never
// refreshed by other CUs' stores, so plain loads of a hot feature keep returning the copy the
// CU first cached while the other CUs of the XCD update it in L2.
// Per-wave scalars (online target variance, Eve) live in RSW [W][8].  Non-covariance binary /
// regression rules only (covariance learners keep one replica per wave, mixed by argmin-KLD).
typedef float f4v __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ F4 ld4m(const float4* p) {
    if constexpr (NT) {
        const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
        return F4{v.x, v.y, v.z, v.w};
    } else {
        return ld4(p);
    }
}

// HOT: the hottest features (hot_slot[i] >= 0, at most HM_HOT_MAX, chosen by the host from the
// pass's feature counts) are not read-modify-written per row: each block sums their gradients
// (sum g, sum g^2, count) in LDS over a chunk of CH rows per wave, then applies them with one
// float atomic on G and one on w per touched hot feature (AdaGrad of the general learner, no or L2
// regularisation; AdaGrad-RDA: atomics on its two sums, w recomputed).  Plain SGD would apply
// a block's summed gradient at full rate and diverge, so it stays Hogwild.  No update of a hot feature is lost, and the atomics on its
// address drop by 4*CH x.  Cold features keep the Hogwild read-modify-write.
constexpr int HM_HOT_MAX = 8192;          // <= 96 KB of LDS accumulators


// Flush of up to 4 hot features per thread: all returning atomics are issued before any result
// is used, so their round trips overlap instead of running back to back.
constexpr int HM_HOT_U = 4;

// The rules whose hot-feature gradients are pre-aggregated (hot_flush4): the general learner's
// AdaGrad with no / L2 regularisation and AdaGrad-RDA (its running sums).  Applying a block's
// MEAN gradient through the other rules' own updates was measured and rejected: momentum /
// Adam-family / RMSprop-Graves diverge (held-out logloss +0.3 .. +29 vs sequential at 2^24,
// profiles/r4/linear_rules_mean_step.jsonl); those rules run plain Hogwild with a per-rule cap
// on the rows in flight (ops/linear.py RULE_WAVES).
__host__ __device__ __forceinline__ bool hot_rda(const Params& P) { return P.reg == R_RDA && P.opt == O_ADAGRAD; }
__host__ __device__ __forceinline__ bool hot_sum_rule(const Params& P) {
    return P.algo == A_GENERAL && P.opt == O_ADAGRAD && (P.reg == R_NO || P.reg == R_L2 || P.reg == R_RDA);
}

__device__ __forceinline__ void hot_flush4(const Params& P, float4* __restrict__ S, float (&gs)[HM_HOT_U],
                                           float (&g2)[HM_HOT_U], const float (&cnt)[HM_HOT_U],
                                           const int (&f)[HM_HOT_U], const StepK& k) {
    // the RDA sums and the weight deltas are non-returning atomics (they retire at L2 without the
    // issuing wave waiting); AdaGrad's accumulator add returns the value it found
    if (P.reg == R_L2) {
#pragma unroll
        for (int u = 0; u < HM_HOT_U; ++u) {
            if (f[u] < 0) continue;
            const float lw = P.lambda * __builtin_nontemporal_load(&S[f[u]].x);
            g2[u] += 2.f * lw * gs[u] + cnt[u] * lw * lw;
            gs[u] += cnt[u] * lw;
        }
    }
    if (hot_rda(P)) {
        // AdaGrad-RDA: only the running sums u = sum g, G = sum g^2 are stored; a hot
        // feature's w is recomputed from them where it is read (rda_w) and once after the pass
#pragma unroll
        for (int u = 0; u < HM_HOT_U; ++u) {
            if (f[u] < 0) continue;
            atomicAdd(&S[f[u]].y, gs[u]);
            atomicAdd(&S[f[u]].z, g2[u]);
        }
    } else if (P.opt == O_ADAGRAD) {
        // the accumulator's value BEFORE this block's add comes back from the atomic: blocks that
        // flush one feature at once are serialised there and each normalises by every earlier
        // block's squared gradients, as the sequential learner would.  (A separately loaded G
        // let up to all blocks normalise by the same stale G: early in a pass, G ~ 0, that is a
        // step sqrt(#blocks) too large — held-out logloss +0.006 .. +0.77 for -reg no.)
        float G0[HM_HOT_U];
#pragma unroll
        for (int u = 0; u < HM_HOT_U; ++u)
            G0[u] = f[u] >= 0 ? atomicAdd(&S[f[u]].y, g2[u]) : 0.f;
#pragma unroll
        for (int u = 0; u < HM_HOT_U; ++u) {
            if (f[u] < 0) continue;
            atomicAdd(&S[f[u]].x, -k.eta * gs[u] / (sqrtf(G0[u] + g2[u]) + P.eps));
        }
    }
}

// AdaGrad-RDA weight from its sums at step t (optimizer_update O_ADAGRAD_RDA)
__device__ __forceinline__ float rda_w(const Params& P, float u, float G, const StepK& k) {
    if (G <= 0.f) return 0.f;
    const float sign = u > 0.f ? 1.f : -1.f;
    const float mean = sign * u / k.t - P.lambda;
    return mean < 0.f ? 0.f : -sign * k.eta * k.t * mean / sqrtf(G);
}

// AdaGrad with L1 / elastic-net regularisation keeps its hot features in "owner" mode (its
// sign(w) term is not a function of summed gradients, so hot_flush4's atomics do not apply): the
// blocks add their per-chunk sums (sum g, sum g^2, rows) to a global accumulator per hot feature
// (non-returning atomics, nothing lost), and ONE thread of the grid owns each hot feature: at
// every chunk end it takes the accumulated sums (atomic exchange) and applies the n-step update
// (hot_nstep) with plain read-modify-write — a single writer, so no update is lost and none is
// applied twice.  Rows still read the hot weights Hogwild (stale by at most a chunk).  One table
// (R = 1) only.  Closed forms of the same n steps for SGD, momentum, RMSprop(-Graves), AdaDelta
// and the Adam family were measured and removed: without the sequential learner's feedback a
// chunk's thousands of steps diverge (profiles/r4/linear_rules_owner_all_rules.jsonl).
__host__ __device__ __forceinline__ bool hot_owner_rule(const Params& P) {
    return P.algo == A_GENERAL && P.opt == O_ADAGRAD && (P.reg == R_L1 || P.reg == R_ELASTIC);
}

// n sequential AdaGrad steps on one feature with the chunk's mean gradient a = sum g / n and mean
// squared gradient b = sum g^2 / n, regularisation evaluated at the state the owner read:
// G += n b; w moves by eta a sum_i 1 / sqrt(G0 + i b) ~ eta a 2n / (sqrt(G_n) + sqrt(G0)) (the
// integral of the normaliser, exact in the limit of many small steps).
__device__ __forceinline__ void hot_nstep(const Params& P, F4& s, float gsum, float g2sum, float n, const StepK& k) {
    if (n <= 0.f) return;
    const float r = P.reg == R_L1 ? P.lambda * sgnf(s.w)
                                  : P.lambda * (P.l1_ratio * sgnf(s.w) + (1.f - P.l1_ratio) * s.w);
    const float a0 = gsum / n;
    const float a = a0 + r;
    const float b = fmaxf(g2sum / n + 2.f * a0 * r + r * r, 0.f);
    const float G0 = s.s1, Gn = G0 + n * b;
    s.w -= k.eta * a * 2.f * n / (sqrtf(Gn) + sqrtf(G0) + 2.f * P.eps);
    s.s1 = Gn;
}

// Block barrier over the LDS accumulators only: waits for this wave's LDS operations, not for
// its outstanding global atomics (a __syncthreads fence would drain those too)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// LDS accumulators, structure of arrays: sum g [H] | sum g^2 [H] | rows [H]
__device__ __forceinline__ void hot_add(float* acc, int H, int h, float g) {
    atomicAdd(acc + h, g);
    atomicAdd(acc + H + h, g * g);
    atomicAdd(acc + 2 * H + h, 1.f);
}

template <bool RELOAD, bool NT, bool HOT>
__global__ __launch_bounds__(256) void linear_shared_kernel(
    Params P, int64_t n_rows, int dims, int64_t t0, int W, int R, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ idx, const float* __restrict__ val, const float* __restrict__ y,
    const int32_t* __restrict__ order, float4* __restrict__ S0, uint8_t* __restrict__ touched0,
    float* __restrict__ RSW, double* __restrict__ loss_out, const int32_t* __restrict__ hot_slot,
    const int32_t* __restrict__ hot_feat, int H, int CH, int min_rows, int every, float4* __restrict__ hacc) {
    extern __shared__ float s_acc[];             // HOT: 3 x H floats, see hot_add
    const bool owner = HOT && hacc != nullptr;   // hot features in owner mode (hot_owner_rule)
    const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc(S0, (short)0, -1, 0x00020000);
    auto store = [&](float4* p, const F4& v) { st4(p, v); };
    const int lane = threadIdx.x & 63;
    const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
    const bool active = g < W;
    if (!HOT && !active) return;                 // wave-uniform: the whole wave leaves
    // replica: XCD x = block % 8 owns replicas x, x + 8, ...; R = 1 or a multiple of 8
    const int b = blockIdx.x;
    const int rep = R == 1 ? 0 : ((b >> 3) % (R >> 3)) * 8 + (b & 7);
    float4* __restrict__ S = S0 + (size_t)rep * dims;
    uint8_t* __restrict__ touched = touched0 + (size_t)rep * dims;
    float rs[HM_REP_SCALARS];
#pragma unroll
    for (int k = 0; k < HM_REP_SCALARS; ++k) rs[k] = active ? RSW[(size_t)g * HM_REP_SCALARS + k] : 0.f;
    if constexpr (HOT) {
        for (int h = threadIdx.x; h < 3 * H; h += 256) s_acc[h] = 0.f;
        lds_barrier();
    }
    double loss_acc = 0.0;
    const int ch = HOT ? CH : 1;
    const int64_t span = (int64_t)W * ch;
    const int64_t nchunks = (n_rows + span - 1) / span;
    for (int64_t ck = 0; ck < nchunks; ++ck) {
        for (int j = 0; j < ch && active; ++j) {
            const int64_t q = ck * span + (int64_t)j * W + g;
            if (q >= n_rows) break;
            const int64_t row = order ? (int64_t)order[q] : q;
            const int64_t s = indptr[row], e = indptr[row + 1];
            const float yy = y[row];
            const float t = (float)(t0 + q + 1);
            rs[RS_T] = t;
            const StepK sk = step_consts(P, t);
            int ci = -1, hs = -1;
            float cx = 0.f;
            if (s + lane < e) {
                ci = idx[s + lane];
                cx = val ? val[s + lane] : 1.f;
                if (ci < 0 || ci >= dims) ci = -1;
                if (HOT && ci >= 0) hs = hot_slot[ci];
            }
            F4 cst = {0.f, 0.f, 0.f, 0.f};
            float p = 0.f, sq = 0.f;
            const bool hrda = HOT && hot_rda(P);
            if (ci >= 0) {
                cst = ld4m<NT>(S + ci);
                p = (hrda && hs >= 0 ? rda_w(P, cst.s1, cst.s2, sk) : cst.w) * cx;
                sq = cx * cx;
            }
            for (int64_t k = s + 64 + lane; k < e; k += 64) {      // rows wider than a wave
                const int i = idx[k];
                const float x = val ? val[k] : 1.f;
                if (i < 0 || i >= dims) continue;
                const F4 st = ld4m<NT>(S + i);
                p += (hrda && hot_slot[i] >= 0 ? rda_w(P, st.s1, st.s2, sk) : st.w) * x;
                sq += x * x;
            }
            p = hm::wave_sum(p);
            sq = hm::wave_sum(sq);
            const RowCoef c = row_rule(P, p, yy, 0.f, sq, rs);
            loss_acc += c.loss;
            if (ci >= 0) {
                touched[ci] = 1;
                if (c.update) {
                    if (HOT && hs >= 0) {
                        hot_add(s_acc, H, hs, c.dloss * cx);
                    } else {
                        if (RELOAD) cst = ld4m<NT>(S + ci);
                        feature_update(P, c, cst, cx, sk, rs[RS_EVE_D]);
                        store(S + ci, cst);
                    }
                }
            }
            for (int64_t k = s + 64 + lane; k < e; k += 64) {
                const int i = idx[k];
                const float x = val ? val[k] : 1.f;
                if (i < 0 || i >= dims) continue;
                touched[i] = 1;
                if (!c.update) continue;
                if (HOT) {
                    const int h = hot_slot[i];
                    if (h >= 0) {
                        hot_add(s_acc, H, h, c.dloss * x);
                        continue;
                    }
                }
                F4 st = ld4m<NT>(S + i);
                feature_update(P, c, st, x, sk, rs[RS_EVE_D]);
                store(S + i, st);
            }
        }
        if constexpr (HOT) {
            // every wave of the block has finished its CH rows of this chunk
            lds_barrier();
            const int64_t tend = t0 + min(n_rows, (ck + 1) * span);
            const StepK sk = step_consts(P, (float)tend);
            // an entry is applied once it holds min_rows rows of this block (the hottest
            // features: every chunk), else every `every` chunks — staggered over the blocks, so
            // they do not all hit the same addresses in the same chunk — and at the end of the
            // pass: the global atomics on hot addresses bound the kernel
            const bool all = ((ck + blockIdx.x) % every) == every - 1 || ck == nchunks - 1;
            for (int h0 = threadIdx.x; h0 < H; h0 += 256 * HM_HOT_U) {
                float gs[HM_HOT_U], g2[HM_HOT_U], cnt[HM_HOT_U];
                int f[HM_HOT_U];
#pragma unroll
                for (int u = 0; u < HM_HOT_U; ++u) {
                    const int h = h0 + u * 256;
                    gs[u] = h < H ? s_acc[h] : 0.f;
                    g2[u] = h < H ? s_acc[H + h] : 0.f;
                    cnt[u] = h < H ? s_acc[2 * H + h] : 0.f;
                    // a hot feature whose rows all had a zero loss gradient needs no update —
                    // unless L2 decays it on every row that holds it (the sequential rule's
                    // g = 0 + lambda w)
                    f[u] = (g2[u] != 0.f || ((P.reg == R_L2 || owner) && cnt[u] > 0.f)) && (all || cnt[u] >= (float)min_rows)
                               ? hot_feat[h] : -1;
                    if (f[u] >= 0) {
                        s_acc[h] = 0.f;
                        s_acc[H + h] = 0.f;
                        s_acc[2 * H + h] = 0.f;
                    }
                }
                if (owner) {
#pragma unroll
                    for (int u = 0; u < HM_HOT_U; ++u) {
                        if (f[u] < 0) continue;
                        float4* A = hacc + h0 + u * 256;
                        atomicAdd(&A->x, gs[u]);
                        atomicAdd(&A->y, g2[u]);
                        atomicAdd(&A->z, cnt[u]);
                    }
                } else {
                    hot_flush4(P, S, gs, g2, cnt, f, sk);
                }
            }
            lds_barrier();
            if (owner) {
                // the hot features this thread owns: h = block + gridDim.x * (thread + 256 j).
                // Bounded skew: another block's (x, y, z) adds are three atomics to
                // different words, so one block's chunk can straddle this exchange — its count in
                // this drain and its gradient sums in the next, or the reverse.  Nothing is lost
                // (every add lands in exactly one drain); the split moves one block-chunk's
                // contribution (<= 32 rows per wave) between two consecutive n-step applications
                // of the feature, i.e. the mean gradient of a drain is off by at most that share.
                for (int h = blockIdx.x + gridDim.x * threadIdx.x; h < H; h += gridDim.x * 256) {
                    const float n = atomicExch(&hacc[h].z, 0.f);
                    if (n <= 0.f) continue;
                    const float gsum = atomicExch(&hacc[h].x, 0.f);
                    const float g2sum = atomicExch(&hacc[h].y, 0.f);
                    float4* p = S + hot_feat[h];
                    F4 st = ld4m<true>(p);
                    hot_nstep(P, st, gsum, g2sum, n, sk);
                    // write-through (SC1): the line leaves this XCD's L2, so the other XCDs'
                    // next reads of the hot feature fetch it (the cold features' stores stay plain)
                    if (dims <= (1 << 28))
                        __builtin_amdgcn_raw_buffer_store_b128(
                            (__attribute__((ext_vector_type(4))) uint32_t){__float_as_uint(st.w), __float_as_uint(st.s1),
                                                                            __float_as_uint(st.s2), __float_as_uint(st.s3)},
                            rs0, (uint32_t)((const char*)p - (const char*)S0), 0, 16);
                    else
                        st4(p, st);
                }
            }
        }
    }
    if (active && lane == 0) {
#pragma unroll
        for (int k = 0; k < HM_REP_SCALARS; ++k) RSW[(size_t)g * HM_REP_SCALARS + k] = rs[k];
        loss_out[g] = loss_acc;
    }
}

// After a HOT AdaGrad-RDA pass: the stored w of every hot feature from its sums at the pass's
// last step (the value the next reader, prediction or export, must see).
__global__ __launch_bounds__(256) void hot_rda_finalize_kernel(Params P, float4* __restrict__ S0, int dims, int R,
                                                               const int32_t* __restrict__ hot_feat, int H,
                                                               float t) {
    const StepK k = step_consts(P, t);
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < (int64_t)H * R; q += (int64_t)gridDim.x * 256) {
        const int r = (int)(q / H), h = (int)(q - (int64_t)r * H);
        float4* s = S0 + (size_t)r * dims + hot_feat[h];
        s->x = rda_w(P, s->y, s->z, k);
    }
}

// After an owner-mode pass: the sums the owners had not taken yet (pushed after their last
// exchange) applied at the pass's last step.
__global__ __launch_bounds__(256) void hot_owner_final_kernel(Params P, float4* __restrict__ S, float4* __restrict__ hacc,
                                                              const int32_t* __restrict__ hot_feat, int H, float t,
                                                              const float* __restrict__ RSW) {
    const StepK k = step_consts(P, t);
    const int h = blockIdx.x * 256 + threadIdx.x;
    if (h >= H) return;
    const float4 A = hacc[h];
    hacc[h] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (A.z <= 0.f) return;
    F4 st = ld4(S + hot_feat[h]);
    hot_nstep(P, st, A.x, A.y, A.z, k);
    st4(S + hot_feat[h], st);
}

// Near-sequential shared-table pass (the "seq" engine): Hivemall's per-row rule
// for every optimizer at -mini_batch 1 on ONE table, W rows in flight.  Row q goes to wave q % W,
// so the rows in flight are always W consecutive rows of the stream (the sequential learner's
// order, each row reading the state up to W - 1 rows stale).  Per wave the rows are software-
// pipelined as in linear_train_kernel: the next row's CSR bounds, first-chunk indices / values and
// label are loaded while this row computes, so a row waits on one dependent round trip (its state
// gather) instead of the shared kernel's three (order -> indptr -> idx -> S; 1.7 M rows/s at 8
// rows in flight).  One-wave blocks; with spread = 8 only every 8th block works, which puts all W
// waves on one XCD under round-robin placement (speed / staleness only, never correctness): its
// L2 is then the one coherent copy every wave reads and writes, instead of 8 write-back L2s whose
// dirty lines the other XCDs do not see (docs/perf_notes.md, the FFM XCD probe: 8 blocks on one
// XCD +1.3e-4 vs +4.3e-3 on 8).  NT loads bypass the CU's L1, which other CUs' stores never refresh.
template <bool NT>
__global__ __launch_bounds__(64) void linear_seq_kernel(
    Params P, int64_t n_rows, int dims, int64_t t0, int W, int spread, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ idx, const float* __restrict__ val, const float* __restrict__ y,
    const int32_t* __restrict__ order, float4* __restrict__ S, uint8_t* __restrict__ touched,
    float* __restrict__ RSW, double* __restrict__ loss_out) {
    const int b = blockIdx.x;
    if (b % spread) return;
    const int g = b / spread;
    if (g >= W) return;
    const int lane = threadIdx.x;
    float rs[HM_REP_SCALARS];
#pragma unroll
    for (int k = 0; k < HM_REP_SCALARS; ++k) rs[k] = RSW[(size_t)g * HM_REP_SCALARS + k];
    double loss_acc = 0.0;
    auto row_of = [&](int64_t q) -> int64_t { return order ? (int64_t)order[q] : q; };
    int64_t cs = 0, ce = 0, pb_s = 0, pb_e = 0;
    int pci = -1;
    float pcx = 0.f, pyy = 0.f;
    if (g < n_rows) {
        const int64_t row0 = row_of(g);
        cs = indptr[row0];
        ce = indptr[row0 + 1];
        if (lane < (int)(ce - cs)) {
            pci = idx[cs + lane];
            pcx = val ? val[cs + lane] : 1.f;
        }
        pyy = y[row0];
        if (g + W < n_rows) {
            const int64_t row1 = row_of(g + W);
            pb_s = indptr[row1];
            pb_e = indptr[row1 + 1];
        }
    }
    for (int64_t q = g; q < n_rows; q += W) {
        const int64_t s = cs, e = ce;
        const int nnz = (int)(e - s);
        const float yy = pyy;
        const float t = (float)(t0 + q + 1);
        rs[RS_T] = t;
        const StepK sk = step_consts(P, t);
        int ci = pci;
        float cx = pcx;
        if (lane >= nnz || ci < 0 || ci >= dims) { ci = -1; cx = 0.f; }
        // ---- the state gather first (the one round trip the row waits on), then the prefetch ----
        F4 cst = {0.f, 0.f, 0.f, 0.f};
        if (ci >= 0) cst = ld4m<NT>(S + ci);
        cs = pb_s;
        ce = pb_e;
        pci = -1;
        pcx = 0.f;
        if (q + W < n_rows) {
            const int n1 = (int)(ce - cs);
            if (lane < n1) {
                pci = idx[cs + lane];
                pcx = val ? val[cs + lane] : 1.f;
            }
            pyy = y[row_of(q + W)];
            if (q + 2 * (int64_t)W < n_rows) {
                const int64_t row2 = row_of(q + 2 * (int64_t)W);
                pb_s = indptr[row2];
                pb_e = indptr[row2 + 1];
            }
        }
        float p = 0.f, sq = 0.f;
        if (ci >= 0) {
            p = cst.w * cx;
            sq = cx * cx;
            touched[ci] = 1;
        }
        for (int64_t k = s + 64 + lane; k < e; k += 64) {      // rows wider than a wave
            const int i = idx[k];
            const float x = val ? val[k] : 1.f;
            if (i < 0 || i >= dims) continue;
            const F4 st = ld4m<NT>(S + i);
            p += st.w * x;
            sq += x * x;
            touched[i] = 1;
        }
        p = hm::wave_sum(p);
        sq = hm::wave_sum(sq);
        const RowCoef c = row_rule(P, p, yy, 0.f, sq, rs);
        loss_acc += c.loss;
        if (!c.update) continue;
        if (ci >= 0) {
            feature_update(P, c, cst, cx, sk, rs[RS_EVE_D]);
            st4(S + ci, cst);
        }
        for (int64_t k = s + 64 + lane; k < e; k += 64) {
            const int i = idx[k];
            const float x = val ? val[k] : 1.f;
            if (i < 0 || i >= dims) continue;
            F4 st = ld4m<NT>(S + i);
            feature_update(P, c, st, x, sk, rs[RS_EVE_D]);
            st4(S + i, st);
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < HM_REP_SCALARS; ++k) RSW[(size_t)g * HM_REP_SCALARS + k] = rs[k];
        loss_out[g] = loss_acc;
    }
}

}  // namespace

// Near-sequential pass (linear_seq_kernel): one table S f32 [dims][4], touched u8 [dims], W waves
// (RSW f32 [W][8], loss_out f64 [W]); spread 1 (waves dealt over every XCD) or 8 (one XCD).
HM_API int hm_linear_train_seq(const Params* P, int64_t n_rows, int dims, int64_t t0, int W, int spread, int nt,
                               const int64_t* indptr, const int32_t* idx, const float* val, const float* y,
                               const int32_t* order, float* S, uint8_t* touched, float* RSW, double* loss_out,
                               hipStream_t stream) {
    if (n_rows <= 0) return 0;
    if (W <= 0 || W > 65536 || dims <= 0 || (spread != 1 && spread != 8) || P->n_labels != 1 || has_covar(P->algo))
        return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)(W * spread));
    if (nt)
        hipLaunchKernelGGL((linear_seq_kernel<true>), grid, dim3(64), 0, stream, *P, n_rows, dims, t0, W, spread,
                           indptr, idx, val, y, order, reinterpret_cast<float4*>(S), touched, RSW, loss_out);
    else
        hipLaunchKernelGGL((linear_seq_kernel<false>), grid, dim3(64), 0, stream, *P, n_rows, dims, t0, W, spread,
                           indptr, idx, val, y, order, reinterpret_cast<float4*>(S), touched, RSW, loss_out);
    HM_LAUNCH_RET();
}

// ip: R, dims, L, mini_batch, touched_cap, (n_rows as int64 separately)
HM_API int hm_linear_train(const Params* P, const int32_t* ip, int64_t n_rows,
                           const int64_t* indptr, const int32_t* idx, const float* val,
                           const float* y, const int32_t* order, float* S, uint8_t* touched,
                           float* RS, double* loss_out, float* gacc, int32_t* tlist,
                           hipStream_t stream) {
    LinLaunch G;
    G.R = ip[0]; G.dims = ip[1]; G.L = ip[2]; G.mini_batch = ip[3]; G.touched_cap = ip[4];
    G.n_rows = n_rows;
    if (G.R <= 0 || G.dims <= 0 || G.L <= 0) return (int)hipErrorInvalidValue;
    if (G.mini_batch > 1 && (gacc == nullptr || tlist == nullptr || G.touched_cap < 64 * 8))
        return (int)hipErrorInvalidValue;
    const size_t mbytes = (size_t)G.L * G.dims * sizeof(float4);
    G.lds_model = mbytes <= 64 * 1024;
    if (G.lds_model) {
        hipLaunchKernelGGL((linear_train_kernel<true>), dim3(G.R), dim3(64), mbytes, stream, *P, G,
                           indptr, idx, val, y, order, reinterpret_cast<float4*>(S), touched, RS,
                           loss_out, reinterpret_cast<float2*>(gacc), tlist);
    } else {
        hipLaunchKernelGGL((linear_train_kernel<false>), dim3(G.R), dim3(64), 0, stream, *P, G,
                           indptr, idx, val, y, order, reinterpret_cast<float4*>(S), touched, RS,
                           loss_out, reinterpret_cast<float2*>(gacc), tlist);
    }
    HM_LAUNCH_RET();
}

HM_API int hm_linear_mix_reduce(const float* S, const uint8_t* touched, int R, int dims, int L,
                                int kld, float* num, float* den, float* cnt, hipStream_t stream) {
    const size_t n = (size_t)L * dims;
    int blocks = (int)((n + 255) / 256);
    blocks = blocks > 8192 ? 8192 : (blocks < 1 ? 1 : blocks);
    hipLaunchKernelGGL(linear_mix_reduce_kernel, dim3(blocks), dim3(256), 0, stream,
                       reinterpret_cast<const float4*>(S), touched, R, dims, L, kld, num, den, cnt);
    HM_LAUNCH_RET();
}

HM_API int hm_linear_mix_apply(float* S, int R, int dims, int L, int kld, const float* num,
                               const float* den, const float* cnt, float* w_out, float* cov_out,
                               hipStream_t stream) {
    const size_t n = (size_t)L * dims;
    int blocks = (int)((n + 255) / 256);
    blocks = blocks > 8192 ? 8192 : (blocks < 1 ? 1 : blocks);
    hipLaunchKernelGGL(linear_mix_apply_kernel, dim3(blocks), dim3(256), 0, stream,
                       reinterpret_cast<float4*>(S), R, dims, L, kld, num, den, cnt, w_out, cov_out);
    HM_LAUNCH_RET();
}

HM_API int hm_linear_predict(const float* w, int dims, int L, const int64_t* indptr,
                             const int32_t* idx, const float* val, int64_t n_rows, float* out,
                             const float* cov, float* var_out, hipStream_t stream) {
    const int64_t total = n_rows * L;
    if (total <= 0) return 0;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(linear_predict_kernel, dim3((int)blocks), dim3(256), 0, stream, w, dims, L,
                       indptr, idx, val, n_rows, out, cov, var_out);
    HM_LAUNCH_RET();
}

// Shared-table Hogwild pass (see linear_shared_kernel).  S f32 [R][dims][4], touched u8
// [R][dims]; W waves (RSW f32 [W][8], loss_out f64 [W]); R = 1 or a multiple of 8 with W / 4 >= R
// workgroups so that every replica gets waves.
// ---------------------------------------------------------------------------------------------
// Mini-batch engine (the general learner's -mini_batch M > 1 on one shared table): Hivemall's
// mini-batch rule, as the sequential engines run it (csrc/host/linear_cpu.cpp train_replica):
// the M rows of a batch are scored against the SAME weights, each row's dloss * x is summed per
// feature, and at the batch end every touched feature takes ONE optimizer step with the batch's
// mean gradient (sum / M) at the step t of the batch's last row.  The rows of a batch are
// independent given the weights, so the whole chip works on one batch at a time:
//   mb_grad:  one wave per row: gather w, dot, row rule; float atomics add dloss * x into GA[i];
//             the first toucher of a feature (atomicOr on its mark) appends it to the batch list;
//   mb_apply: one thread per listed feature: optimizer_update with GA[i] / M, clears GA / mark.
// Two launches per batch, no host sync.  Exact up to the order of the fp32 gradient sums.
// Eve (a per-row loss feedback chain) is not a batch rule and is refused.
__global__ __launch_bounds__(256) void linear_mb_grad_kernel(
    Params P, int dims, int64_t b0, int64_t b1, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ idx, const float* __restrict__ val, const float* __restrict__ y,
    const int32_t* __restrict__ order, const float4* __restrict__ S, uint8_t* __restrict__ touched,
    float* __restrict__ GA, uint32_t* __restrict__ mark, int32_t* __restrict__ list, int32_t* __restrict__ cnt,
    double* __restrict__ loss_out) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
    float rs[HM_REP_SCALARS] = {};
    double lsum = 0.0;
    for (int64_t q = b0 + w0; q < b1; q += nw) {
        const int64_t row = order ? (int64_t)order[q] : q;
        const int64_t s = indptr[row], e = indptr[row + 1];
        float p = 0.f;
        for (int64_t k = s + lane; k < e; k += 64) {
            const int i = idx[k];
            if (i < 0 || i >= dims) continue;
            p += S[i].x * (val ? val[k] : 1.f);
        }
        p = hm::wave_sum(p);
        const RowCoef c = row_rule(P, p, y[row], 0.f, 0.f, rs);
        lsum += c.loss;
        for (int64_t k = s + lane; k < e; k += 64) {
            const int i = idx[k];
            if (i < 0 || i >= dims) continue;
            touched[i] = 1;
            if (!c.update) continue;
            atomicAdd(GA + i, c.dloss * (val ? val[k] : 1.f));
            if (atomicOr(mark + i, 1u) == 0u) list[atomicAdd(cnt, 1)] = i;
        }
    }
    if (lane == 0 && lsum != 0.0) atomicAdd(loss_out, lsum);
}

__global__ __launch_bounds__(256) void linear_mb_apply_kernel(
    Params P, float4* __restrict__ S, float* __restrict__ GA, uint32_t* __restrict__ mark,
    const int32_t* __restrict__ list, const int32_t* __restrict__ cnt, int32_t* __restrict__ cnt_next,
    float t_last, float inv) {
    const int n = *cnt;
    const StepK sk = step_consts(P, t_last);
    for (int k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
        const int i = list[k];
        F4 st = ld4(S + i);
        optimizer_update(P, st, GA[i] * inv, sk, 1.f);
        st4(S + i, st);
        GA[i] = 0.f;
        mark[i] = 0u;
    }
    // the counter the NEXT batch appends to (its last reader was the previous apply launch)
    if (blockIdx.x == 0 && threadIdx.x == 0) *cnt_next = 0;
}

// One pass of the mini-batch engine over n_rows (step of row q = t0 + q + 1).  GA f32 [dims] and
// mark u32 [dims] zeroed (left zeroed again at the end), list i32 [cap >= min(dims, M * max nnz)],
// cnt i32 [2] (zeroed here).
HM_API int hm_linear_train_minibatch(const Params* P, int64_t n_rows, int dims, int64_t t0, int M,
                                     const int64_t* indptr, const int32_t* idx, const float* val,
                                     const float* y, const int32_t* order, float* S, uint8_t* touched,
                                     float* GA, uint32_t* mark, int32_t* list, int32_t* cnt,
                                     double* loss_out, hipStream_t stream) {
    if (n_rows <= 0) return 0;
    if (M <= 1 || dims <= 0 || P->n_labels != 1 || P->algo != A_GENERAL || P->opt == O_EVE)
        return (int)hipErrorInvalidValue;
    const int gb = (int)((M + 3) / 4 < 4096 ? (M + 3) / 4 : 4096);     // one wave per row
    // both batch counters start at 0 (the last batch of a previous pass leaves its own set)
    const hipError_t ze = hipMemsetAsync(cnt, 0, 2 * sizeof(int32_t), stream);
    if (ze != hipSuccess) return (int)ze;
    int b = 0;
    for (int64_t b0 = 0; b0 < n_rows; b0 += M, ++b) {
        const int64_t b1 = b0 + M < n_rows ? b0 + M : n_rows;
        int32_t* c = cnt + (b & 1);
        int32_t* cn = cnt + ((b + 1) & 1);
        hipLaunchKernelGGL(linear_mb_grad_kernel, dim3(gb), dim3(256), 0, stream, *P, dims, b0, b1, indptr, idx, val, y,
                           order, reinterpret_cast<const float4*>(S), touched, GA, mark, list, c, loss_out);
        hipLaunchKernelGGL(linear_mb_apply_kernel, dim3(1024), dim3(256), 0, stream, *P, reinterpret_cast<float4*>(S),
                           GA, mark, list, c, cn, (float)(t0 + b1), 1.f / (float)(b1 - b0));
    }
    HM_LAUNCH_RET();
}

HM_API int hm_linear_train_shared(const Params* P, int64_t n_rows, int dims, int64_t t0, int W, int R,
                                  int reload, int nt, const int64_t* indptr, const int32_t* idx, const float* val,
                                  const float* y, const int32_t* order, float* S, uint8_t* touched,
                                  float* RSW, double* loss_out, const int32_t* hot_slot, const int32_t* hot_feat,
                                  int H, int CH, int min_rows, int every, float* hacc,
                                  hipStream_t stream) {
    if (n_rows <= 0) return 0;
    if (W <= 0 || dims <= 0 || P->n_labels != 1 || has_covar(P->algo)) return (int)hipErrorInvalidValue;
    if (R != 1 && (R % 8 != 0 || (W + 3) / 4 < R)) return (int)hipErrorInvalidValue;
    const bool hot = H > 0;
    const size_t lds = hot ? (size_t)H * 3 * sizeof(float) : 0;
    // hot features: pre-aggregated sums (hot_sum_rule), or owner mode (hot_owner_rule, R = 1, with
    // the zeroed float4 [H] accumulators hacc)
    const bool own = hot && hacc != nullptr;
    if (hot && (hot_slot == nullptr || hot_feat == nullptr || H > HM_HOT_MAX || CH <= 0 || min_rows <= 0 || every <= 0 ||
                !(own ? (hot_owner_rule(*P) && R == 1) : hot_sum_rule(*P))))
        return (int)hipErrorInvalidValue;
#define HM_SHARED_LAUNCH(RL, NTT, HT)                                                                  \
    hipLaunchKernelGGL((linear_shared_kernel<RL, NTT, HT>), dim3((W + 3) / 4), dim3(256), lds, stream, *P, n_rows, \
                       dims, t0, W, R, indptr, idx, val, y, order, reinterpret_cast<float4*>(S), touched,   \
                       RSW, loss_out, hot_slot, hot_feat, H, CH, min_rows, every,                       \
                       own ? reinterpret_cast<float4*>(hacc) : nullptr)
    if (hot) {
        if (reload && nt) HM_SHARED_LAUNCH(true, true, true);
        else if (reload) HM_SHARED_LAUNCH(true, false, true);
        else if (nt) HM_SHARED_LAUNCH(false, true, true);
        else HM_SHARED_LAUNCH(false, false, true);
        if (own) {
            hipLaunchKernelGGL(hot_owner_final_kernel, dim3((unsigned)((H + 255) / 256)), dim3(256), 0, stream, *P,
                               reinterpret_cast<float4*>(S), reinterpret_cast<float4*>(hacc), hot_feat, H,
                               (float)(t0 + n_rows), RSW);
        } else if (hot_rda(*P)) {
            const int64_t tot = (int64_t)H * R;
            hipLaunchKernelGGL(hot_rda_finalize_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, *P,
                               reinterpret_cast<float4*>(S), dims, R, hot_feat, H, (float)(t0 + n_rows));
        }
    } else {
        if (reload && nt) HM_SHARED_LAUNCH(true, true, false);
        else if (reload) HM_SHARED_LAUNCH(true, false, false);
        else if (nt) HM_SHARED_LAUNCH(false, true, false);
        else HM_SHARED_LAUNCH(false, false, false);
    }
#undef HM_SHARED_LAUNCH
    HM_LAUNCH_RET();
}
