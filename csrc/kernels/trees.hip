// Histogram tree learning + batched tree inference for gfx950 (RandomForest / GBT).
//
// Upstream (core/src/main/java/hivemall/smile/classification/
// {DecisionTree,RandomForestClassifierUDTF,GradientTreeBoostingClassifierUDTF}.java,
// smile/regression/RegressionTree.java, smile/tools/TreePredictUDF.java) grows trees with
// exact splits over pre-sorted columns.  This engine uses LightGBM/XGBoost-hist style
// quantised splits instead (documented in docs/compat.md): features are quantised to <= 256
// bins (uint8), rows are kept grouped by tree node, and every level builds per-(node,
// feature, bin) sums of NS statistics (GBT: residual, hessian, count; RF: per-class
// bootstrap-weighted counts; regression: w·y, w).
//
// hist_build: the level's rows are grouped by node (rows[seg[k] .. seg[k+1]) belong to output
//   node k).  A fixed grid of blocks splits the position range [seg[0], seg[S]) into equal
//   chunks (the host never has to know the row count: no sync before the launch); a block walks
//   the node segments its chunk overlaps.  Per (block, node) piece: a large piece privatises the
//   feature group's histogram in LDS, laid out [f][s][b], as 32-bit FIXED-POINT sums
//   (ds_add_u32), and flushes the non-zero bins to the fp32 global histogram with float atomics;
//   a small piece (deep levels: few rows per node) adds straight to global memory.
//   Why fixed point: on gfx950 ds_add_f32 retires 0.33 lane-ops per CU-clock whatever the
//   address pattern, ds_add_u32 3.5 (random bins) to 8.4 (distinct addresses) — measured by
//   benchmarks/probes/lds_atomic_probe.hip (profiles/lds_atomic_probe_r1.jsonl).  The scale per
//   statistic is a power of two chosen in-kernel from the block's chunk length and max|stat|
//   (device array), so a block's partial sum cannot overflow 2^31; quantisation error per row
//   is <= max|stat| * 2^-17 at the root of an 11M-row HIGGS level.
//   Feature groups (4/8/16 features, one aligned load of the row's bins) keep the LDS image
//   <= 48 KB so three blocks share a CU.  The tree builder only histograms the smaller child of
//   every split and derives the sibling as parent - child (models/trees.py).
#include "common.h"

// Split-feature flag of a nominal (one-vs-rest) node: go left when x == threshold (prediction)
// or bin == split bin (training); ordinal nodes go left when x <= threshold / bin <= split bin.
#define HM_TREE_CAT 0x40000000
#define HM_TREE_DLEFT 0x20000000   // learned default direction: missing (NaN) goes left

namespace {


template <int FGW> struct BinWords;
template <> struct BinWords<1> { using T = uint32_t; };
template <> struct BinWords<2> { using T = uint2; };
template <> struct BinWords<4> { using T = uint4; };
struct alignas(32) U8W { uint4 a, b; };             // 32 features: one 32-B row of bins
template <> struct BinWords<8> { using T = U8W; };

// Rows handled per thread per step: all their loads are issued before the first atomic, so a
// wave keeps HIST_U row gathers (index -> stats + bin words) in flight instead of one.
constexpr int HIST_U = 4;

template <int NS, int FGW, bool GLOBAL, bool PK = false>
__device__ __forceinline__ void hist_rows(const uint8_t* __restrict__ bins, int dpad, int f0, int nf,
                                          int B, const int32_t* __restrict__ rows,
                                          const float* __restrict__ stats, int64_t s0, int64_t s1,
                                          float* __restrict__ h, const float* scale) {
    using W = typename BinWords<FGW>::T;
    for (int64_t q0 = s0 + threadIdx.x; q0 < s1; q0 += (int64_t)blockDim.x * HIST_U) {
        int64_t r[HIST_U];
#pragma unroll
        for (int u = 0; u < HIST_U; ++u) {
            const int64_t q = q0 + (int64_t)u * blockDim.x;
            r[u] = q < s1 ? (int64_t)rows[q] : -1;
        }
        float st[HIST_U][NS];
        uint32_t w[HIST_U][FGW];
#pragma unroll
        for (int u = 0; u < HIST_U; ++u) {
            if (r[u] >= 0) {
#pragma unroll
                for (int s = 0; s < NS; ++s) st[u][s] = stats[r[u] * NS + s];
                const W v = *reinterpret_cast<const W*>(bins + r[u] * dpad + f0);
                if constexpr (FGW == 1) {
                    w[u][0] = v;
                } else if constexpr (FGW == 2) {
                    w[u][0] = v.x; w[u][1] = v.y;
                } else if constexpr (FGW == 4) {
                    w[u][0] = v.x; w[u][1] = v.y; w[u][2] = v.z; w[u][3] = v.w;
                } else {
                    w[u][0] = v.a.x; w[u][1] = v.a.y; w[u][2] = v.a.z; w[u][3] = v.a.w;
                    w[u][4] = v.b.x; w[u][5] = v.b.y; w[u][6] = v.b.z; w[u][7] = v.b.w;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < HIST_U; ++u) {
            if (r[u] < 0) continue;
#pragma unroll
            for (int j = 0; j < FGW * 4; ++j) {
                if (j < nf) {
                    const int bin = (w[u][j >> 2] >> (8 * (j & 3))) & 0xff;
                    if constexpr (PK && !GLOBAL) {
                        // statistics 2p, 2p+1 as one 64-bit LDS add: lo + hi * 2^32 with lo
                        // sign-extended sums both exactly while |sum lo| < 2^31 (the fixed-point
                        // scale bounds every sum by 2^30); an odd last statistic is a 32-bit add
                        constexpr int NP = NS / 2;
                        unsigned long long* h64 = reinterpret_cast<unsigned long long*>(h);
#pragma unroll
                        for (int q = 0; q < NP; ++q) {
                            const long long lo = __float2int_rn(st[u][2 * q] * scale[2 * q]);
                            const long long hi = __float2int_rn(st[u][2 * q + 1] * scale[2 * q + 1]);
                            atomicAdd(h64 + (j * NP + q) * B + bin,
                                      (unsigned long long)(lo + (long long)((unsigned long long)hi << 32)));
                        }
                        if constexpr (NS & 1)
                            atomicAdd(reinterpret_cast<int*>(h64 + (size_t)nf * NP * B) + j * B + bin,
                                      __float2int_rn(st[u][NS - 1] * scale[NS - 1]));
                        continue;
                    }
#pragma unroll
                    for (int s = 0; s < NS; ++s) {
                        if constexpr (GLOBAL) {
                            if (st[u][s] != 0.f) atomicAdd(h + ((size_t)j * B + bin) * NS + s, st[u][s]);
                        } else {
                            atomicAdd(reinterpret_cast<int*>(h) + (j * NS + s) * B + bin,
                                      __float2int_rn(st[u][s] * scale[s]));
                        }
                    }
                }
            }
        }
    }
}

template <int NS, int FGW, int TPB = 256, bool PK = false>
__global__ __launch_bounds__(TPB) void hist_kernel(const uint8_t* __restrict__ bins, int d, int dpad,
                                                   int B, const int32_t* __restrict__ rows,
                                                   const int64_t* __restrict__ seg, int n_seg,
                                                   const float* __restrict__ stats,
                                                   const float* __restrict__ smax,
                                                   float* __restrict__ hist) {
    constexpr int FG = FGW * 4;
    extern __shared__ __attribute__((aligned(16))) float s_hist[];
    const int f0 = blockIdx.y * FG;
    const int nf = min(FG, d - f0);
    if (nf <= 0) return;
    const int64_t nblk = gridDim.x;
    const int64_t lo = seg[0], hi = seg[n_seg];
    const int64_t chunk = ((hi - lo + nblk - 1) / nblk + 255) / 256 * 256;
    const int64_t p0 = lo + (int64_t)blockIdx.x * chunk;
    const int64_t p1 = min(hi, p0 + chunk);
    if (p0 >= p1) return;
    // fixed-point scale per statistic: chunk * max|stat| * scale <= 2^30
    float scale[NS], inv[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const float m = fmaxf(smax[s], 1e-30f) * (float)chunk;
        const float e = fminf(fmaxf(floorf(log2f(1073741824.f / m)), -60.f), 60.f);
        scale[s] = exp2f(e);
        inv[s] = exp2f(-e);
    }
    // first node whose segment ends after p0
    int a = 0, b = n_seg - 1;
    while (a < b) {
        const int m = (a + b) >> 1;
        if (seg[m + 1] <= p0) a = m + 1; else b = m;
    }
    const int hsz = nf * NS * B;
    int* s_int = reinterpret_cast<int*>(s_hist);
    for (int k = a; k < n_seg; ++k) {
        if (seg[k] >= p1) break;
        const int64_t s0 = max(p0, seg[k]), s1 = min(p1, seg[k + 1]);
        if (s0 >= s1) continue;
        float* gh = hist + ((size_t)k * d + f0) * B * NS;
        if ((s1 - s0) * nf * 4 < hsz) {  // few rows: straight to global memory
            hist_rows<NS, FGW, true>(bins, dpad, f0, nf, B, rows, stats, s0, s1, gh, scale);
            continue;
        }
        for (int i = threadIdx.x; i < hsz; i += blockDim.x) s_int[i] = 0;
        __syncthreads();
        hist_rows<NS, FGW, false, PK>(bins, dpad, f0, nf, B, rows, stats, s0, s1, s_hist, scale);
        __syncthreads();
        if constexpr (PK) {
            constexpr int NP = NS / 2;
            const unsigned long long* s64 = reinterpret_cast<const unsigned long long*>(s_hist);
            for (int i = threadIdx.x; i < nf * NP * B; i += blockDim.x) {
                const long long v = (long long)s64[i];
                if (v == 0) continue;
                const int f = i / (NP * B);
                const int rem = i - f * NP * B;
                const int q = rem / B;
                const int bin = rem - q * B;
                const int lo = (int)(unsigned)(unsigned long long)v;
                const long long hi = (v - lo) >> 32;
                float* o = gh + ((size_t)f * B + bin) * NS + 2 * q;
                if (lo != 0) atomicAdd(o, (float)lo * inv[2 * q]);
                if (hi != 0) atomicAdd(o + 1, (float)hi * inv[2 * q + 1]);
            }
            if constexpr (NS & 1) {
                const int* s32 = reinterpret_cast<const int*>(s64 + (size_t)nf * NP * B);
                for (int i = threadIdx.x; i < nf * B; i += blockDim.x) {
                    const int v = s32[i];
                    if (v != 0) atomicAdd(gh + (size_t)i * NS + NS - 1, (float)v * inv[NS - 1]);
                }
            }
            __syncthreads();
            continue;
        }
        for (int i = threadIdx.x; i < hsz; i += blockDim.x) {
            const int v = s_int[i];
            if (v != 0) {
                const int f = i / (NS * B);
                const int rem = i - f * NS * B;
                const int s = rem / B;
                const int bin = rem - s * B;
                float iv = inv[0];
#pragma unroll
                for (int t = 1; t < NS; ++t) iv = s == t ? inv[t] : iv;
                atomicAdd(gh + ((size_t)f * B + bin) * NS + s, (float)v * iv);
            }
        }
        __syncthreads();
    }
}

// (Round 5, measured and removed: a feature-lane all-features histogram -- the image laid out
// [bin][32 features], each lane adding one feature of a staged row, so a wave's adds hit distinct
// banks whatever the bins.  Bank conflicts fell from 6.7 to 0.2-0.3 cycles per LDS instruction,
// but the kernel ran 1.5-2.0x slower (root 11 M x 28, NS = 2: 269 vs 178 us; GBDT 2.85-2.93 vs
// 2.09 ms per tree): the staging adds LDS instructions and the larger LDS footprint halves the
// blocks per CU.  docs/perf_notes.md, profiles/r5/hist_fl/.)
// Column |max| finish: every wave's maxima -> LDS -> one integer atomicMax per column per BLOCK
// (non-negative floats order like their bit patterns).  Per-wave atomics on the same 3 words
// serialised: 8,192 of them cost ~0.28 ms per 11M-row tree (profiles/gbt_r2/).
template <int NS>
__device__ __forceinline__ void block_absmax_flush(float (&m)[NS], float* __restrict__ out) {
    __shared__ float s_m[4][NS];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        float v = m[s];
        for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
        if (lane == 0) s_m[w][s] = v;
    }
    __syncthreads();
    if (threadIdx.x < NS) {
        const int s = threadIdx.x;
        const float v = fmaxf(fmaxf(s_m[0][s], s_m[1][s]), fmaxf(s_m[2][s], s_m[3][s]));
        atomicMax(reinterpret_cast<int*>(out) + s, __float_as_int(v));
    }
}

// out[s] = max_r |stats[r, s]| (out zeroed by the caller)
template <int NS>
__global__ __launch_bounds__(256) void absmax_kernel(const float* __restrict__ stats, int64_t n,
                                                     float* __restrict__ out) {
    float m[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) m[s] = 0.f;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
        for (int s = 0; s < NS; ++s) m[s] = fmaxf(m[s], fabsf(stats[r * NS + s]));
    }
    block_absmax_flush<NS>(m, out);
}

// Binary logistic boosting, one fused pass per tree (models/trees.py GBT, models/xgboost.py):
// p = sigmoid(F[r]) and, times the row's subsample mask (NULL = every row),
//   XGB = 0: GBT   stats[r] = {R = y - p, |R| (1 - |R|), 1}            (NS = 3)
//   XGB = 1: xgb   stats[r] = {g = p - y, max(p (1 - p), 1e-16)}       (NS = 2)
// plus the columns' |max| for the histogram's fixed-point scale (smax zeroed by the caller).
// Replaces ~8 tensor passes over n rows (sigmoid, sub, abs, clamp, stack, mask multiply, absmax).
// MODE 0: Friedman GBT {r, h, w}; 1: XGBoost {g, h}; 2: GBT with the split statistics {r w, w}
// only and h to hh [n] (the Newton leaf values are summed per leaf after the tree is grown,
// hm_gbt2_leaf_values: the histograms carry 2 statistics instead of 3).
template <int MODE>
__global__ __launch_bounds__(256) void gbt_stats_kernel(const float* __restrict__ F, const float* __restrict__ y,
                                                        const uint8_t* __restrict__ mask, int64_t n,
                                                        float* __restrict__ stats, float* __restrict__ smax,
                                                        float* __restrict__ hh) {
    constexpr int NS = MODE == 0 ? 3 : 2;
    float m[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) m[s] = 0.f;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        const float p = 1.f / (1.f + __expf(-F[r]));
        const float w = (mask == nullptr || mask[r]) ? 1.f : 0.f;
        float st[NS];
        if constexpr (MODE == 1) {
            st[0] = (p - y[r]) * w;
            st[1] = fmaxf(p * (1.f - p), 1e-16f) * w;
        } else {
            const float R = y[r] - p;
            const float aR = fabsf(R);
            st[0] = R * w;
            if constexpr (MODE == 0) {
                st[1] = aR * (1.f - aR) * w;
                st[2] = w;
            } else {
                st[1] = w;
                hh[r] = aR * (1.f - aR) * w;
            }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            stats[r * NS + s] = st[s];
            m[s] = fmaxf(m[s], fabsf(st[s]));
        }
    }
    block_absmax_flush<NS>(m, smax);
}

// Per-node sums {sum r, sum h} of the rows' final nodes (leaf[r] < T), block-private in LDS as
// 64-bit fixed point (r, h scaled by 2^24; |r| <= 1, h <= 1/4 for the logistic GBT): integer LDS
// adds instead of ds_add_f32 (~10x slower on gfx950), exact sums within the block.
constexpr float LEAF_FIX = 16777216.f;
constexpr int LEAF_BLOCKS = 1024;
template <typename NT>
__global__ __launch_bounds__(256) void leaf_sums_kernel(const NT* __restrict__ leaf, const float* __restrict__ st2,
                                                        const float* __restrict__ hh, int64_t n, int T,
                                                        float* __restrict__ sums) {
    extern __shared__ unsigned long long s_sum[];
    // one copy of the sums per wave when they fit (copies = 4: a tree's 256 leaves drew most of a
    // wave's 64 adds onto the same few words), folded into copy 0 at the end
    const int copies = 2 * T <= 2048 ? 4 : 1;
    for (int k = threadIdx.x; k < 2 * T * copies; k += blockDim.x) s_sum[k] = 0ull;
    __syncthreads();
    unsigned long long* my = s_sum + (copies > 1 ? (threadIdx.x >> 6) % copies : 0) * 2 * T;
    // LEAF_U rows per thread with every load issued before the first LDS add
    constexpr int LEAF_U = 8;
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r0 < n; r0 += step * LEAF_U) {
        int l[LEAF_U];
        float h[LEAF_U], g[LEAF_U];
#pragma unroll
        for (int u = 0; u < LEAF_U; ++u) {
            const int64_t r = r0 + u * step;
            const bool in = r < n;
            l[u] = in ? leaf[r] : -1;
            h[u] = in ? hh[r] : 0.f;
            g[u] = in ? st2[2 * r] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < LEAF_U; ++u) {
            // masked / inactive rows have no leaf; a saturated row (|r| = 1 in fp32: h = 0) still
            // adds its residual to the Newton numerator, as the host formulation does
            if (l[u] < 0 || l[u] >= T) continue;
            if (g[u] != 0.f) atomicAdd(&my[2 * l[u]], (unsigned long long)llrintf(g[u] * LEAF_FIX));
            if (h[u] != 0.f) atomicAdd(&my[2 * l[u] + 1], (unsigned long long)llrintf(h[u] * LEAF_FIX));
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < 2 * T; k += blockDim.x) {
        unsigned long long v = s_sum[k];
        for (int c = 1; c < copies; ++c) v += s_sum[c * 2 * T + k];
        if (v != 0ull) atomicAdd(sums + k, (float)(long long)v * (1.f / LEAF_FIX));
    }
}

// Bootstrap multiplicities (RandomForest bagging): the m draws with replacement over n rows are
// split into K chunks of c rows by a multinomial drawn on the host (exact: the chunk counts of m
// uniform draws), then block k draws its chunk's cnt[k] rows uniformly with a counter hash of
// (seed, k, j) and counts them in an LDS histogram.  Replaces torch.bincount over m random ids
// (450 µs for 11 M: global atomics onto random addresses) with LDS atomics.
constexpr int BOOT_CHUNK = 12288;
__global__ __launch_bounds__(1024) void bootstrap_counts_kernel(const int64_t* __restrict__ cnt, int64_t n, int c,
                                                                uint64_t seed, float* __restrict__ out) {
    __shared__ int s_h[BOOT_CHUNK];
    const int k = blockIdx.x;
    const int64_t r0 = (int64_t)k * c;
    const int len = (int)min((int64_t)c, n - r0);
    for (int i = threadIdx.x; i < len; i += blockDim.x) s_h[i] = 0;
    __syncthreads();
    const int64_t m = cnt[k];
    const uint32_t s0 = (uint32_t)seed, s1 = (uint32_t)(seed >> 32);
    for (int64_t j = threadIdx.x; j < m; j += blockDim.x) {
        // splitmix-style mix of (seed, chunk, draw)
        uint64_t z = ((uint64_t)(s0 ^ (uint32_t)k * 0x9E3779B9u) << 32 | (uint32_t)j) + (uint64_t)s1 * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const int i = (int)(((z >> 32) * (uint64_t)len) >> 32);
        atomicAdd(&s_h[i], 1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < len; i += blockDim.x) out[r0 + i] = (float)s_h[i];
}

// Leaf values of the nodes that are leaves (split_feat < 0): sum r / sum h (0 when sum h ~ 0).
__global__ __launch_bounds__(256) void leaf_newton_kernel(const float* __restrict__ sums, const int32_t* __restrict__ sf,
                                                          int T, float* __restrict__ vals) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= T || sf[k] >= 0) return;
    const float h = sums[2 * k + 1];
    vals[k] = fabsf(h) > 1e-12f ? sums[2 * k] / h : 0.f;
}

// F[r * ldf + k] += scale * vals[leaf[r] * ldv] for every routed row (leaf >= 0).
template <typename NT>
__global__ __launch_bounds__(256) void gbt_apply_kernel(float* __restrict__ F, int ldf, int k,
                                                        const float* __restrict__ vals, int ldv,
                                                        const NT* __restrict__ leaf, int64_t n, float scale) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        const int l = leaf[r];
        if (l >= 0) F[r * ldf + k] += scale * vals[(int64_t)l * ldv];
    }
}

// Flattened forest: node k of the forest has feature[k] (<0: leaf), threshold[k] (go left
// when x <= threshold), left[k]/right[k] (absolute node ids), value offset voff[k] into
// values (n_out floats per leaf).  roots[t] = root node of tree t.
__global__ __launch_bounds__(256) void tree_predict_kernel(
    const float* __restrict__ X, int64_t n, int d, const int32_t* __restrict__ feature,
    const float* __restrict__ threshold, const int32_t* __restrict__ left,
    const int32_t* __restrict__ right, const int32_t* __restrict__ voff,
    const float* __restrict__ values, const int32_t* __restrict__ roots, int n_trees, int n_out,
    float* __restrict__ out /* [n, n_trees, n_out] or summed [n, n_out] */, int sum_trees,
    const float* __restrict__ tree_w) {
    const int64_t total = n * (int64_t)n_trees;
    for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = g / n_trees;
        const int t = (int)(g - row * n_trees);
        int k = roots[t];
        const float* x = X + row * d;
        for (int depth = 0; depth < 64; ++depth) {
            int f = feature[k];
            if (f < 0) break;
            const bool cat = f & HM_TREE_CAT;
            const bool dl = f & HM_TREE_DLEFT;
            f &= ~(HM_TREE_CAT | HM_TREE_DLEFT);
            const float v = x[f];
            const float t = threshold[k];
            // NaN goes right (Smile: x <= t ? true : false; nominal: x == t ? true : false) unless
            // the split learned a default direction (XGBoost's sparsity-aware splits)
            k = (v != v) ? (dl ? left[k] : right[k]) : ((cat ? v == t : v <= t) ? left[k] : right[k]);
        }
        const float* val = values + voff[k];
        if (sum_trees) {
            const float w = tree_w ? tree_w[t] : 1.f;
            for (int o = 0; o < n_out; ++o) atomicAdd(out + row * n_out + o, w * val[o]);
        } else {
            float* dst = out + (row * n_trees + t) * n_out;
            for (int o = 0; o < n_out; ++o) dst[o] = val[o];
        }
    }
}

// Quantisation: bins[r, f] = #edges[f] < x  (edges sorted, n_edges per feature), NaN -> last bin.
__global__ __launch_bounds__(256) void quantize_kernel(const float* __restrict__ X, int64_t n,
                                                       int d, int dpad,
                                                       const float* __restrict__ edges,
                                                       int n_edges, uint8_t* __restrict__ bins) {
    const int64_t total = n * (int64_t)d;
    for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = g / d;
        const int f = (int)(g - r * d);
        const float v = X[g];
        const float* e = edges + (size_t)f * n_edges;
        int lo = 0, hi = n_edges;
        if (v != v) {
            lo = n_edges;
        } else {
            while (lo < hi) {  // first edge >= v
                const int mid = (lo + hi) >> 1;
                if (e[mid] < v) lo = mid + 1; else hi = mid;
            }
        }
        bins[r * dpad + f] = (uint8_t)lo;
    }
}

// Row routing after a level's splits: node_of_row[r] -> child id (or stays when the node
// became a leaf).  split_feat[node] < 0 means leaf; HM_TREE_CAT marks a nominal split.
// Bin of (row r, feature f) at bins[r * rs + f * cs]: row-major (rs = dpad, cs = 1) or the
// feature-major copy (rs = 1, cs = n), where a wave's rows read one 64-B run per distinct split
// feature instead of 64 whole 32-B rows.
// Latency-bound like route_count_kernel below (node -> split -> bins -> child per row): the split
// tables of nodes [lo, lo + ROUTE_TAB) in LDS and ROUTE_U rows per thread in flight; node ids
// below lo are leaves of earlier levels (or -1) and keep their id.
constexpr int ROUTE_U = 8;
constexpr int ROUTE_TAB = 1024;
template <typename NT>
__global__ __launch_bounds__(256) void route_kernel(const uint8_t* __restrict__ bins, int64_t n,
                                                    int64_t rs, int64_t cs, NT* __restrict__ node_of_row,
                                                    const int32_t* __restrict__ split_feat,
                                                    const int32_t* __restrict__ split_bin,
                                                    const int32_t* __restrict__ left_child,
                                                    const int32_t* __restrict__ right_child, int miss_bin,
                                                    int lo, int hi) {
    __shared__ int4 s_tab[ROUTE_TAB];          // {split_feat, split_bin, left, right} of node lo + i
    const int ntab = max(0, min(ROUTE_TAB, hi - lo));
    for (int i = threadIdx.x; i < ntab; i += blockDim.x)
        s_tab[i] = make_int4(split_feat[lo + i], split_bin[lo + i], left_child[lo + i], right_child[lo + i]);
    __syncthreads();
    const int G = gridDim.x;
    const int64_t chunk = (n + G - 1) / G;
    const int64_t r0 = (int64_t)blockIdx.x * chunk, r1 = min(n, r0 + chunk);
    for (int64_t q0 = r0 + threadIdx.x; q0 < r1; q0 += (int64_t)blockDim.x * ROUTE_U) {
        int nd[ROUTE_U], b[ROUTE_U];
        int4 t[ROUTE_U];
#pragma unroll
        for (int u = 0; u < ROUTE_U; ++u) {
            const int64_t q = q0 + (int64_t)u * blockDim.x;
            nd[u] = q < r1 ? (int)node_of_row[q] : -1;
        }
#pragma unroll
        for (int u = 0; u < ROUTE_U; ++u) {
            const int i = nd[u] - lo;
            if (nd[u] < lo) t[u] = make_int4(-1, 0, 0, 0);
            else if (i < ntab) t[u] = s_tab[i];
            else t[u] = make_int4(split_feat[nd[u]], split_bin[nd[u]], left_child[nd[u]], right_child[nd[u]]);
        }
#pragma unroll
        for (int u = 0; u < ROUTE_U; ++u) {
            const int64_t q = q0 + (int64_t)u * blockDim.x;
            b[u] = t[u].x >= 0 ? bins[q * rs + (int64_t)(t[u].x & ~(HM_TREE_CAT | HM_TREE_DLEFT)) * cs] : 0;
        }
#pragma unroll
        for (int u = 0; u < ROUTE_U; ++u) {
            if (t[u].x < 0) continue;
            const bool cat = t[u].x & HM_TREE_CAT;
            const bool dl = t[u].x & HM_TREE_DLEFT;
            const bool go_left = b[u] == miss_bin ? dl : (cat ? b[u] == t[u].y : b[u] <= t[u].y);
            node_of_row[q0 + (int64_t)u * blockDim.x] = (NT)(go_left ? t[u].z : t[u].w);
        }
    }
}


// ---------------------------------------------------------------------------------------------
// Fused split search of one tree level (replaces ~30 tensor ops over [L, d, B, NS] per level).
// One 256-thread block per node; each wave takes features f = wave, wave + 4, ...; a lane owns
// ceil(B / 64) consecutive bins, the bin prefix sums are a wave scan, the best bin is a wave
// argmax and the best feature a block argmax.  Criteria (split gain = score(L) + score(R) -
// score(parent), children need weight >= min_leaf):
//   0 gini     S = class counts        score = sum S^2 / W              W = sum S
//   1 entropy  S = class counts        score = sum S log(S / W)         W = sum S
//   2 variance S = (sum w y, sum w)    score = S0^2 / S1                W = S1
//   3 gbt      S = (sum r, sum h, n)   score = S0^2 / (S2 + lambda)     W = S2
//   4 xgb      S = (sum g, sum h)      score = T(S0)^2 / (S1 + lambda)  W = S1 (T: L1 soft threshold)
// Nominal columns (cat[f]) score "bin == b" against the rest, never the last bin (NaN / beyond
// the category list).  mtry < d draws the node's candidate features by ranking a counter hash
// of (seed, node, feature) — the same draw on the host engine (trees_cpu.cpp).
struct SplitParams {
    int L, d, B, NS, n_edges;
    int crit, mtry, node_base;
    float lam, alpha, min_leaf;
    uint32_t seed;
    int miss;     // 1: bin B-1 holds the missing values; each ordinal candidate is scored with
                  // them on the right and on the left, the better one is the default direction
};

__host__ __device__ __forceinline__ uint32_t feat_key(uint32_t seed, uint32_t node, uint32_t f) {
    uint32_t h = seed * 0x9E3779B1u ^ (node + 0x7F4A7C15u) * 0x85EBCA77u ^ (f + 1u) * 0xC2B2AE3Du;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    return h;
}

__device__ __forceinline__ float soft_thr(float g, float a) {
    if (a <= 0.f) return g;
    const float m = fabsf(g) - a;
    return m > 0.f ? copysignf(m, g) : 0.f;
}

template <int NS>
__device__ __forceinline__ float split_weight(const float* S, int crit) {
    if (crit <= 1) { float w = 0.f;
#pragma unroll
        for (int s = 0; s < NS; ++s) w += S[s];
        return w; }
    if (crit == 3) return NS > 2 ? S[NS > 2 ? 2 : 0] : 0.f;
    if (crit == 5) return NS > 1 ? S[NS > 1 ? 1 : 0] : 0.f;
    return NS > 1 ? S[NS > 1 ? 1 : 0] : 0.f;
}

template <int NS>
__device__ __forceinline__ float split_score(const float* S, int crit, float lam, float alpha) {
    if (crit == 0) {
        float w = 0.f, q = 0.f;
#pragma unroll
        for (int s = 0; s < NS; ++s) { w += S[s]; q += S[s] * S[s]; }
        return w > 0.f ? q / fmaxf(w, 1e-30f) : 0.f;
    }
    if (crit == 1) {
        float w = 0.f;
#pragma unroll
        for (int s = 0; s < NS; ++s) w += S[s];
        const float iw = 1.f / fmaxf(w, 1e-30f);
        float e = 0.f;
#pragma unroll
        for (int s = 0; s < NS; ++s) e += S[s] * logf(fmaxf(S[s] * iw, 1e-30f));
        return e;
    }
    const float s0 = S[0];
    if (crit == 2) { const float s1 = S[NS > 1 ? 1 : 0]; return s1 > 0.f ? s0 * s0 / fmaxf(s1, 1e-30f) : 0.f; }
    if (crit == 3) { const float s2 = S[NS > 2 ? 2 : 0]; return s2 > 0.f ? s0 * s0 / (s2 + lam) : 0.f; }
    if (crit == 5) { const float s1 = S[NS > 1 ? 1 : 0]; return s1 > 0.f ? s0 * s0 / (s1 + lam) : 0.f; }
    const float s1 = S[NS > 1 ? 1 : 0];
    const float g = soft_thr(s0, alpha);
    return s1 > 0.f ? g * g / (s1 + lam) : 0.f;
}

// 16 waves per node: every wave scans <= 2 features (d <= 32) instead of 7 in series — the
// kernel is a chain of dependent histogram reads per feature, and the upper levels have only
// 1 .. 64 nodes (blocks) for 256 CUs
// (512 for > 4 statistics: their per-lane state fits 128 VGPRs only at 1024 without spilling)
template <int NS> constexpr int sf_threads() { return NS <= 4 ? 1024 : 512; }
template <int NS>
__global__ __launch_bounds__(sf_threads<NS>()) void split_find_kernel(SplitParams P, const float* __restrict__ hist,
                                                         const uint8_t* __restrict__ cat,
                                                         const uint8_t* __restrict__ fmask,
                                                         float* __restrict__ out_gain,
                                                         int32_t* __restrict__ out_feat,
                                                         int32_t* __restrict__ out_bin,
                                                         float* __restrict__ out_left,
                                                         float* __restrict__ out_tot) {
    constexpr int NW = sf_threads<NS>() / 64;
    __shared__ float s_gain[NW];
    __shared__ int s_idx[NW];
    __shared__ float s_left[NW][NS];
    const int node = blockIdx.x;
    const int lane = hm::lane_id(), wave = hm::wave_id();
    const int B = P.B, d = P.d;
    const int bpl = (B + 63) / 64;              // bins per lane (<= 4)
    const int b0 = lane * bpl;
    const float* hn = hist + (size_t)node * d * B * NS;
    // parent totals (feature 0's histogram), identical in every wave
    float tot[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) tot[s] = 0.f;
    for (int k = 0; k < bpl; ++k)
        if (b0 + k < B)
#pragma unroll
            for (int s = 0; s < NS; ++s) tot[s] += hn[(size_t)(b0 + k) * NS + s];
#pragma unroll
    for (int s = 0; s < NS; ++s) tot[s] = hm::wave_sum(tot[s]);
    const float parent = split_score<NS>(tot, P.crit, P.lam, P.alpha);

    float best = -INFINITY;
    int best_i = 0x7FFFFFFF;
    float best_left[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) best_left[s] = 0.f;
    for (int f = wave; f < d; f += NW) {   // <= 2 features per wave at d <= 32
        if (fmask && !fmask[f]) continue;
        if (P.mtry > 0 && P.mtry < d) {
            // candidate iff fewer than mtry features rank before f (wave-uniform loop)
            const uint32_t kf = feat_key(P.seed, (uint32_t)(P.node_base + node), (uint32_t)f);
            int before = 0;
            for (int g = lane; g < d; g += 64) {
                const uint32_t kg = feat_key(P.seed, (uint32_t)(P.node_base + node), (uint32_t)g);
                before += (kg < kf || (kg == kf && g < f)) ? 1 : 0;
            }
            for (int o = 32; o > 0; o >>= 1) before += __shfl_xor(before, o, 64);
            if (before >= P.mtry) continue;
        }
        const bool is_cat = cat && cat[f];
        const float* hf = hn + (size_t)f * B * NS;
        const bool fmiss = P.miss && !is_cat;
        float M[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) M[s] = fmiss ? hf[(size_t)(B - 1) * NS + s] : 0.f;
        float h[4][NS];
        float lsum[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) lsum[s] = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool in = k < bpl && b0 + k < B;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                h[k][s] = in ? hf[(size_t)(b0 + k) * NS + s] : 0.f;
                lsum[s] += h[k][s];
            }
        }
        // exclusive wave scan of the lane sums -> running left statistics
        float run[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            float v = lsum[s];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const float t = __shfl_up(v, o, 64);
                if (lane >= o) v += t;
            }
            run[s] = v - lsum[s];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k >= bpl || b0 + k >= B) break;
            const int b = b0 + k;
            float left[NS], right[NS];
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                run[s] += h[k][s];
                left[s] = is_cat ? h[k][s] : run[s];
                right[s] = tot[s] - left[s];
            }
            if (fmiss && b == B - 1) break;         // the missing bin is not a threshold
            for (int v = 0; v < (fmiss ? 2 : 1); ++v) {
                if (v == 1) {                        // the missing rows on the left
#pragma unroll
                    for (int s = 0; s < NS; ++s) {
                        left[s] += M[s];
                        right[s] -= M[s];
                    }
                }
                bool ok = split_weight<NS>(left, P.crit) >= P.min_leaf &&
                          split_weight<NS>(right, P.crit) >= P.min_leaf;
                if (is_cat && b >= P.n_edges) ok = false;
                if (!ok) continue;
                const float g = split_score<NS>(left, P.crit, P.lam, P.alpha) +
                                split_score<NS>(right, P.crit, P.lam, P.alpha) - parent;
                const int i = (f * B + b) * 2 + v;   // ties: smaller (feature, bin), missing right
                if (g > best || (g == best && i < best_i)) {
                    best = g;
                    best_i = i;
#pragma unroll
                    for (int s = 0; s < NS; ++s) best_left[s] = left[s];
                }
            }
        }
    }
    // wave argmax (ties -> smaller flattened (feature, bin) index)
    for (int o = 32; o > 0; o >>= 1) {
        const float og = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(best_i, o, 64);
        float ol[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) ol[s] = __shfl_xor(best_left[s], o, 64);
        if (og > best || (og == best && oi < best_i)) {
            best = og;
            best_i = oi;
#pragma unroll
            for (int s = 0; s < NS; ++s) best_left[s] = ol[s];
        }
    }
    if (lane == 0) {
        s_gain[wave] = best;
        s_idx[wave] = best_i;
#pragma unroll
        for (int s = 0; s < NS; ++s) s_left[wave][s] = best_left[s];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int w = 0;
        for (int k = 1; k < NW; ++k)
            if (s_gain[k] > s_gain[w] || (s_gain[k] == s_gain[w] && s_idx[k] < s_idx[w])) w = k;
        const bool found = s_idx[w] != 0x7FFFFFFF;
        const int fb = s_idx[w] >> 1;
        out_gain[node] = found ? s_gain[w] : -INFINITY;
        out_feat[node] = found ? fb / B : 0;
        // bit 16 of the bin: the missing values go left at this split
        out_bin[node] = found ? (fb % B) | ((s_idx[w] & 1) << 16) : 0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            out_left[node * NS + s] = s_left[w][s];
            out_tot[node * NS + s] = tot[s];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Split search for class-count statistics with more classes than the register kernel holds
// (NS > 8: RandomForest with up to 256 classes).  Gini and entropy scores decompose over the
// classes (gini = sum S^2 / W, entropy = sum S log S - W log W), so the kernel walks the classes
// one at a time and keeps, per candidate bin, only (W, sum f(S)) of the left and right child: 4
// bins x 4 floats per lane whatever NS is.  Same candidates, mtry draw, nominal rule and
// tie-break as split_find_kernel; the left statistics of the winning split are re-summed per
// class at the end (thread per class).
// gini: term S^2, score T / W.  entropy: term S log(S / W) with the child weight W known from a
// first pass over the classes (no T - W log W cancellation), score T.
__device__ __forceinline__ float wide_term(float S, float W, int crit) {
    return crit == 0 ? S * S : S * logf(fmaxf(S / fmaxf(W, 1e-30f), 1e-30f));
}
__device__ __forceinline__ float wide_score(float W, float T, int crit) {
    if (W <= 0.f) return 0.f;
    return crit == 0 ? T / fmaxf(W, 1e-30f) : T;
}

__global__ __launch_bounds__(256) void split_find_wide_kernel(SplitParams P, const float* __restrict__ hist,
                                                              const uint8_t* __restrict__ cat,
                                                              const uint8_t* __restrict__ fmask,
                                                              float* __restrict__ out_gain,
                                                              int32_t* __restrict__ out_feat,
                                                              int32_t* __restrict__ out_bin,
                                                              float* __restrict__ out_left,
                                                              float* __restrict__ out_tot) {
    __shared__ float s_gain[4];
    __shared__ int s_idx[4];
    const int node = blockIdx.x;
    const int lane = hm::lane_id(), wave = hm::wave_id();
    const int B = P.B, d = P.d, NS = P.NS;
    const int bpl = (B + 63) / 64;
    const int b0 = lane * bpl;
    const float* hn = hist + (size_t)node * d * B * NS;
    // parent score from feature 0's histogram (class order 0..NS-1, as the host engine)
    auto node_class = [&](int c) {
        float v = 0.f;
        for (int k = 0; k < bpl; ++k)
            if (b0 + k < B) v += hn[(size_t)(b0 + k) * NS + c];
        return hm::wave_sum(v);
    };
    float pw = 0.f, pt = 0.f;
    for (int c = 0; c < NS; ++c) pw += node_class(c);
    for (int c = 0; c < NS; ++c) pt += wide_term(node_class(c), pw, P.crit);
    const float parent = wide_score(pw, pt, P.crit);

    float best = -INFINITY;
    int best_i = 0x7FFFFFFF;
    for (int f = wave; f < d; f += 4) {
        if (fmask && !fmask[f]) continue;
        if (P.mtry > 0 && P.mtry < d) {
            const uint32_t kf = feat_key(P.seed, (uint32_t)(P.node_base + node), (uint32_t)f);
            int before = 0;
            for (int g = lane; g < d; g += 64) {
                const uint32_t kg = feat_key(P.seed, (uint32_t)(P.node_base + node), (uint32_t)g);
                before += (kg < kf || (kg == kf && g < f)) ? 1 : 0;
            }
            for (int o = 32; o > 0; o >>= 1) before += __shfl_xor(before, o, 64);
            if (before >= P.mtry) continue;
        }
        const bool is_cat = cat && cat[f];
        const float* hf = hn + (size_t)f * B * NS;
        float wl[4] = {0.f, 0.f, 0.f, 0.f}, tl[4] = {0.f, 0.f, 0.f, 0.f};
        float wr[4] = {0.f, 0.f, 0.f, 0.f}, tr[4] = {0.f, 0.f, 0.f, 0.f};
        // pass 0 (entropy only): child weights; pass 1: the score terms
        for (int pass = P.crit == 1 ? 0 : 1; pass < 2; ++pass) {
            for (int c = 0; c < NS; ++c) {
                float h[4];
                float lsum = 0.f;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    h[k] = (k < bpl && b0 + k < B) ? hf[(size_t)(b0 + k) * NS + c] : 0.f;
                    lsum += h[k];
                }
                float v = lsum;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const float t = __shfl_up(v, o, 64);
                    if (lane >= o) v += t;
                }
                const float tc = hm::wave_sum(lsum);
                float run = v - lsum;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    run += h[k];
                    const float l = is_cat ? h[k] : run;
                    const float r = tc - l;
                    if (pass == 0 || P.crit == 0) { wl[k] += l; wr[k] += r; }
                    if (pass == 1) { tl[k] += wide_term(l, wl[k], P.crit); tr[k] += wide_term(r, wr[k], P.crit); }
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int b = b0 + k;
            if (k >= bpl || b >= B) break;
            if (wl[k] < P.min_leaf || wr[k] < P.min_leaf) continue;
            if (is_cat && b >= P.n_edges) continue;
            const float g = wide_score(wl[k], tl[k], P.crit) + wide_score(wr[k], tr[k], P.crit) - parent;
            const int i = f * B + b;
            if (g > best || (g == best && i < best_i)) { best = g; best_i = i; }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float og = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(best_i, o, 64);
        if (og > best || (og == best && oi < best_i)) { best = og; best_i = oi; }
    }
    if (lane == 0) { s_gain[wave] = best; s_idx[wave] = best_i; }
    __syncthreads();
    int w = 0;
    for (int k = 1; k < 4; ++k)
        if (s_gain[k] > s_gain[w] || (s_gain[k] == s_gain[w] && s_idx[k] < s_idx[w])) w = k;
    const bool found = s_idx[w] != 0x7FFFFFFF;
    if (threadIdx.x == 0) {
        out_gain[node] = found ? s_gain[w] : -INFINITY;
        out_feat[node] = found ? s_idx[w] / B : 0;
        out_bin[node] = found ? s_idx[w] % B : 0;
    }
    // per class: node total (feature 0) and the winning split's left statistics
    const int bf = found ? s_idx[w] / B : 0, bb = found ? s_idx[w] % B : -1;
    const bool bcat = found && cat && cat[bf];
    for (int c = threadIdx.x; c < NS; c += blockDim.x) {
        float t = 0.f, l = 0.f;
        for (int b = 0; b < B; ++b) {
            t += hn[(size_t)b * NS + c];
            const float hv = hn[((size_t)bf * B + b) * NS + c];
            if (bcat ? b == bb : b <= bb) l += hv;
        }
        out_tot[(size_t)node * NS + c] = t;
        out_left[(size_t)node * NS + c] = found ? l : 0.f;
    }
}

// ---------------------------------------------------------------------------------------------
// Level row partition (replaces a full 16-bit key sort of the active rows per level): the rows
// of the smaller child of every split, grouped by child, as the next level's histogram input.
// key(r) = lut[node_of_row[r] - nb] (32767 / out of range: not histogrammed).  Two passes over
// fixed row chunks (one per block): count per (key, block) in LDS, a device-wide inclusive scan
// of the key-major counts (torch.cumsum), then scatter with LDS rank counters.  Order inside a
// (key, block) cell is arbitrary; the histogram sums do not depend on it (32-bit fixed point).
template <typename NT>
__device__ __forceinline__ int part_key(const NT* __restrict__ node_of_row,
                                        const int16_t* __restrict__ lut, int row, int nb, int nlut,
                                        int nkeys) {
    const int c = node_of_row[row] - nb;
    if (c < 0 || c >= nlut) return -1;
    const int k = lut[c];
    return k < nkeys ? k : -1;
}

template <typename NT>
__global__ __launch_bounds__(256) void part_count_kernel(const int32_t* __restrict__ rows, int64_t m,
                                                         const NT* __restrict__ node_of_row,
                                                         const int16_t* __restrict__ lut, int nb,
                                                         int nlut, int nkeys,
                                                         int64_t* __restrict__ counts /* [nkeys][G] */) {
    extern __shared__ int s_cnt[];
    const int G = gridDim.x;
    for (int k = threadIdx.x; k < nkeys; k += blockDim.x) s_cnt[k] = 0;
    __syncthreads();
    const int64_t chunk = (m + G - 1) / G;
    const int64_t r0 = (int64_t)blockIdx.x * chunk, r1 = min(m, r0 + chunk);
    for (int64_t q = r0 + threadIdx.x; q < r1; q += blockDim.x) {
        const int k = part_key(node_of_row, lut, rows[q], nb, nlut, nkeys);
        if (k >= 0) atomicAdd(&s_cnt[k], 1);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nkeys; k += blockDim.x) counts[(size_t)k * G + blockIdx.x] = s_cnt[k];
}

constexpr int PART_U = 4;
constexpr int PART_LUT = 2048;
template <typename NT>
__global__ __launch_bounds__(256) void part_scatter_kernel(const int32_t* __restrict__ rows, int64_t m,
                                                           const NT* __restrict__ node_of_row,
                                                           const int16_t* __restrict__ lut, int nb,
                                                           int nlut, int nkeys,
                                                           const int64_t* __restrict__ counts,
                                                           const int64_t* __restrict__ incl,
                                                           int32_t* __restrict__ out,
                                                           int64_t* __restrict__ seg /* [nkeys+1] */) {
    extern __shared__ int64_t s_pos[];
    __shared__ int16_t s_lut[PART_LUT];
    const int G = gridDim.x;
    const int nl = min(nlut, PART_LUT);
    for (int k = threadIdx.x; k < nkeys; k += blockDim.x) {
        const size_t c = (size_t)k * G + blockIdx.x;
        s_pos[k] = incl[c] - counts[c];               // first slot of this (key, block) cell
    }
    for (int i = threadIdx.x; i < nl; i += blockDim.x) s_lut[i] = lut[i];
    if (blockIdx.x == 0) {
        for (int k = threadIdx.x; k <= nkeys; k += blockDim.x)
            seg[k] = k == 0 ? 0 : incl[(size_t)k * G - 1];
    }
    __syncthreads();
    const int64_t chunk = (m + G - 1) / G;
    const int64_t r0 = (int64_t)blockIdx.x * chunk, r1 = min(m, r0 + chunk);
    // PART_U rows per thread in flight (the row -> node -> key chain is latency-bound); the lut
    // in LDS.  The rank within a (key, block) cell is whatever the LDS atomics hand out.
    for (int64_t q0 = r0 + threadIdx.x; q0 < r1; q0 += (int64_t)blockDim.x * PART_U) {
        int row[PART_U], nd[PART_U];
#pragma unroll
        for (int u = 0; u < PART_U; ++u) {
            const int64_t q = q0 + (int64_t)u * blockDim.x;
            row[u] = q < r1 ? (rows ? rows[q] : (int)q) : -1;     // rows == NULL: every row, in order
        }
#pragma unroll
        for (int u = 0; u < PART_U; ++u) nd[u] = row[u] >= 0 ? (int)node_of_row[row[u]] : -1;
#pragma unroll
        for (int u = 0; u < PART_U; ++u) {
            const int c = nd[u] - nb;
            if (row[u] < 0 || nd[u] < 0 || c < 0 || c >= nlut) continue;
            const int k = c < PART_LUT ? s_lut[c] : lut[c];
            if (k >= nkeys) continue;
            const int64_t pos = atomicAdd(reinterpret_cast<unsigned long long*>(&s_pos[k]), 1ull);
            out[pos] = row[u];
        }
    }
}

// A level's routing and the small-children counting of part_count_kernel in one pass, when
// every row is active (rows 0 .. n-1 in order): each row's bins byte, node and lut entry are read
// once, instead of once by route_kernel over all rows and again (with the row index) by
// part_count_kernel.  Same (key, block) cells as part_count_kernel (same grid and chunking), so
// part_scatter_kernel (rows = NULL) places the rows identically.
// The pass is latency-bound, not bandwidth-bound (the root level, 55 MB, took as long as the
// deepest): per row node -> split -> bins -> child is a dependent chain.  So the split tables
// of the level's nodes [lo, lo + ROUTE_TAB) and the lut sit in LDS (two of the four dependent
// loads become LDS reads) and ROUTE_U rows per thread are in flight.  Node ids below lo are
// leaves of earlier levels (their rows stay); ids in [lo + ROUTE_TAB, nb) read global memory.
constexpr int ROUTE_BALLOT_KEYS = 16;
constexpr int ROUTE_LUT = 2048;
template <typename NT>
__global__ __launch_bounds__(256) void route_count_kernel(const uint8_t* __restrict__ bins, int64_t n,
                                                          int64_t rs, int64_t cs,
                                                          NT* __restrict__ node_of_row,
                                                          const int32_t* __restrict__ split_feat,
                                                          const int32_t* __restrict__ split_bin,
                                                          const int32_t* __restrict__ left_child,
                                                          const int32_t* __restrict__ right_child, int miss_bin,
                                                          const int16_t* __restrict__ lut, int nb, int nlut,
                                                          int nkeys, int64_t* __restrict__ counts, int lo) {
    extern __shared__ int s_cnt[];
    __shared__ int4 s_tab[ROUTE_TAB];          // {split_feat, split_bin, left, right} of node lo + i
    __shared__ int16_t s_lut[ROUTE_LUT];
    const int G = gridDim.x;
    const int ntab = max(0, min(ROUTE_TAB, nb - lo));
    const int nl = min(nlut, ROUTE_LUT);
    for (int k = threadIdx.x; k < nkeys; k += blockDim.x) s_cnt[k] = 0;
    for (int i = threadIdx.x; i < ntab; i += blockDim.x)
        s_tab[i] = make_int4(split_feat[lo + i], split_bin[lo + i], left_child[lo + i], right_child[lo + i]);
    for (int i = threadIdx.x; i < nl; i += blockDim.x) s_lut[i] = lut[i];
    __syncthreads();
    const int64_t chunk = (n + G - 1) / G;
    const int64_t r0 = (int64_t)blockIdx.x * chunk, r1 = min(n, r0 + chunk);
    uint32_t wcnt[ROUTE_BALLOT_KEYS];
#pragma unroll
    for (int q = 0; q < ROUTE_BALLOT_KEYS; ++q) wcnt[q] = 0;
    // every wave runs the same trip count (ballots need the whole wave): the bound is the block's
    for (int64_t q0 = r0 + threadIdx.x; q0 - threadIdx.x < r1; q0 += (int64_t)blockDim.x * ROUTE_U) {
        int nd[ROUTE_U];
        int4 t[ROUTE_U];
        int b[ROUTE_U];
#pragma unroll
        for (int u = 0; u < ROUTE_U; ++u) {
            const int64_t q = q0 + (int64_t)u * blockDim.x;
            nd[u] = q < r1 ? node_of_row[q] : -1;
        }
#pragma unroll
        for (int u = 0; u < ROUTE_U; ++u) {
            const int i = nd[u] - lo;
            if (nd[u] < lo) t[u] = make_int4(-1, 0, 0, 0);              // -1 or an earlier leaf
            else if (i < ntab) t[u] = s_tab[i];
            else t[u] = make_int4(split_feat[nd[u]], split_bin[nd[u]], left_child[nd[u]], right_child[nd[u]]);
        }
#pragma unroll
        for (int u = 0; u < ROUTE_U; ++u) {
            const int64_t q = q0 + (int64_t)u * blockDim.x;
            b[u] = t[u].x >= 0 ? bins[q * rs + (int64_t)(t[u].x & ~(HM_TREE_CAT | HM_TREE_DLEFT)) * cs] : 0;
        }
#pragma unroll
        for (int u = 0; u < ROUTE_U; ++u) {
            if (t[u].x < 0) continue;
            const int64_t q = q0 + (int64_t)u * blockDim.x;
            const bool cat = t[u].x & HM_TREE_CAT;
            const bool dl = t[u].x & HM_TREE_DLEFT;
            const bool go_left = b[u] == miss_bin ? dl : (cat ? b[u] == t[u].y : b[u] <= t[u].y);
            nd[u] = go_left ? t[u].z : t[u].w;
            node_of_row[q] = (NT)nd[u];
        }
#pragma unroll
        for (int u = 0; u < ROUTE_U; ++u) {
            const int c = nd[u] - nb;
            int k = -1;
            if (nd[u] >= 0 && c >= 0 && c < nlut) {
                k = c < ROUTE_LUT ? s_lut[c] : lut[c];
                if (k >= nkeys) k = -1;
            }
            if (nkeys <= ROUTE_BALLOT_KEYS) {
                // few keys (the upper levels): every row of a wave hits one of <= 16 LDS words,
                // so count them with ballots into wave-uniform registers instead
#pragma unroll
                for (int q = 0; q < ROUTE_BALLOT_KEYS; ++q)
                    if (q < nkeys) wcnt[q] += __popcll(__ballot(k == q));
            } else if (k >= 0) {
                atomicAdd(&s_cnt[k], 1);
            }
        }
    }
    if (nkeys <= ROUTE_BALLOT_KEYS && (threadIdx.x & 63) == 0) {
#pragma unroll
        for (int q = 0; q < ROUTE_BALLOT_KEYS; ++q)
            if (q < nkeys && wcnt[q]) atomicAdd(&s_cnt[q], (int)wcnt[q]);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nkeys; k += blockDim.x) counts[(size_t)k * G + blockIdx.x] = s_cnt[k];
}

// Next-level histograms from the parents' and the smaller children's: for split i (parent
// node li[i]), child 2i+sr[i] gets Hs[i] and child 2i+1-sr[i] gets H[li[i]] - Hs[i].
__global__ __launch_bounds__(256) void hist_sibling_kernel(const float* __restrict__ H,
                                                           const float* __restrict__ Hs,
                                                           const int64_t* __restrict__ li,
                                                           const uint8_t* __restrict__ small_right,
                                                           int64_t per, int n_split,
                                                           float* __restrict__ Hn) {
    const int i = blockIdx.y;
    if (i >= n_split) return;
    const float4* hp = reinterpret_cast<const float4*>(H + (size_t)li[i] * per);
    const float4* hs = reinterpret_cast<const float4*>(Hs + (size_t)i * per);
    const int sr = small_right[i] ? 1 : 0;
    float4* dsmall = reinterpret_cast<float4*>(Hn + (size_t)(2 * i + sr) * per);
    float4* dbig = reinterpret_cast<float4*>(Hn + (size_t)(2 * i + 1 - sr) * per);
    const int64_t n4 = per / 4;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n4; e += (int64_t)gridDim.x * blockDim.x) {
        const float4 a = hp[e], b = hs[e];
        dsmall[e] = b;
        dbig[e] = make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
    }
}
// Heap-layout next level: parent l's children are 2l, 2l+1 of Hn; split parents get Hs[l] (the
// smaller child's histogram) and H[l] - Hs[l], the children slots of parents that did not split
// get zeros (their nodes exist in the fixed-shape level but hold no rows: no split is found).
__global__ __launch_bounds__(256) void hist_sibling_heap_kernel(const float* __restrict__ H,
                                                                const float* __restrict__ Hs,
                                                                const int32_t* __restrict__ split_feat,
                                                                const uint8_t* __restrict__ small_right,
                                                                int64_t per, int L, float* __restrict__ Hn) {
    const int l = blockIdx.y;
    if (l >= L) return;
    const bool split = split_feat[l] >= 0;
    const float4* hp = reinterpret_cast<const float4*>(H + (size_t)l * per);
    const float4* hs = reinterpret_cast<const float4*>(Hs + (size_t)l * per);
    const int sr = small_right[l] ? 1 : 0;
    float4* dsmall = reinterpret_cast<float4*>(Hn + (size_t)(2 * l + sr) * per);
    float4* dbig = reinterpret_cast<float4*>(Hn + (size_t)(2 * l + 1 - sr) * per);
    const int64_t n4 = per / 4;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n4; e += (int64_t)gridDim.x * blockDim.x) {
        if (split) {
            const float4 a = hp[e], b = hs[e];
            dsmall[e] = b;
            dbig[e] = make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
        } else {
            dsmall[e] = z;
            dbig[e] = z;
        }
    }
}
}  // namespace

// hist [n_seg, d, B, NS] (zeroed by the caller) += statistics of rows[seg[k]..seg[k+1]) for
// every node k.  seg lives on the device.  FG (features per group) is 4, 8 or 16 and bins rows
// are padded to a multiple of 16 bytes, so a row's group is one aligned 4/8/16-byte load.
// smax: device [NS] upper bounds of |stats[:, s]| (fixed-point scaling of the LDS sums).
HM_API int hm_hist_build(const uint8_t* bins, int d, int dpad, int B, const int32_t* rows,
                         const int64_t* seg, int n_seg, const float* stats, const float* smax,
                         int NS, int FG, float* hist, int nblk, hipStream_t stream) {
    if (n_seg <= 0) return 0;
    if (nblk <= 0) nblk = 1024;
    if (B > 256 || NS <= 0 || NS > 8 || (FG != 4 && FG != 8 && FG != 16 && FG != 32) || (dpad & 15) ||
        (FG == 32 && (dpad & 31)))
        return (int)hipErrorInvalidValue;
    // FG = 32: every feature of a <= 32-feature row in one pass -- one 32-B bins load, one row
    // index and one stats load per row instead of one each per 16-feature group -- into one LDS
    // image of up to 160 KB shared by a 1024-thread block (16 waves hide the row gathers).
    const size_t lds = (size_t)(FG == 32 ? min(d, 32) : FG) * B * NS * sizeof(float);
    if (lds > (FG == 32 ? 160 * 1024 : 64 * 1024)) return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)nblk, (unsigned)((d + FG - 1) / FG));
#define HM_H(K, W)                                                                                  \
    case K * 100 + W:                                                                               \
        hipLaunchKernelGGL((hist_kernel<K, W>), grid, dim3(256), lds, stream, bins, d, dpad, B, rows, \
                           seg, n_seg, stats, smax, hist);                                          \
        break;
#define HM_HN(K) HM_H(K, 1) HM_H(K, 2) HM_H(K, 4)
    // statistics pairs as 64-bit LDS adds (default; HM_HIST_PACK=0: one 32-bit add per statistic).
    // GBDT 11 M x 28 depth 8: 4.14 -> 4.03 ms per tree with the all-features pass (r4h/gbdt_ab.log)
    static const bool pack = [] { const char* e = getenv("HM_HIST_PACK"); return !(e && e[0] == '0'); }();
    if (pack && (NS == 2 || NS == 3) && (FG == 16 || FG == 32)) {
#define HM_HP(K, W, T) { \
            static bool attr_set = false; \
            if (!attr_set) { \
                (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hist_kernel<K, W, T, true>), \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
                attr_set = true; \
            } \
            hipLaunchKernelGGL((hist_kernel<K, W, T, true>), grid, dim3(T), lds, stream, bins, d, dpad, B, rows, \
                               seg, n_seg, stats, smax, hist); }
        if (NS == 2 && FG == 16) HM_HP(2, 4, 256)
        else if (NS == 3 && FG == 16) HM_HP(3, 4, 256)
        else if (NS == 2) HM_HP(2, 8, 1024)
        else HM_HP(3, 8, 1024)
#undef HM_HP
        HM_LAUNCH_RET();
    }
    if (FG == 32) {
        switch (NS) {
#define HM_HW(K) case K: { \
            static bool attr_set = false; \
            if (!attr_set) { \
                (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hist_kernel<K, 8, 1024>), \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
                attr_set = true; \
            } \
            hipLaunchKernelGGL((hist_kernel<K, 8, 1024>), grid, dim3(1024), lds, stream, bins, d, dpad, B, rows, seg, \
                               n_seg, stats, smax, hist); \
            break; }
            HM_HW(1) HM_HW(2) HM_HW(3) HM_HW(4)
#undef HM_HW
            default: return (int)hipErrorInvalidValue;
        }
        HM_LAUNCH_RET();
    }
    switch (NS * 100 + FG / 4) {
        HM_HN(1) HM_HN(2) HM_HN(3) HM_HN(4) HM_HN(5) HM_HN(6) HM_HN(7) HM_HN(8)
        default: return (int)hipErrorInvalidValue;
    }
#undef HM_HN
#undef HM_H
    HM_LAUNCH_RET();
}

HM_API int hm_absmax_cols(const float* stats, int64_t n, int NS, float* out, hipStream_t stream) {
    if (n <= 0) return 0;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 1024) blocks = 1024;
#define HM_A(K) \
    case K: hipLaunchKernelGGL((absmax_kernel<K>), dim3((int)blocks), dim3(256), 0, stream, stats, n, out); break;
    switch (NS) {
        HM_A(1) HM_A(2) HM_A(3) HM_A(4) HM_A(5) HM_A(6) HM_A(7) HM_A(8)
        default: return (int)hipErrorInvalidValue;
    }
#undef HM_A
    HM_LAUNCH_RET();
}

HM_API int hm_tree_predict(const float* X, int64_t n, int d, const int32_t* feature,
                           const float* threshold, const int32_t* left, const int32_t* right,
                           const int32_t* voff, const float* values, const int32_t* roots,
                           int n_trees, int n_out, float* out, int sum_trees, const float* tree_w,
                           hipStream_t stream) {
    const int64_t total = n * (int64_t)n_trees;
    if (total <= 0) return 0;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(tree_predict_kernel, dim3((int)blocks), dim3(256), 0, stream, X, n, d, feature,
                       threshold, left, right, voff, values, roots, n_trees, n_out, out, sum_trees,
                       tree_w);
    HM_LAUNCH_RET();
}

HM_API int hm_quantize(const float* X, int64_t n, int d, int dpad, const float* edges, int n_edges,
                       uint8_t* bins, hipStream_t stream) {
    const int64_t total = n * (int64_t)d;
    if (total <= 0) return 0;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(quantize_kernel, dim3((int)blocks), dim3(256), 0, stream, X, n, d, dpad, edges,
                       n_edges, bins);
    HM_LAUNCH_RET();
}

// miss_bin: the bin of missing values (rows there follow the split's HM_TREE_DLEFT flag), or -1.
// node16: node_of_row is int16 (trees of < 32,767 nodes: half the bytes per routing pass).
// col_stride > 0: bins is the feature-major copy [d, col_stride] (dpad unused).
// [lo, hi): the level's node ids (lower ids are leaves of earlier levels or -1).
HM_API int hm_route_rows(const uint8_t* bins, int64_t n, int dpad, int64_t col_stride, int lo, int hi,
                         void* node_of_row,
                         const int32_t* split_feat, const int32_t* split_bin,
                         const int32_t* left_child, const int32_t* right_child, int miss_bin, int node16,
                         hipStream_t stream) {
    if (n <= 0) return 0;
    if (col_stride > 0 && col_stride < n) return (int)hipErrorInvalidValue;
    if (lo < 0 || hi < lo) return (int)hipErrorInvalidValue;
    int64_t blocks = (n + 4095) / 4096;
    if (blocks > 1024) blocks = 1024;
    const int64_t rs = col_stride > 0 ? 1 : dpad, cs = col_stride > 0 ? col_stride : 1;
    if (node16)
        hipLaunchKernelGGL(route_kernel<int16_t>, dim3((int)blocks), dim3(256), 0, stream, bins, n, rs, cs,
                           (int16_t*)node_of_row, split_feat, split_bin, left_child, right_child, miss_bin, lo, hi);
    else
        hipLaunchKernelGGL(route_kernel<int32_t>, dim3((int)blocks), dim3(256), 0, stream, bins, n, rs, cs,
                           (int32_t*)node_of_row, split_feat, split_bin, left_child, right_child, miss_bin, lo, hi);
    HM_LAUNCH_RET();
}

// Best split of every node of a level: hist [L, d, B, NS] -> gain [L] (-inf: none), feature,
// bin, left-child statistics [L, NS] and node totals [L, NS].  cat / fmask: [d] bytes or null.
// ip: L, d, B, NS, n_edges, crit, mtry, node_base, seed, miss;  fp: lambda, alpha, min_leaf.
// With miss (NS <= 8 kernel) bin B-1 holds the missing values and bit 16 of the returned bin
// says they go left at that split.
HM_API int hm_split_find(const float* hist, const int32_t* ip, const float* fp, const uint8_t* cat,
                         const uint8_t* fmask, float* gain, int32_t* feat, int32_t* bin, float* left,
                         float* tot, hipStream_t stream) {
    SplitParams P;
    P.L = ip[0]; P.d = ip[1]; P.B = ip[2]; P.NS = ip[3]; P.n_edges = ip[4]; P.crit = ip[5];
    P.mtry = ip[6]; P.node_base = ip[7]; P.seed = (uint32_t)ip[8]; P.miss = ip[9];
    P.lam = fp[0]; P.alpha = fp[1]; P.min_leaf = fp[2];
    if (P.L <= 0) return 0;
    if (P.B <= 0 || P.B > 256 || P.d <= 0 || P.crit < 0 || P.crit > 5) return (int)hipErrorInvalidValue;
    if (P.NS > 8) {   // many classes: gini / entropy only, classes walked one at a time
        if (P.crit > 1 || P.NS > 4096 || P.miss) return (int)hipErrorInvalidValue;
        hipLaunchKernelGGL(split_find_wide_kernel, dim3(P.L), dim3(256), 0, stream, P, hist, cat, fmask,
                           gain, feat, bin, left, tot);
        HM_LAUNCH_RET();
    }
#define HM_SF(K) \
    case K: hipLaunchKernelGGL((split_find_kernel<K>), dim3(P.L), dim3(sf_threads<K>()), 0, stream, P, hist, cat, fmask, \
                               gain, feat, bin, left, tot); break;
    switch (P.NS) {
        HM_SF(1) HM_SF(2) HM_SF(3) HM_SF(4) HM_SF(5) HM_SF(6) HM_SF(7) HM_SF(8)
        default: return (int)hipErrorInvalidValue;
    }
#undef HM_SF
    HM_LAUNCH_RET();
}

// Row partition of a level, pass 1: counts [nkeys][G] (int64, G = grid) of the active rows per
// small-child key.  Pass 2 (after incl = inclusive cumsum of the flattened counts, int64):
// rows grouped by key into out[0 .. seg[nkeys]), segment starts seg [nkeys + 1].
HM_API int hm_partition_count(const int32_t* rows, int64_t m, const void* node_of_row,
                              const int16_t* lut, int nb, int nlut, int nkeys, int grid,
                              int64_t* counts, int node16, hipStream_t stream) {
    if (nkeys <= 0 || nkeys > 8192 || grid <= 0) return (int)hipErrorInvalidValue;
    if (node16)
        hipLaunchKernelGGL(part_count_kernel<int16_t>, dim3(grid), dim3(256), (size_t)nkeys * sizeof(int), stream,
                           rows, m, (const int16_t*)node_of_row, lut, nb, nlut, nkeys, counts);
    else
        hipLaunchKernelGGL(part_count_kernel<int32_t>, dim3(grid), dim3(256), (size_t)nkeys * sizeof(int), stream,
                           rows, m, (const int32_t*)node_of_row, lut, nb, nlut, nkeys, counts);
    HM_LAUNCH_RET();
}

// route_count_kernel: route rows 0 .. n-1 one level down and count the small children's rows
// per (key, block) cell; follow with hm_partition_scatter(rows = NULL, m = n, same grid).
// col_stride > 0: bins is the feature-major copy [d, col_stride] (see route_kernel).
HM_API int hm_route_count(const uint8_t* bins, int64_t n, int dpad, int64_t col_stride, int lo,
                          void* node_of_row, const int32_t* split_feat,
                          const int32_t* split_bin, const int32_t* left_child, const int32_t* right_child,
                          int miss_bin, const int16_t* lut, int nb, int nlut, int nkeys, int grid,
                          int64_t* counts, int node16, hipStream_t stream) {
    if (nkeys <= 0 || nkeys > 8192 || grid <= 0 || n <= 0 || n > INT32_MAX) return (int)hipErrorInvalidValue;
    if (col_stride > 0 && col_stride < n) return (int)hipErrorInvalidValue;
    if (lo < 0 || lo > nb) return (int)hipErrorInvalidValue;
    const int64_t rs = col_stride > 0 ? 1 : dpad, cs = col_stride > 0 ? col_stride : 1;
    if (node16)
        hipLaunchKernelGGL(route_count_kernel<int16_t>, dim3(grid), dim3(256), (size_t)nkeys * sizeof(int), stream,
                           bins, n, rs, cs, (int16_t*)node_of_row, split_feat, split_bin, left_child, right_child,
                           miss_bin, lut, nb, nlut, nkeys, counts, lo);
    else
        hipLaunchKernelGGL(route_count_kernel<int32_t>, dim3(grid), dim3(256), (size_t)nkeys * sizeof(int), stream,
                           bins, n, rs, cs, (int32_t*)node_of_row, split_feat, split_bin, left_child, right_child,
                           miss_bin, lut, nb, nlut, nkeys, counts, lo);
    HM_LAUNCH_RET();
}

HM_API int hm_partition_scatter(const int32_t* rows, int64_t m, const void* node_of_row,
                                const int16_t* lut, int nb, int nlut, int nkeys, int grid,
                                const int64_t* counts, const int64_t* incl, int32_t* out,
                                int64_t* seg, int node16, hipStream_t stream) {
    if (nkeys <= 0 || nkeys > 8192 || grid <= 0) return (int)hipErrorInvalidValue;
    if (node16)
        hipLaunchKernelGGL(part_scatter_kernel<int16_t>, dim3(grid), dim3(256), (size_t)nkeys * sizeof(int64_t),
                           stream, rows, m, (const int16_t*)node_of_row, lut, nb, nlut, nkeys, counts, incl, out, seg);
    else
        hipLaunchKernelGGL(part_scatter_kernel<int32_t>, dim3(grid), dim3(256), (size_t)nkeys * sizeof(int64_t),
                           stream, rows, m, (const int32_t*)node_of_row, lut, nb, nlut, nkeys, counts, incl, out, seg);
    HM_LAUNCH_RET();
}

// Hn [2 * n_split, per] from H [L, per], Hs [n_split, per] (per = d * B * NS, a multiple of 4).
HM_API int hm_hist_sibling(const float* H, const float* Hs, const int64_t* li, const uint8_t* small_right,
                           int64_t per, int n_split, float* Hn, hipStream_t stream) {
    if (n_split <= 0) return 0;
    if (per % 4) return (int)hipErrorInvalidValue;
    int64_t bx = (per / 4 + 255) / 256;
    if (bx > 64) bx = 64;
    hipLaunchKernelGGL(hist_sibling_kernel, dim3((unsigned)bx, (unsigned)n_split), dim3(256), 0, stream,
                       H, Hs, li, small_right, per, n_split, Hn);
    HM_LAUNCH_RET();
}

// Heap-layout sibling histograms (hist_sibling_heap_kernel): H, Hs [L, per], Hn [2L, per].
HM_API int hm_hist_sibling_heap(const float* H, const float* Hs, const int32_t* split_feat, const uint8_t* small_right,
                                int64_t per, int L, float* Hn, hipStream_t stream) {
    if (L <= 0) return 0;
    if (per % 4) return (int)hipErrorInvalidValue;
    int64_t bx = (per / 4 + 255) / 256;
    if (bx > 64) bx = 64;
    hipLaunchKernelGGL(hist_sibling_heap_kernel, dim3((unsigned)bx, (unsigned)L), dim3(256), 0, stream, H, Hs,
                       split_feat, small_right, per, L, Hn);
    HM_LAUNCH_RET();
}

// Fused binary-logistic GBT statistics (see gbt_stats_kernel): F, y [n] fp32, mask [n] uint8
// or NULL; stats [n, 3] fp32 out; smax [3] zeroed by the caller.
HM_API int hm_gbt_stats(const float* F, const float* y, const uint8_t* mask, int64_t n, float* stats,
                        float* smax, hipStream_t stream) {
    if (n <= 0) return 0;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL((gbt_stats_kernel<0>), dim3((int)blocks), dim3(256), 0, stream, F, y, mask, n, stats, smax,
                       nullptr);
    HM_LAUNCH_RET();
}

// The XGBoost binary-logistic form: stats [n, 2] = {p - y, max(p (1 - p), 1e-16)} x mask.
HM_API int hm_xgb_stats(const float* F, const float* y, const uint8_t* mask, int64_t n, float* stats,
                        float* smax, hipStream_t stream) {
    if (n <= 0) return 0;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL((gbt_stats_kernel<1>), dim3((int)blocks), dim3(256), 0, stream, F, y, mask, n, stats, smax,
                       nullptr);
    HM_LAUNCH_RET();
}

// Binary-logistic GBT with 2 split statistics: stats [n, 2] = {r, 1} x mask, hh [n] = |r| (1 - |r|)
// x mask (r = y - sigmoid(F)); smax [2] zeroed by the caller.
HM_API int hm_gbt2_stats(const float* F, const float* y, const uint8_t* mask, int64_t n, float* stats,
                         float* smax, float* hh, hipStream_t stream) {
    if (n <= 0) return 0;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL((gbt_stats_kernel<2>), dim3((int)blocks), dim3(256), 0, stream, F, y, mask, n, stats, smax, hh);
    HM_LAUNCH_RET();
}

// sums [T, 2] (zeroed by the caller) += {sum r, sum h} of the rows of every node (leaf [n] ids < T).
HM_API int hm_leaf_sums(const void* leaf, const float* st2, const float* hh, int64_t n, int T, float* sums,
                        int node16, hipStream_t stream) {
    if (n <= 0) return 0;
    if (T <= 0 || T > 8192) return (int)hipErrorInvalidValue;
    // every block ends with 2T float atomic adds onto the same 2T addresses; the row loop is
    // latency-bound, so up to 1,024 blocks (95 -> 55 µs per 11 M rows vs 256 blocks)
    int64_t blocks = (n + 4095) / 4096;
    if (blocks > LEAF_BLOCKS) blocks = LEAF_BLOCKS;
    static bool attr_set = false;     // 64-bit sums of up to 8,192 nodes: 128 KB of LDS
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&leaf_sums_kernel<int16_t>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&leaf_sums_kernel<int32_t>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    if (node16)
        hipLaunchKernelGGL(leaf_sums_kernel<int16_t>, dim3((int)blocks), dim3(256), (size_t)T * 2 * sizeof(unsigned long long) * (2 * T <= 2048 ? 4 : 1), stream,
                           (const int16_t*)leaf, st2, hh, n, T, sums);
    else
        hipLaunchKernelGGL(leaf_sums_kernel<int32_t>, dim3((int)blocks), dim3(256), (size_t)T * 2 * sizeof(unsigned long long) * (2 * T <= 2048 ? 4 : 1), stream,
                           (const int32_t*)leaf, st2, hh, n, T, sums);
    HM_LAUNCH_RET();
}

// vals[k] = sums[k, 0] / sums[k, 1] for the leaves (sf[k] < 0) among nodes 0 .. T-1.
// out [n] = bootstrap multiplicities; cnt [K] = draws per chunk of `chunk` rows (sum = m),
// K = ceil(n / chunk), chunk <= 12288.
HM_API int hm_bootstrap_counts(const int64_t* cnt, int64_t n, int chunk, uint64_t seed, float* out,
                               hipStream_t stream) {
    if (n <= 0) return 0;
    if (chunk <= 0 || chunk > BOOT_CHUNK) return (int)hipErrorInvalidValue;
    const int64_t K = (n + chunk - 1) / chunk;
    if (K > INT32_MAX) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(bootstrap_counts_kernel, dim3((unsigned)K), dim3(1024), 0, stream, cnt, n, chunk, seed, out);
    HM_LAUNCH_RET();
}

HM_API int hm_leaf_newton(const float* sums, const int32_t* sf, int T, float* vals, hipStream_t stream) {
    if (T <= 0) return 0;
    hipLaunchKernelGGL(leaf_newton_kernel, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, stream, sums, sf, T, vals);
    HM_LAUNCH_RET();
}

// F[r * ldf + k] += scale * vals[leaf[r] * ldv] for leaf[r] >= 0.
HM_API int hm_gbt_apply(float* F, int ldf, int k, const float* vals, int ldv, const void* leaf, int64_t n,
                        float scale, int node16, hipStream_t stream) {
    if (n <= 0) return 0;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (node16)
        hipLaunchKernelGGL(gbt_apply_kernel<int16_t>, dim3((int)blocks), dim3(256), 0, stream, F, ldf, k, vals, ldv,
                           (const int16_t*)leaf, n, scale);
    else
        hipLaunchKernelGGL(gbt_apply_kernel<int32_t>, dim3((int)blocks), dim3(256), 0, stream, F, ldf, k, vals, ldv,
                           (const int32_t*)leaf, n, scale);
    HM_LAUNCH_RET();
}

// ---------------------------------------------------------------------------------------------
// Level finalisation (one launch per level instead of ~40 tensor ops; models/trees.py build):
// from the split search's per-node results decide which nodes split, number their children,
// and lay out everything the next level needs — leaf values, node records (flagged feature,
// threshold, children), the compacted list of splitting nodes, which child is the smaller
// (histogrammed) one, the partition LUT and the split count (the level's one host read).
// One 1024-thread block; thread t owns a contiguous chunk of the L nodes, so children are
// numbered in node order (an exclusive block scan of the per-thread counts), as the
// cumsum-based host path does.
struct LevelParams {
    int L, NS, d, E, crit, n_out, nb, has_cat;
    int heap;   // children at nb + 2l, nb + 2l + 1 for parent l (fixed-shape levels, no host read)
    int last;   // the children are leaves: write their records too, values from (left, tot - left)
    float lam, alpha, min_gain, min_split;
};

// Leaf output(s) of statistics S(s), s < NS (models/trees.py _leaf_values).
template <typename SF>
__device__ __forceinline__ void leaf_value(const LevelParams& P, SF S, float* v) {
    if (P.crit <= 1) {
        float w = 0.f;
        for (int s = 0; s < P.NS; ++s) w += S(s);
        for (int s = 0; s < P.NS; ++s) v[s] = w > 0.f ? S(s) / fmaxf(w, 1e-30f) : 1.f / (float)P.NS;
    } else if (P.crit == 2 || P.crit == 5) {   // gbt2: the mean residual until hm_gbt2_leaf_values
        v[0] = S(1) > 0.f ? S(0) / fmaxf(S(1), 1e-30f) : 0.f;
    } else if (P.crit == 4) {
        const float den = S(1) + P.lam;
        v[0] = den > 0.f ? -soft_thr(S(0), P.alpha) / fmaxf(den, 1e-30f) : 0.f;
    } else {
        v[0] = fabsf(S(1)) > 1e-12f ? S(0) / S(1) : 0.f;
    }
}

__device__ __forceinline__ float node_weight(const float* S, int NS, int crit) {
    if (crit <= 1) {                         // gini / entropy: sum of class counts
        float w = 0.f;
        for (int s = 0; s < NS; ++s) w += S[s];
        return w;
    }
    if (crit == 2 || crit == 4 || crit == 5) return S[1];  // variance / xgb / gbt2: count
    return S[2];                              // gbt: count
}

__global__ __launch_bounds__(1024) void level_finalize_kernel(
    LevelParams P, const float* __restrict__ gain, const int32_t* __restrict__ feat,
    const int32_t* __restrict__ bins_raw, const float* __restrict__ left, const float* __restrict__ tot,
    const float* __restrict__ edges, const uint8_t* __restrict__ cat, float* __restrict__ vals,
    int32_t* __restrict__ feats_out, float* __restrict__ thrs_out, int32_t* __restrict__ lc_out,
    int32_t* __restrict__ rc_out, int32_t* __restrict__ sb_out, int64_t* __restrict__ li_out,
    uint8_t* __restrict__ small_right, int16_t* __restrict__ lut, int32_t* __restrict__ n_split,
    double* __restrict__ imp) {
    __shared__ int s_cnt[1024];
    const int t = threadIdx.x;
    const int chunk = (P.L + 1023) / 1024;
    const int l0 = min(P.L, t * chunk), l1 = min(P.L, l0 + chunk);
    const float gmin = fmaxf(1e-12f, P.min_gain);
    auto is_ok = [&](int l) {
        const float g = gain[l];
        return g > gmin && isfinite(g) && node_weight(tot + (size_t)l * P.NS, P.NS, P.crit) >= P.min_split;
    };
    int cnt = 0;
    for (int l = l0; l < l1; ++l) cnt += is_ok(l) ? 1 : 0;
    s_cnt[t] = cnt;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {      // inclusive Hillis-Steele scan
        const int v = t >= o ? s_cnt[t - o] : 0;
        __syncthreads();
        s_cnt[t] += v;
        __syncthreads();
    }
    int rank = s_cnt[t] - cnt;                 // exclusive prefix
    if (t == 1023) n_split[0] = s_cnt[1023];
    for (int l = l0; l < l1; ++l) {
        const float* S = tot + (size_t)l * P.NS;
        // leaf value(s) of the node
        leaf_value(P, [&](int s) { return S[s]; }, vals + (size_t)l * P.n_out);
        // last level: the children's records (relative to this level's first node, nb - L)
        auto leaf_child = [&](int c, const float* Lf, bool right) {
            const int rel = c - P.nb + P.L;
            if (Lf) {
                if (right) leaf_value(P, [&](int s) { return S[s] - Lf[s]; }, vals + (size_t)rel * P.n_out);
                else leaf_value(P, [&](int s) { return Lf[s]; }, vals + (size_t)rel * P.n_out);
            } else {
                for (int s = 0; s < P.n_out; ++s) vals[(size_t)rel * P.n_out + s] = 0.f;
            }
            feats_out[rel] = -1;
            thrs_out[rel] = INFINITY;
            lc_out[rel] = -1;
            rc_out[rel] = -1;
            sb_out[rel] = 0;
        };
        const int bf = feat[l];
        const int br = bins_raw[l];
        const int bb = br & 0xFFFF;
        sb_out[l] = bb;
        if (!is_ok(l)) {
            feats_out[l] = -1;
            thrs_out[l] = INFINITY;
            lc_out[l] = -1;
            rc_out[l] = -1;
            if (P.heap) {
                small_right[l] = 0;
                lut[2 * l] = (int16_t)32767;
                lut[2 * l + 1] = (int16_t)32767;
                if (P.last) {                    // unreachable slots, still valid records
                    leaf_child(P.nb + 2 * l, nullptr, false);
                    leaf_child(P.nb + 2 * l + 1, nullptr, true);
                }
            }
            continue;
        }
        const bool fok = bf >= 0 && bf < P.d;
        int flag = bf;
        if (P.has_cat && fok && cat[bf]) flag |= HM_TREE_CAT;
        if ((br >> 16) & 1) flag |= HM_TREE_DLEFT;
        feats_out[l] = flag;
        thrs_out[l] = (fok && bb < P.E) ? edges[(size_t)bf * P.E + bb] : INFINITY;
        const int lc = P.nb + 2 * (P.heap ? l : rank);
        lc_out[l] = lc;
        rc_out[l] = lc + 1;
        if (P.last) {
            leaf_child(lc, left + (size_t)l * P.NS, false);
            leaf_child(lc + 1, left + (size_t)l * P.NS, true);
        }
        li_out[rank] = l;
        if (fok) atomicAdd(imp + bf, (double)gain[l]);   // split-gain importance
        const float* Lf = left + (size_t)l * P.NS;
        float rgt[8];
        float wl, wr;
        if (P.NS <= 8) {
            for (int s = 0; s < P.NS; ++s) rgt[s] = S[s] - Lf[s];
            wl = node_weight(Lf, P.NS, P.crit);
            wr = node_weight(rgt, P.NS, P.crit);
        } else {                               // many classes: weights are sums of counts
            wl = 0.f; wr = 0.f;
            for (int s = 0; s < P.NS; ++s) { wl += Lf[s]; wr += S[s] - Lf[s]; }
        }
        const int sr = wr < wl ? 1 : 0;
        const int key = P.heap ? l : rank;     // heap: segments / histograms indexed by parent
        small_right[key] = (uint8_t)sr;
        lut[2 * key + sr] = (int16_t)key;
        lut[2 * key + 1 - sr] = (int16_t)32767;
        ++rank;
    }
}

// ip: L, NS, d, E, crit, n_out, nb, has_cat, heap, last;  fp: lam, alpha, min_gain, min_split.
// last = 1: the children are leaves and their records are written too, at [L, L + 2 * splits)
// (heap: [L, 3L)) of the same pointers — the caller sizes them.  The per-node
// outputs (vals .. sb_out) are written at [0, L) of the pointers given (the caller offsets them to
// the level's first node id); li_out / small_right / lut are per split; imp [d] += split gains.
HM_API int hm_level_finalize(const int32_t* ip, const float* fp, const float* gain, const int32_t* feat,
                             const int32_t* bins_raw, const float* left, const float* tot, const float* edges,
                             const uint8_t* cat, float* vals, int32_t* feats_out, float* thrs_out, int32_t* lc_out,
                             int32_t* rc_out, int32_t* sb_out, int64_t* li_out, uint8_t* small_right, int16_t* lut,
                             int32_t* n_split, double* imp, hipStream_t stream) {
    LevelParams P;
    P.L = ip[0]; P.NS = ip[1]; P.d = ip[2]; P.E = ip[3]; P.crit = ip[4]; P.n_out = ip[5]; P.nb = ip[6];
    P.has_cat = ip[7];
    P.heap = ip[8];
    P.last = ip[9];
    P.lam = fp[0]; P.alpha = fp[1]; P.min_gain = fp[2]; P.min_split = fp[3];
    if (P.L <= 0 || P.NS <= 0 || (P.crit > 1 && P.NS > 8) || P.E <= 0) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(level_finalize_kernel, dim3(1), dim3(1024), 0, stream, P, gain, feat, bins_raw, left, tot,
                       edges, cat, vals, feats_out, thrs_out, lc_out, rc_out, sb_out, li_out, small_right, lut,
                       n_split, imp);
    HM_LAUNCH_RET();
}
