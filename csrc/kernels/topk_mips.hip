// Fused top-k maximum-inner-product search on the gfx950 matrix cores.
//
//   out[q] = top-KT over items n of  s(q, n) = <Q[q], I[n]> + item_bias[n]
//            (items excluded per query by a sorted CSR list, or n == q + self_offset)
//
// This is the GEMM-shaped hot op behind Hivemall's recommendation and similarity queries:
//   * mf_predict / bprmf_predict joined over every (user, item) pair followed by
//     each_top_k(k, user, score, item) — reference: core/src/main/java/hivemall/mf/
//     {MFPredictionUDF,BPRMFPredictionUDF}.java + tools/EachTopKUDTF.java (SURVEY.md §2.3.5,
//     §2.3.8, kernel K8) — with populate_not_in-style exclusion of already-seen items;
//   * cosine-similarity kNN over L2-normalised rows (knn/similarity/CosineSimilarityUDF.java,
//     the item-kNN restriction of train_slim).
// The M x N score matrix is never written: each tile of scores lives in MFMA accumulators
// for the few instructions it takes to filter it against the per-row running threshold.
//
// Design (MI355X-first):
//   * 256-thread block = 4 waves, BM = 64 query rows (16 per wave), items swept in tiles of
//     BN = 64, staged in stages of several tiles.  A fragments (the wave's 16 query rows,
//     Kd = 32*KS) stay in VGPRs for the whole launch; each stage is staged once per block in LDS
//     (XOR-swizzled 16-B chunks, so the 16 lanes of a ds_read_b128 phase cover all 64 banks)
//     and shared by the 4 waves.  The next stage is prefetched into registers while the MFMAs
//     and filters of the current one run (one-tile stages left the L2/MALL latency of the
//     prefetch exposed every 64 items: 6.4 ms for the ML-20M all-users top-10).
//   * The tile loop holds no global memory instruction in the common (no exclusion) variant:
//     with any VMEM load in the loop, hipcc's waitcnt pass drains vmcnt(0) before entering it,
//     i.e. waits for the stage prefetch right after issuing it (measured: the whole sweep ran
//     at one exposed L2/MALL latency per stage, 4.8-7 ms instead of ~1.x ms).  The exclusion
//     variant (binary search of the CSR list per candidate) keeps that drain.
//   * v_mfma_f32_16x16x32_bf16: lane l holds score(row 4*(l>>4)+r, item l&15) of each 16x16
//     sub-tile in accumulator register r.
//   * Running top-k per row in LDS: candidates (score > row threshold) are appended at
//     count + (prefix of the lane group's ballot) — counts and thresholds live in registers,
//     no LDS atomics.  After every 32-item half tile a row whose buffer could overflow is
//     compacted by its wave to its best KT (each entry ranked against all others through
//     v_readlane broadcasts, then moved to its rank), and the threshold becomes the KT-th score.
//     Measured on the ML-20M all-users top-10 sweep: a 128-element bitonic sort of shuffles
//     4.8 ms, ranking by LDS broadcast reads 6.6 ms (one LDS round trip per comparison).  After the first few tiles almost nothing passes the threshold, so the sweep
//     runs at MFMA + compare speed.
//   * Optional split of the item range over `splits` blocks per row block (small M): each
//     split writes its own top-KT; the caller merges (ops/topk_mips.py).
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BM = 64;      // query rows per block
constexpr int BN = 64;      // items per tile
constexpr int NT = 256;     // threads per block
constexpr int KT_MAX = 64;

struct MipsParams {
    int M, N, KT, splits, n_per_split;
    int self_offset;        // exclude n == q + self_offset when >= 0... (INT_MIN: off)
    int use_self;
};

// Entry order: higher score first; equal scores -> lower item index first.
__device__ __forceinline__ bool better(float sa, int ia, float sb, int ib) {
    return sa > sb || (sa == sb && ia < ib);
}

__device__ __forceinline__ bool is_excluded(const int64_t* __restrict__ ptr,
                                            const int32_t* __restrict__ ex, int q, int n) {
    int64_t lo = ptr[q], hi = ptr[q + 1];
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int v = ex[mid];
        if (v == n) return true;
        if (v < n) lo = mid + 1; else hi = mid;
    }
    return false;
}

// Swizzled chunk position: 16-B chunk c of tile row n (CPR chunks per row).
template <int CPR>
__device__ __forceinline__ int swz(int n, int c) {
    if constexpr (CPR >= 16) return n * CPR + (c ^ (n & 15));
    else return n * CPR + (c ^ ((n / (16 / CPR)) & (CPR - 1)));
}

// KS: Kd / 32.  CAPV: candidate slots per row (64 for KT <= 32, 96 for KT <= 64).
// A stage of TILES x 64 items is staged per barrier period (32 KB of LDS at CAPV = 64, 16 KB at
// 96, so the block stays at 64 KB and two blocks fit a CU); the next stage is prefetched into
// 32 VGPRs while the MFMAs and filters of the current one run.
template <int KS, int CAPV, bool EXCL>
__global__ __launch_bounds__(NT, 2) void mips_topk_kernel(
    MipsParams P, const bf16x8* __restrict__ Q, const bf16x8* __restrict__ I,
    const float* __restrict__ item_bias, const int64_t* __restrict__ ex_ptr,
    const int32_t* __restrict__ ex_idx, int32_t* __restrict__ out_idx, float* __restrict__ out_score)
{
    constexpr int CPR = 4 * KS;                          // 16-B chunks per row (Kd = 32*KS bf16)
    constexpr int TILES = (CAPV == 64 ? 8 : 4) / KS > 0 ? (CAPV == 64 ? 8 : 4) / KS : 1;
    constexpr int STAGE = BN * TILES;                    // items per stage
    constexpr int PRE = STAGE * CPR / NT;                // 16-B chunks per thread per stage
    __shared__ uint4 s_tile[STAGE * CPR];
    __shared__ float s_bias[STAGE];
    __shared__ float2 s_cand[BM * CAPV];                 // (score, item index bits)

    const int tid = threadIdx.x, lane = hm::lane_id(), w = hm::wave_id();
    const int g = lane >> 4;                             // lane group: rows 4g..4g+3 of the wave
    const int rb = blockIdx.x / P.splits, split = blockIdx.x % P.splits;
    const int q0 = rb * BM;
    const int n_begin = split * P.n_per_split;
    const int n_end = min(P.N, n_begin + P.n_per_split);
    const int KT = P.KT;

    // A fragments: the wave's 16 query rows, held for the whole sweep
    bf16x8 a[KS];
    {
        const int q = q0 + w * 16 + (lane & 15);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if (q < P.M) a[ks] = Q[(size_t)q * CPR + ks * 4 + (lane >> 4)];
            else a[ks] = bf16x8{};
        }
        // retire the A loads here: left pending, the loop-header merge of the waitcnt pass
        // made the first MFMA of every tile wait vmcnt(0), i.e. for the stage prefetch
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(a[ks]));
    }

    // register prefetch of one stage.  (A uint4[PRE] array stayed a stack object: stored to
    // scratch right after the loads — i.e. waited for at once — and reloaded at the commit;
    // a vector value is kept in VGPRs.)
    typedef uint32_t preg_t __attribute__((ext_vector_type(4 * PRE)));
    preg_t pre;
    float pre_b[(STAGE + NT - 1) / NT];
#define MIPS_FETCH(N0)                                                                         \
    do {                                                                                       \
        _Pragma("unroll") for (int r = 0; r < PRE; ++r) {                                      \
            const int e = tid + NT * r;                                                        \
            const int n = min((N0) + e / CPR, n_end - 1);                                      \
            const uint4 v_ = reinterpret_cast<const uint4*>(I)[(size_t)n * CPR + (e % CPR)];  \
            pre[4 * r] = v_.x; pre[4 * r + 1] = v_.y; pre[4 * r + 2] = v_.z; pre[4 * r + 3] = v_.w; \
        }                                                                                      \
        _Pragma("unroll") for (int r = 0; r < (STAGE + NT - 1) / NT; ++r)                      \
            pre_b[r] = item_bias ? item_bias[min((N0) + tid + NT * r, n_end - 1)] : 0.f;       \
    } while (0)
#define MIPS_COMMIT()                                                                          \
    do {                                                                                       \
        _Pragma("unroll") for (int r = 0; r < PRE; ++r) {                                      \
            const int e = tid + NT * r;                                                        \
            s_tile[swz<CPR>(e / CPR, e % CPR)] =                                               \
                make_uint4(pre[4 * r], pre[4 * r + 1], pre[4 * r + 2], pre[4 * r + 3]);         \
        }                                                                                      \
        _Pragma("unroll") for (int r = 0; r < (STAGE + NT - 1) / NT; ++r)                      \
            if (tid + NT * r < STAGE) s_bias[tid + NT * r] = pre_b[r];                         \
    } while (0)

    // Per-row state of this lane's 4 rows (uniform over the 16 lanes of the group): running
    // threshold and candidate count.  Kept in registers; no LDS atomics.
    const int rl0 = w * 16 + 4 * g;
    float thr[4];
    int cnt[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) { thr[r] = -INFINITY; cnt[r] = 0; }
    const uint64_t grp = 0xFFFFull << (16 * g);

    // Compact row rl (count c, wave-uniform) to its best KT by rank: entry j sits in lane j (and
    // lane j - 64), each lane ranks its own entries against all c of them — broadcast through
    // v_readlane into SGPRs, no LDS round trip per comparison — and the KT best move to their
    // rank.  Returns the new count; *kth receives the KT-th score when c >= KT.
    auto compact = [&](int rl, int c, float* kth) -> int {
        float2* row = s_cand + rl * CAPV;
        const float2 e0 = lane < c ? row[lane] : make_float2(-INFINITY, 0.f);
        const float2 e1 = (CAPV > 64 && lane + 64 < c) ? row[lane + 64] : make_float2(-INFINITY, 0.f);
        const int i0 = __float_as_int(e0.y), i1 = __float_as_int(e1.y);
        const int s0b = __float_as_int(e0.x), s1b = __float_as_int(e1.x);
        int r0 = 0, r1 = 0;
        const int c0 = c < 64 ? c : 64;
        for (int j = 0; j < c0; ++j) {
            const float oj = __int_as_float(__builtin_amdgcn_readlane(s0b, j));
            const int ij = __builtin_amdgcn_readlane(i0, j);
            r0 += better(oj, ij, e0.x, i0);
            if (CAPV > 64) r1 += better(oj, ij, e1.x, i1);
        }
        if (CAPV > 64) {
            for (int j = 64; j < c; ++j) {
                const float oj = __int_as_float(__builtin_amdgcn_readlane(s1b, j - 64));
                const int ij = __builtin_amdgcn_readlane(i1, j - 64);
                r0 += better(oj, ij, e0.x, i0);
                r1 += better(oj, ij, e1.x, i1);
            }
        }
        const bool v0 = lane < c, v1 = CAPV > 64 && lane + 64 < c;
        if (v0 && r0 < KT) row[r0] = e0;
        if (v1 && r1 < KT) row[r1] = e1;
        if (c >= KT) {
            const uint64_t m0 = __builtin_amdgcn_ballot_w64(v0 && r0 == KT - 1);
            const uint64_t m1 = __builtin_amdgcn_ballot_w64(v1 && r1 == KT - 1);
            *kth = m0 ? __shfl(e0.x, __builtin_ctzll(m0), 64) : __shfl(e1.x, __builtin_ctzll(m1), 64);
        }
        return c < KT ? c : KT;
    };
    auto wave_sync = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };

    if (n_begin < n_end) MIPS_FETCH(n_begin);
    __syncthreads();
    if (n_begin < n_end) MIPS_COMMIT();
    __syncthreads();

    for (int s0 = n_begin; s0 < n_end; s0 += STAGE) {
        if (s0 + STAGE < n_end) MIPS_FETCH(s0 + STAGE);  // in flight during the whole stage

        for (int t = 0; t < TILES; ++t) {
            const int n0 = s0 + t * BN;
            if (n0 >= n_end) break;
            // ---- 64 x 64 score tile on the matrix cores ----
            f32x4 acc[4];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
                const int n = t * BN + nt * 16 + (lane & 15);
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    const uint4 raw = s_tile[swz<CPR>(n, ks * 4 + (lane >> 4))];
                    bf16x8 b;
                    __builtin_memcpy(&b, &raw, 16);
                    acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], b, acc[nt], 0, 0, 0);
                }
            }
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const float bn = s_bias[t * BN + nt * 16 + (lane & 15)];
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[nt][r] += bn;
            }

            // ---- filter against the running thresholds, two 32-item halves ----
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                bool any = false;
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int n = n0 + (2 * h + u) * 16 + (lane & 15);
#pragma unroll
                    for (int r = 0; r < 4; ++r) any |= (n < n_end) & (acc[2 * h + u][r] > thr[r]);
                }
                if (!__builtin_amdgcn_ballot_w64(any)) continue;
                // candidate ballots of this half: m[r][u] (per row r of the lane group, 16-item
                // sub-tile u) and the number each row would append
                uint64_t m[4][2];
                int add[4];
#define MIPS_BALLOTS()                                                                         \
                _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                \
                    const int q = q0 + rl0 + r;                                                \
                    add[r] = 0;                                                                \
                    _Pragma("unroll") for (int u = 0; u < 2; ++u) {                            \
                        const int n = n0 + (2 * h + u) * 16 + (lane & 15);                     \
                        bool c = (n < n_end) & (acc[2 * h + u][r] > thr[r]) & (q < P.M);       \
                        if (EXCL) {                                                            \
                            if (c && P.use_self && n == q + P.self_offset) c = false;          \
                            if (c && ex_ptr) c = !is_excluded(ex_ptr, ex_idx, q, n);           \
                        }                                                                      \
                        m[r][u] = __builtin_amdgcn_ballot_w64(c);                              \
                        add[r] += __popcll(m[r][u] & grp);                                     \
                    }                                                                          \
                }
                MIPS_BALLOTS();
                // a row whose buffer would overflow is compacted first (only when it is really
                // full: reserving room for a whole half tile made KT close to the capacity
                // compact on every candidate — 76 ms instead of a few for KT = 64)
                // ... or, eagerly, once 16 entries beyond KT have accumulated: a tight threshold
                // keeps later halves on the fast path (capacity-only triggering: 7.1 ms, eager
                // at a fixed 32 free slots: 4.8-5.6 ms, but one compaction per candidate at KT
                // near the capacity)
                bool need = false;
#pragma unroll
                for (int r = 0; r < 4; ++r) need |= (cnt[r] + add[r] > CAPV) | (cnt[r] + add[r] >= KT + 16);
                if (__builtin_amdgcn_ballot_w64(need)) {
                    wave_sync();
                    // one (not unrolled) pass over the wave's 16 rows keeps a single copy of the
                    // compaction code in the loop (16 inlined copies made a 33-48 KB kernel)
                    for (int rr = 0; rr < 16; ++rr) {
                        const int gg = rr >> 2, r = rr & 3;
                        const int cr = r == 0 ? cnt[0] : r == 1 ? cnt[1] : r == 2 ? cnt[2] : cnt[3];
                        const int ar = r == 0 ? add[0] : r == 1 ? add[1] : r == 2 ? add[2] : add[3];
                        const int c = __shfl(cr, 16 * gg, 64);
                        const int ca = c + __shfl(ar, 16 * gg, 64);
                        if (ca > CAPV || ca >= KT + 16) {
                            float kth = -INFINITY;
                            const int nc = compact(w * 16 + rr, c, &kth);
                            if (g == gg) {
#pragma unroll
                                for (int k = 0; k < 4; ++k) {
                                    if (k == r) {
                                        cnt[k] = nc;
                                        if (c >= KT) thr[k] = kth;
                                    }
                                }
                            }
                        }
                    }
                    wave_sync();
                    MIPS_BALLOTS();     // thresholds moved
                }
#undef MIPS_BALLOTS
                // append: slot = count + prefix of the group's ballot (no atomics)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    int base = cnt[r];
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const uint64_t mu = m[r][u];
                        if ((mu >> lane) & 1ull) {
                            const uint64_t mg = mu & grp;
                            const int pos = base + (int)__builtin_amdgcn_mbcnt_hi(
                                (uint32_t)(mg >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mg, 0u));
                            s_cand[(rl0 + r) * CAPV + pos] =
                                make_float2(acc[2 * h + u][r], __int_as_float(n0 + (2 * h + u) * 16 + (lane & 15)));
                        }
                        base += __popcll(mu & grp);
                    }
                    cnt[r] = base;
                }
            }
        }
        __syncthreads();                                 // every wave is done with the stage
        if (s0 + STAGE < n_end) MIPS_COMMIT();
        __syncthreads();                                 // next stage visible
    }

    // ---- final: best KT of every row of this wave, in order ----
    wave_sync();
    for (int rr = 0; rr < 16; ++rr) {
        const int gg = rr >> 2, r = rr & 3;
        const int rl = w * 16 + rr;
        const int q = q0 + rl;
        const int cr = r == 0 ? cnt[0] : r == 1 ? cnt[1] : r == 2 ? cnt[2] : cnt[3];
        const int c = __shfl(cr, 16 * gg, 64);
        if (q < P.M) {
            float kth;
            const int nc = compact(rl, c, &kth);
            wave_sync();
            if (lane < KT) {
                const size_t o = ((size_t)split * P.M + q) * KT + lane;
                const float2 e = s_cand[rl * CAPV + lane];
                const bool ok = lane < nc;
                out_idx[o] = ok ? __float_as_int(e.y) : -1;
                out_score[o] = ok ? e.x : -INFINITY;
            }
        }
    }
}

#undef MIPS_FETCH
#undef MIPS_COMMIT

template <int KS>
int launch(const MipsParams& P, const void* Q, const void* I, const float* bias,
           const int64_t* ex_ptr, const int32_t* ex_idx, int32_t* oi, float* os, hipStream_t st) {
    const int blocks = ((P.M + BM - 1) / BM) * P.splits;
    const auto* q = reinterpret_cast<const bf16x8*>(Q);
    const auto* it = reinterpret_cast<const bf16x8*>(I);
    const bool ex = P.use_self || ex_ptr;
#define MIPS_GO(CAPV, EX) hipLaunchKernelGGL((mips_topk_kernel<KS, CAPV, EX>), dim3(blocks), dim3(NT), 0, st, \
                                            P, q, it, bias, ex_ptr, ex_idx, oi, os)
    if (P.KT <= 32) { if (ex) MIPS_GO(64, true); else MIPS_GO(64, false); }
    else { if (ex) MIPS_GO(96, true); else MIPS_GO(96, false); }
#undef MIPS_GO
    HM_LAUNCH_RET();
}

// ---------------------------------------------------------------------------------------------
// Register top-k variant (KT <= 32, the common recommendation sizes).  The score tile is
// computed transposed — v_mfma_f32_32x32x16_bf16 with the ITEMS as the A (row) operand and the
// QUERIES as the B (column) operand — so lane l owns query l & 31 for the whole sweep and holds
// 16 of every 32 items' scores (lane l ^ 32 holds the other 16).  Each lane keeps its own sorted
// top-KTC list in VGPRs (insertion = a compare/select network, no memory, no cross-lane
// coordination) and its threshold is always exact, so after the first tiles nearly every score
// fails one compare.  The two half-lists of a query are merged by shuffles at the end.
// Measured on the ML-20M all-users top-10 sweep (profiles/mips/): 2.8 ms (3.7 ms before the
// per-lane candidate queue) against 5-7 ms for the
// LDS-candidate-buffer kernel above (ballots, appends, compactions) and 46 ms for GEMM + topk.
// Counters: ~237K VALU instructions per wave, most of them in insertions (about one network
// pass per 32-item tile per wave, although typically one or two of the 64 lanes insert);
// prefetching the next tile's A fragments from LDS changed nothing at k = 10 and cost 55 % at
// k = 32 (VGPRs).
template <int KS2, int KTC, bool EXCL>
__global__ __launch_bounds__(NT) void mips_topk_reg_kernel(
    MipsParams P, const bf16x8* __restrict__ Q, const bf16x8* __restrict__ I,
    const float* __restrict__ item_bias, const int64_t* __restrict__ ex_ptr,
    const int32_t* __restrict__ ex_idx, int32_t* __restrict__ out_idx, float* __restrict__ out_score)
{
    constexpr int CPR = 2 * KS2;                         // 16-B chunks per row (Kd = 16*KS2)
    constexpr int STAGE = 32768 / (CPR * 16);            // items per 32 KB stage
    constexpr int PRE = STAGE * CPR / NT;                // = 8 chunks per thread
    constexpr int BQ = 128;                              // queries per block (32 per wave)
    typedef __attribute__((ext_vector_type(16))) float f32x16;
    __shared__ uint4 s_tile[STAGE * CPR];
    __shared__ float s_bias[STAGE];

    const int tid = threadIdx.x, lane = hm::lane_id(), w = hm::wave_id();
    const int h = lane >> 5;
    const int rb = blockIdx.x / P.splits, split = blockIdx.x % P.splits;
    const int q = rb * BQ + w * 32 + (lane & 31);
    const int n_begin = split * P.n_per_split;
    const int n_end = min(P.N, n_begin + P.n_per_split);
    const int KT = P.KT;

    // B fragments: this lane's query, k = 16 ks + 8 h + j
    bf16x8 b[KS2];
#pragma unroll
    for (int ks = 0; ks < KS2; ++ks) b[ks] = q < P.M ? Q[(size_t)q * CPR + 2 * ks + h] : bf16x8{};
#pragma unroll
    for (int ks = 0; ks < KS2; ++ks) asm volatile("" ::"v"(b[ks]));   // retire before the loop

    typedef uint32_t preg_t __attribute__((ext_vector_type(4 * PRE)));
    preg_t pre;
    float pre_b[(STAGE + NT - 1) / NT];
#define MIPS_FETCH(N0)                                                                         \
    do {                                                                                       \
        _Pragma("unroll") for (int r = 0; r < PRE; ++r) {                                      \
            const int e = tid + NT * r;                                                        \
            const int n = min((N0) + e / CPR, n_end - 1);                                      \
            const uint4 v_ = reinterpret_cast<const uint4*>(I)[(size_t)n * CPR + (e % CPR)];  \
            pre[4 * r] = v_.x; pre[4 * r + 1] = v_.y; pre[4 * r + 2] = v_.z; pre[4 * r + 3] = v_.w; \
        }                                                                                      \
        _Pragma("unroll") for (int r = 0; r < (STAGE + NT - 1) / NT; ++r)                      \
            pre_b[r] = item_bias ? item_bias[min((N0) + tid + NT * r, n_end - 1)] : 0.f;       \
    } while (0)
#define MIPS_COMMIT()                                                                          \
    do {                                                                                       \
        _Pragma("unroll") for (int r = 0; r < PRE; ++r) {                                      \
            const int e = tid + NT * r;                                                        \
            s_tile[swz<CPR>(e / CPR, e % CPR)] =                                               \
                make_uint4(pre[4 * r], pre[4 * r + 1], pre[4 * r + 2], pre[4 * r + 3]);         \
        }                                                                                      \
        _Pragma("unroll") for (int r = 0; r < (STAGE + NT - 1) / NT; ++r)                      \
            if (tid + NT * r < STAGE) s_bias[tid + NT * r] = pre_b[r];                         \
    } while (0)

    // sorted (descending) private top-KTC of this lane
    typedef __attribute__((ext_vector_type(KTC))) float lsv_t;   // vectors stay in VGPRs
    typedef __attribute__((ext_vector_type(KTC))) int liv_t;
    lsv_t ls;
    liv_t li;
#pragma unroll
    for (int i = 0; i < KTC; ++i) { ls[i] = -INFINITY; li[i] = INT_MAX; }
    float thr = -INFINITY;
    auto insert = [&](float sv, int nv) {
#pragma unroll
        for (int i = 0; i < KTC; ++i) {
            const bool c = better(sv, nv, ls[i], li[i]);
            const float ts = ls[i];
            const int ti = li[i];
            ls[i] = c ? sv : ts;
            li[i] = c ? nv : ti;
            sv = c ? ts : sv;
            nv = c ? ti : nv;
        }
    };
    auto kth = [&]() {
        float t = ls[0];
#pragma unroll
        for (int i = 1; i < KTC; ++i) t = (i == KT - 1) ? ls[i] : t;
        return t;
    };

    // per-lane queue of candidates not yet in the sorted list
    float qs0 = 0.f, qs1 = 0.f, qs2 = 0.f, qs3 = 0.f;
    int qi0 = 0, qi1 = 0, qi2 = 0, qi3 = 0, qn = 0;
    auto flush_queue = [&]() {
        if (qn > 0) insert(qs0, qi0);
        if (qn > 1) insert(qs1, qi1);
        if (qn > 2) insert(qs2, qi2);
        if (qn > 3) insert(qs3, qi3);
        qn = 0;
        thr = kth();
    };

    if (n_begin < n_end) MIPS_FETCH(n_begin);
    __syncthreads();
    if (n_begin < n_end) MIPS_COMMIT();
    __syncthreads();

    for (int s0 = n_begin; s0 < n_end; s0 += STAGE) {
        if (s0 + STAGE < n_end) MIPS_FETCH(s0 + STAGE);

        for (int t = 0; t < STAGE / 32; ++t) {
            const int n0 = s0 + t * 32;
            if (n0 >= n_end) break;
            f32x16 acc = {};
            const int it = t * 32 + (lane & 31);
#pragma unroll
            for (int ks = 0; ks < KS2; ++ks) {
                const uint4 raw = s_tile[swz<CPR>(it, 2 * ks + h)];
                bf16x8 a;
                __builtin_memcpy(&a, &raw, 16);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[ks], acc, 0, 0, 0);
            }
            // lane's items: n0 + (reg & 3) + 8 (reg >> 2) + 4 h
            const int ib = t * 32 + 4 * h;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float4 bb = *reinterpret_cast<const float4*>(&s_bias[ib + 8 * j]);
                acc[4 * j] += bb.x; acc[4 * j + 1] += bb.y; acc[4 * j + 2] += bb.z; acc[4 * j + 3] += bb.w;
            }
            const int nb = n0 + 4 * h;
            if (n0 + 32 > n_end) {                       // tail tile only (uniform branch)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (nb + (r & 3) + 8 * (r >> 2) >= n_end) acc[r] = -INFINITY;
            }
            // fast path: 16 compares against the exact threshold (their lane masks OR-ed on
            // the scalar unit); per-register bit masks are built only when something passes
            bool any = false;
#pragma unroll
            for (int r = 0; r < 16; ++r) any |= acc[r] > thr;
            if (!__builtin_amdgcn_ballot_w64(any)) continue;
            // pending candidates of this lane as a bit mask; one insertion site (a copy of the
            // network per register made the compile run for tens of minutes)
            uint32_t pend = 0u;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = nb + (r & 3) + 8 * (r >> 2);
                bool c = acc[r] > thr;
                if (EXCL) {
                    if (c && P.use_self && n == q + P.self_offset) c = false;
                    if (c && ex_ptr && q < P.M) c = !is_excluded(ex_ptr, ex_idx, q, n);
                }
                pend |= (uint32_t)c << r;
            }
            // append to the lane's 4-entry queue (~30 VALU per lockstep pass); the sorted lists
            // are updated only when some lane's queue is full — late in the sweep one or two of
            // the 64 lanes have a candidate per tile, and a full insertion pass per tile for the
            // whole wave was most of the kernel's VALU work
            while (__builtin_amdgcn_ballot_w64(pend != 0u)) {
                if (pend && qn < 4) {
                    const int r = __builtin_ctz(pend);
                    pend &= pend - 1u;
                    float sv = acc[0];
#pragma unroll
                    for (int k = 1; k < 16; ++k) sv = r == k ? acc[k] : sv;
                    const int nv = nb + (r & 3) + 8 * (r >> 2);
                    qs0 = qn == 0 ? sv : qs0; qi0 = qn == 0 ? nv : qi0;
                    qs1 = qn == 1 ? sv : qs1; qi1 = qn == 1 ? nv : qi1;
                    qs2 = qn == 2 ? sv : qs2; qi2 = qn == 2 ? nv : qi2;
                    qs3 = qn == 3 ? sv : qs3; qi3 = qn == 3 ? nv : qi3;
                    ++qn;
                }
                if (__builtin_amdgcn_ballot_w64(qn == 4 && pend != 0u)) {
                    flush_queue();
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        if (!(acc[r] > thr)) pend &= ~(1u << r);
                }
            }
        }
        __syncthreads();
        if (s0 + STAGE < n_end) MIPS_COMMIT();
        __syncthreads();
    }

    flush_queue();
    // merge the two half-lists of each query: lanes l + 32 publish theirs through LDS (the
    // stage buffer is free now), lanes l insert them
    float2* s_half = reinterpret_cast<float2*>(s_tile) + (size_t)w * 32 * KTC;
    if (h == 1) {
#pragma unroll
        for (int i = 0; i < KTC; ++i) s_half[(lane & 31) * KTC + i] = make_float2(ls[i], __int_as_float(li[i]));
    }
    __syncthreads();
    if (h == 0) {
        for (int i = 0; i < KT; ++i) {
            const float2 e = s_half[lane * KTC + i];
            insert(e.x, __float_as_int(e.y));
        }
    }
    if (h == 0 && q < P.M) {
        const size_t o = ((size_t)split * P.M + q) * KT;
#pragma unroll
        for (int i = 0; i < KTC; ++i) {
            if (i < KT) {
                const bool ok = ls[i] != -INFINITY || li[i] != INT_MAX;
                out_idx[o + i] = ok ? li[i] : -1;
                out_score[o + i] = ok ? ls[i] : -INFINITY;
            }
        }
    }
#undef MIPS_FETCH
#undef MIPS_COMMIT
}

template <int KS2>
int launch_reg(const MipsParams& P, const void* Q, const void* I, const float* bias,
               const int64_t* ex_ptr, const int32_t* ex_idx, int32_t* oi, float* os, hipStream_t st) {
    const int blocks = ((P.M + 127) / 128) * P.splits;
    const auto* q = reinterpret_cast<const bf16x8*>(Q);
    const auto* it = reinterpret_cast<const bf16x8*>(I);
    const bool ex = P.use_self || ex_ptr;
#define MIPS_GO(KTC, EX) hipLaunchKernelGGL((mips_topk_reg_kernel<KS2, KTC, EX>), dim3(blocks), dim3(NT), 0, st, \
                                           P, q, it, bias, ex_ptr, ex_idx, oi, os)
    if (P.KT <= 8) { if (ex) MIPS_GO(8, true); else MIPS_GO(8, false); }
    else if (P.KT <= 16) { if (ex) MIPS_GO(16, true); else MIPS_GO(16, false); }
    else { if (ex) MIPS_GO(32, true); else MIPS_GO(32, false); }
#undef MIPS_GO
    HM_LAUNCH_RET();
}

}  // namespace

// Q [M][Kd] bf16, I [N][Kd] bf16 (Kd = 32, 64, 128 or 256; zero-padded by the caller),
// item_bias [N] fp32 or null, exclusion CSR (ex_ptr [M+1] int64, ex_idx sorted per row) or null,
// self_offset: exclude item q + self_offset for query q (use_self = 1).
// Output [splits][M][KT] (idx int32, -1 = none; score fp32, -inf = none), best first.
HM_API int hm_mips_topk(int M, int N, int Kd, int KT, int splits, int use_self, int self_offset,
                        const void* Q, const void* I, const float* item_bias,
                        const int64_t* ex_ptr, const int32_t* ex_idx,
                        int32_t* out_idx, float* out_score, hipStream_t stream) {
    if (M <= 0 || N <= 0 || KT <= 0 || KT > KT_MAX || splits <= 0) return (int)hipErrorInvalidValue;
    MipsParams P;
    P.M = M; P.N = N; P.KT = KT; P.splits = splits;
    P.n_per_split = ((N + splits - 1) / splits + BN - 1) / BN * BN;
    P.use_self = use_self; P.self_offset = self_offset;
    if (KT <= 32) {
        switch (Kd) {
            case 32: return launch_reg<2>(P, Q, I, item_bias, ex_ptr, ex_idx, out_idx, out_score, stream);
            case 64: return launch_reg<4>(P, Q, I, item_bias, ex_ptr, ex_idx, out_idx, out_score, stream);
            case 128: return launch_reg<8>(P, Q, I, item_bias, ex_ptr, ex_idx, out_idx, out_score, stream);
            case 256: return launch_reg<16>(P, Q, I, item_bias, ex_ptr, ex_idx, out_idx, out_score, stream);
            default: return (int)hipErrorInvalidValue;
        }
    }
    switch (Kd) {
        case 32: return launch<1>(P, Q, I, item_bias, ex_ptr, ex_idx, out_idx, out_score, stream);
        case 64: return launch<2>(P, Q, I, item_bias, ex_ptr, ex_idx, out_idx, out_score, stream);
        case 128: return launch<4>(P, Q, I, item_bias, ex_ptr, ex_idx, out_idx, out_score, stream);
        case 256: return launch<8>(P, Q, I, item_bias, ex_ptr, ex_idx, out_idx, out_score, stream);
        default: return (int)hipErrorInvalidValue;
    }
}
