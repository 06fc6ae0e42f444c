// Factorization machine (Rendle 2010) fused train / predict kernel for gfx950.
//
// Semantics: Hivemall FactorizationMachineUDTF (train_fm) as pinned in docs/compat.md
// (upstream core/src/main/java/hivemall/fm/FactorizationMachineUDTF.java,
// FactorizationMachineModel.java):
//   p   = w0 + Σ w_i x_i + ½ Σ_f [(Σ_i v_if x_i)² − Σ_i v_if² x_i²]
//   d   = dloss/dp : classification −y/(1+exp(y p)) (y ∈ {−1,+1}); regression clip(p) − y
//   w0 -= η (d + 2 λ0 w0) ; w_i -= η (d x_i + 2 λw w_i)
//   v_if -= η (d x_i (S_f − v_if x_i) + 2 λv v_if),   S_f = Σ_j v_jf x_j
//   η = eta0 / t^power_t (inverse) | eta0 (fixed) | eta0/(1+t/total) (simple)
//
// MI355X design:
//   * V is a [dims][KP] table in bf16 (default; Criteo-1TB config) or fp32.  One row of V is
//     KP·2 bytes = one 16-B load for KP = 8: every lane gathers its feature's whole factor
//     vector with a single dwordx4 load.
//   * bf16 updates use stochastic rounding (hash-based, deterministic per (row, feature,
//     factor, seed)) so the SGD steps that are far below one bf16 ulp are kept in
//     expectation instead of being rounded away.
//   * one wave64 = one row; lanes span the non-zeros (Criteo: 39 of 64 lanes); S_f and the
//     linear term are DPP wave reductions; the ½Σ v²x² term is folded into one reduction.
//   * 4 waves per 256-thread block, grid-stride over rows; Hogwild across waves (no atomics
//     except the single global-bias add per row).
#include "common.h"

namespace {

// w0 shard i lives at w0[i * W0_STRIDE] (its own 128-B line: atomics to one line serialise)
constexpr int W0_STRIDE = 32;

struct FMParams {
    int dims, k;              // k = real factor count (<= KP)
    int classification, train;
    int eta_kind;             // 0 fixed, 1 simple, 2 inverse
    float eta0, power_t, total_steps;
    float lambda0, lambda_w, lambda_v;
    float min_target, max_target;
    int use_w0;
    int w0_shards;            // w0 = sum of w0[0..w0_shards) (<= 64)
    int w0_every;             // fm_pipe_kernel: most rows between re-reads of the w0 shards (>= 1)
    float w0_tol;             // ... and a re-read as soon as the wave's own bias steps since the
                              // last one add up to more than w0_tol x eta (0: off)
    uint32_t seed;
    const uint8_t* hot;       // per-feature flags (nullable): a hot feature's V row / w stores go
                              // out SC1 (write-through, dropped from the writer's XCD L2) ...
    uint32_t hot_mask;        // ... on the rows whose hash & hot_mask == 0 (0: every row)
    int xcds;                 // fm_pipe_kernel: waves on this many of the 8 XCDs (8: all; fewer:
                              // only blocks with blockIdx % 8 < xcds work — round-robin placement)
    long long vstride;        // V elements between feature rows (>= KP)
    long long wstride;        // floats between features' w (1: its own array; a record: inside
                              // the feature's V row, so the gather and the store touch one line)
};

// w of feature i (strided: separate array or a field of the feature's record)
#define FW(i) w[(size_t)(i) * (size_t)P.wstride]

__device__ __forceinline__ float fm_eta(const FMParams& P, float t) {
    if (P.eta_kind == 0) return P.eta0;
    if (P.eta_kind == 1) return P.total_steps > 0.f ? P.eta0 / (1.f + t / P.total_steps) : P.eta0;
    return P.eta0 / powf(t > 1.f ? t : 1.f, P.power_t);
}

__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ c * 0xC2B2AE3Du;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    return h;
}


// Buffer-store / -load cache policy: SC1 (bit 4).  An SC1 store writes through and DROPS the line
// from the writing XCD's L2; an SC1 load bypasses the CU's L1 (MI355X_MICROARCH.md §Workgroup
// dispatch).  Per-XCD L2s are not coherent: with plain stores an XCD keeps reading its own copy
// of a hot feature's line while the other seven update theirs.
constexpr int CPOL_SC1 = 16;
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
typedef uint32_t u2v __attribute__((ext_vector_type(2)));

template <int KP, bool BF16>
struct VRow {
    float v[KP];
    // WT: the same row load / store through buffer ops with SC1 (rsrc over V, byte offsets < 4 GiB)
    __device__ __forceinline__ void load_sc1(__amdgpu_buffer_rsrc_t rs, int i, size_t vs) {
        const uint32_t off = (uint32_t)((size_t)i * vs * (BF16 ? 2 : 4));
        if constexpr (BF16) {
            if constexpr (KP % 8 == 0) {
#pragma unroll
                for (int c = 0; c < KP / 8; ++c) {
                    const u4v q = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16u * c, 0, CPOL_SC1);
                    const uint32_t wds[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        v[c * 8 + 2 * j] = __uint_as_float(wds[j] << 16);
                        v[c * 8 + 2 * j + 1] = __uint_as_float(wds[j] & 0xFFFF0000u);
                    }
                }
            } else {
                const u2v q = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, CPOL_SC1);
                v[0] = __uint_as_float(q.x << 16);
                v[1] = __uint_as_float(q.x & 0xFFFF0000u);
                v[2] = __uint_as_float(q.y << 16);
                v[3] = __uint_as_float(q.y & 0xFFFF0000u);
            }
        } else {
#pragma unroll
            for (int c = 0; c < KP / 4; ++c) {
                const u4v q = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16u * c, 0, CPOL_SC1);
                v[4 * c] = __uint_as_float(q.x); v[4 * c + 1] = __uint_as_float(q.y);
                v[4 * c + 2] = __uint_as_float(q.z); v[4 * c + 3] = __uint_as_float(q.w);
            }
        }
    }
    __device__ __forceinline__ void store_sc1(__amdgpu_buffer_rsrc_t rs, int i, size_t vs, uint32_t rbase) const {
        const uint32_t off = (uint32_t)((size_t)i * vs * (BF16 ? 2 : 4));
        if constexpr (BF16) {
            uint32_t wds[KP / 2];
#pragma unroll
            for (int j = 0; j < KP / 2; ++j) {
                const uint32_t r = hash3(rbase, (uint32_t)i, (uint32_t)j);
                wds[j] = hm::pack_bf16x2_sr(v[2 * j], r, v[2 * j + 1], r >> 16 | r << 16);
            }
            if constexpr (KP % 8 == 0) {
#pragma unroll
                for (int c = 0; c < KP / 8; ++c)
                    __builtin_amdgcn_raw_buffer_store_b128((u4v){wds[4 * c], wds[4 * c + 1], wds[4 * c + 2], wds[4 * c + 3]},
                                                           rs, off + 16u * c, 0, CPOL_SC1);
            } else {
                __builtin_amdgcn_raw_buffer_store_b64((u2v){wds[0], wds[1]}, rs, off, 0, CPOL_SC1);
            }
        } else {
#pragma unroll
            for (int c = 0; c < KP / 4; ++c)
                __builtin_amdgcn_raw_buffer_store_b128((u4v){__float_as_uint(v[4 * c]), __float_as_uint(v[4 * c + 1]),
                                                             __float_as_uint(v[4 * c + 2]), __float_as_uint(v[4 * c + 3])},
                                                       rs, off + 16u * c, 0, CPOL_SC1);
        }
    }
    __device__ __forceinline__ void load(const void* V, int i, size_t vs) {
        if constexpr (BF16) {
            const uint16_t* p = reinterpret_cast<const uint16_t*>(V) + (size_t)i * vs;
            if constexpr (KP % 8 == 0) {
#pragma unroll
                for (int c = 0; c < KP / 8; ++c) {
                    const uint4 q = reinterpret_cast<const uint4*>(p)[c];
                    const uint32_t wds[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        v[c * 8 + 2 * j] = __uint_as_float(wds[j] << 16);
                        v[c * 8 + 2 * j + 1] = __uint_as_float(wds[j] & 0xFFFF0000u);
                    }
                }
            } else {
                const uint2 q = *reinterpret_cast<const uint2*>(p);  // KP == 4
                v[0] = __uint_as_float(q.x << 16);
                v[1] = __uint_as_float(q.x & 0xFFFF0000u);
                v[2] = __uint_as_float(q.y << 16);
                v[3] = __uint_as_float(q.y & 0xFFFF0000u);
            }
        } else {
            const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(V) + (size_t)i * vs);
#pragma unroll
            for (int c = 0; c < KP / 4; ++c) {
                const float4 q = p[c];
                v[4 * c] = q.x; v[4 * c + 1] = q.y; v[4 * c + 2] = q.z; v[4 * c + 3] = q.w;
            }
        }
    }
    __device__ __forceinline__ void store(void* V, int i, size_t vs, uint32_t rbase) const {
        if constexpr (BF16) {
            uint16_t* p = reinterpret_cast<uint16_t*>(V) + (size_t)i * vs;
            uint32_t wds[KP / 2];
#pragma unroll
            for (int j = 0; j < KP / 2; ++j) {
                const uint32_t r = hash3(rbase, (uint32_t)i, (uint32_t)j);
                wds[j] = hm::pack_bf16x2_sr(v[2 * j], r, v[2 * j + 1], r >> 16 | r << 16);
            }
            if constexpr (KP % 8 == 0) {
#pragma unroll
                for (int c = 0; c < KP / 8; ++c)
                    reinterpret_cast<uint4*>(p)[c] = make_uint4(wds[4 * c], wds[4 * c + 1], wds[4 * c + 2], wds[4 * c + 3]);
            } else {
                *reinterpret_cast<uint2*>(p) = make_uint2(wds[0], wds[1]);
            }
        } else {
            float4* p = reinterpret_cast<float4*>(reinterpret_cast<float*>(V) + (size_t)i * vs);
#pragma unroll
            for (int c = 0; c < KP / 4; ++c) p[c] = make_float4(v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]);
        }
    }
};

template <int KP, bool BF16>
__global__ __launch_bounds__(256) void fm_kernel(FMParams P, const int64_t* __restrict__ indptr,
                                                 const int32_t* __restrict__ idx,
                                                 const float* __restrict__ val,
                                                 const float* __restrict__ y, int64_t n_rows,
                                                 int64_t t0, float* __restrict__ w,
                                                 void* __restrict__ V, float* __restrict__ w0,
                                                 float* __restrict__ pred, float* __restrict__ loss) {
    const int lane = hm::lane_id();
    const int64_t gw = (int64_t)blockIdx.x * (blockDim.x / 64) + hm::wave_id();
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t row = gw; row < n_rows; row += nw) {
        const int64_t s = indptr[row], e = indptr[row + 1];
        const int nnz = (int)(e - s);
        // global-bias shards (one 128-B line each) are read at the top of the row, in flight
        // with the feature gathers instead of after the reductions
        const float w0part = (P.use_w0 && lane < P.w0_shards) ? w0[lane * W0_STRIDE] : 0.f;
        // ---- forward: lanes over non-zeros (chunks of 64) ----
        float S[KP];
#pragma unroll
        for (int f = 0; f < KP; ++f) S[f] = 0.f;
        float lin = 0.f, sq = 0.f;
        VRow<KP, BF16> vr;
        int ci = -1;
        float cx = 0.f, cw = 0.f;
        for (int base = 0; base < nnz; base += 64) {
            const int j = base + lane;
            int i = -1;
            float x = 0.f;
            if (j < nnz) {
                i = idx[s + j];
                x = val ? val[s + j] : 1.f;
                if (i < 0 || i >= P.dims) i = -1;
            }
            VRow<KP, BF16> t;
            float wi = 0.f;
            if (i >= 0) {
                t.load(V, i, P.vstride);
                wi = FW(i);
            } else {
#pragma unroll
                for (int f = 0; f < KP; ++f) t.v[f] = 0.f;
                x = 0.f;
            }
            lin += wi * x;
#pragma unroll
            for (int f = 0; f < KP; ++f) {
                const float vx = t.v[f] * x;
                S[f] += vx;
                sq += vx * vx;
            }
            if (base == 0) { vr = t; ci = i; cx = x; cw = wi; }
        }
        lin = hm::wave_sum(lin);
        sq = hm::wave_sum(sq);
        float pair = 0.f;
#pragma unroll
        for (int f = 0; f < KP; ++f) {
            S[f] = hm::wave_sum(S[f]);
            pair += S[f] * S[f];
        }
        float p = lin + 0.5f * (pair - sq);
        const float w0v = P.use_w0 ? hm::wave_sum(w0part) : 0.f;
        p += w0v;
        const float yy = y ? y[row] : 0.f;
        float d;
        if (P.classification) {
            const float z = yy * p;
            d = -yy / (1.f + __expf(z));
            if (lane == 0) {
                if (pred) pred[row] = p;
                if (loss) loss[row] = hm::log1pexp(-z);
            }
        } else {
            const float pc = fminf(fmaxf(p, P.min_target), P.max_target);
            d = pc - yy;
            if (lane == 0) {
                if (pred) pred[row] = pc;
                if (loss) loss[row] = 0.5f * d * d;
            }
        }
        if (!P.train) continue;
        const float eta = fm_eta(P, (float)(t0 + row + 1));
        const uint32_t rbase = P.seed ^ (uint32_t)(t0 + row) * 0x9E3779B9u;
        auto upd = [&](VRow<KP, BF16>& t, int i, float x, float wi) {
            FW(i) = wi - eta * (d * x + 2.f * P.lambda_w * wi);
#pragma unroll
            for (int f = 0; f < KP; ++f) {
                const float g = d * x * (S[f] - t.v[f] * x) + 2.f * P.lambda_v * t.v[f];
                t.v[f] = f < P.k ? t.v[f] - eta * g : 0.f;
            }
            t.store(V, i, P.vstride, rbase);
        };
        if (ci >= 0) upd(vr, ci, cx, cw);
        for (int base = 64; base < nnz; base += 64) {  // rows wider than one wave
            const int j = base + lane;
            if (j >= nnz) continue;
            const int i = idx[s + j];
            if (i < 0 || i >= P.dims) continue;
            const float x = val ? val[s + j] : 1.f;
            VRow<KP, BF16> t;
            t.load(V, i, P.vstride);
            upd(t, i, x, FW(i));
        }
        // per-row atomic (batching w0 deltas per wave was measured to diverge: every wave's
        // locally-converged delta is summed -> ~#waves x overshoot on the hottest parameter),
        // into one of w0_shards addresses: a single address serialised every row of the chip
        // (~40 M rows/s at any grid, profiles/fm_grid_probe_r1.log); the sum of the shards
        // receives exactly the same per-row deltas
        if (P.use_w0 && lane == 0)
            atomicAdd(w0 + (int)(gw % P.w0_shards) * W0_STRIDE, -eta * (d + 2.f * P.lambda0 * w0v));
    }
}

// Pipelined variant (default): the same per-row math and Hogwild update as fm_kernel, with the
// row's dependent load chain taken off the critical path.  A wave's next row (row + nw) has its
// CSR bounds loaded one iteration ahead and its indices/values at the top of the current
// iteration (read-only data, so nothing goes stale): on entry to a row only the V/w gathers are
// left to wait for — one global round trip instead of three (indptr -> idx -> V).  V is NOT
// prefetched across rows: the wave's own update of the current row may touch the next row's
// features.  Reductions are DPP wave sums (~8 instructions against ~36 for the shuffle
// butterfly; EXEC is full in the forward pass).
// WT (A/B experiment, variant 2 / 3): 1 = every V row / w store SC1 (write-through, dropped from
// the writer's L2), 2 = also the row gathers SC1 (past the CU's L1).
template <int KP, bool BF16, int WT = 0>
__global__ __launch_bounds__(256) void fm_pipe_kernel(FMParams P, const int64_t* __restrict__ indptr,
                                                      const int32_t* __restrict__ idx,
                                                      const float* __restrict__ val,
                                                      const float* __restrict__ y, int64_t n_rows,
                                                      int64_t t0, float* __restrict__ w,
                                                      void* __restrict__ V, float* __restrict__ w0,
                                                      float* __restrict__ pred, float* __restrict__ loss) {
    const int lane = hm::lane_id();
    // XCD confinement (P.xcds < 8): the launch has 8 / xcds x the blocks and only those with
    // blockIdx % 8 < xcds work, i.e. every wave on xcds XCDs under round-robin placement (speed and
    // staleness only, never correctness): one XCD's L2 is a coherent copy of the hot features
    const int bx = (int)blockIdx.x;
    if (P.xcds < 8 && (bx & 7) >= P.xcds) return;
    const int64_t lbx = P.xcds < 8 ? (int64_t)(bx >> 3) * P.xcds + (bx & 7) : (int64_t)bx;
    const int64_t lgrid = P.xcds < 8 ? (int64_t)(gridDim.x >> 3) * P.xcds : (int64_t)gridDim.x;
    const int64_t gw = lbx * (blockDim.x / 64) + hm::wave_id();
    const int64_t nw = lgrid * (blockDim.x / 64);
    if (gw >= n_rows) return;                                  // wave-uniform
    // pipeline registers: bounds of the current row, first-chunk (index, value) of it
    int64_t s = indptr[gw], e = indptr[gw + 1];
    int ci = -1;
    float cx = 0.f;
    if (lane < e - s) {
        ci = idx[s + lane];
        cx = val ? val[s + lane] : 1.f;
    }
    int64_t ns = 0, ne = 0;                                   // bounds of row + nw
    if (gw + nw < n_rows) { ns = indptr[gw + nw]; ne = indptr[gw + nw + 1]; }
    // the global-bias shards are read one row ahead too: the atomics of the other waves keep
    // those lines out of L2, so a same-row read was a memory round trip on the critical path
    // (one row of extra staleness on a parameter every wave of the chip updates anyway)
    float w0part = (P.use_w0 && lane < P.w0_shards) ? w0[lane * W0_STRIDE] : 0.f;
    float yy = y ? y[gw] : 0.f;
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(V, (short)0, -1, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(w, (short)0, -1, 0x00020000);
    int since = 0;            // rows since the last re-read of the shards
    float acc = 0.f;          // the wave's own bias steps since then (wave-uniform)
    for (int64_t row = gw; row < n_rows; row += nw) {
        const int nnz = (int)(e - s);
        int i = (ci >= 0 && ci < P.dims) ? ci : -1;
        // the w0 shards are re-read at most every w0_every rows; in between the wave adds its
        // own deltas to its copy (lane 0), so only the other waves' updates are seen late.  The
        // re-read comes early when the wave's own steps drift one way (|sum| > w0_tol x eta):
        // the bias is then moving, and every other wave's copy with it (early training)
        const bool w0_ref = P.w0_every <= 1 || since + 1 >= P.w0_every ||
                            (P.w0_tol > 0.f && fabsf(acc) > P.w0_tol * fm_eta(P, (float)(t0 + row + 1)));
        float x = i >= 0 ? cx : 0.f;
        // ---- gathers of this row (the only loads the forward waits for) ----
        VRow<KP, BF16> vr;
        float wi = 0.f;
        // the hot flag is loaded with the gathers (needed only at the update store)
        const bool hotf = WT == 0 && P.hot != nullptr && i >= 0 && P.hot[i] != 0 &&
                          (hash3(P.seed, (uint32_t)(t0 + row), (uint32_t)i) & P.hot_mask) == 0u;
        if (i >= 0) {
            if constexpr (WT == 2) {
                vr.load_sc1(vrs, i, P.vstride);
                wi = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                         wrs, (uint32_t)((size_t)i * P.wstride * 4), 0, CPOL_SC1));
            } else {
                vr.load(V, i, P.vstride);
                wi = FW(i);
            }
        } else {
#pragma unroll
            for (int f = 0; f < KP; ++f) vr.v[f] = 0.f;
        }
        // ---- prefetch: next row's indices/values/label/bias shards, the row after's bounds ----
        const int64_t nrow = row + nw;
        int pi = -1;
        float px = 0.f, pw0 = 0.f, py = 0.f;
        int64_t ns2 = 0, ne2 = 0;
        if (nrow < n_rows) {
            if (w0_ref) pw0 = (P.use_w0 && lane < P.w0_shards) ? w0[lane * W0_STRIDE] : 0.f;
            py = y ? y[nrow] : 0.f;
            if (lane < ne - ns) {
                pi = idx[ns + lane];
                px = val ? val[ns + lane] : 1.f;
            }
            if (nrow + nw < n_rows) { ns2 = indptr[nrow + nw]; ne2 = indptr[nrow + nw + 1]; }
        }
        // ---- forward ----
        float S[KP];
        float lin = wi * x, sq = 0.f;
#pragma unroll
        for (int f = 0; f < KP; ++f) {
            const float vx = vr.v[f] * x;
            S[f] = vx;
            sq += vx * vx;
        }
        for (int base = 64; base < nnz; base += 64) {             // rows wider than one wave
            const int j = base + lane;
            int i2 = -1;
            float x2 = 0.f;
            if (j < nnz) {
                i2 = idx[s + j];
                x2 = val ? val[s + j] : 1.f;
                if (i2 < 0 || i2 >= P.dims) i2 = -1;
            }
            if (i2 >= 0) {
                VRow<KP, BF16> t;
                t.load(V, i2, P.vstride);
                lin += FW(i2) * x2;
#pragma unroll
                for (int f = 0; f < KP; ++f) {
                    const float vx = t.v[f] * x2;
                    S[f] += vx;
                    sq += vx * vx;
                }
            }
        }
        lin = hm::wave_sum_uniform(lin);
        sq = hm::wave_sum_uniform(sq);
        float pair = 0.f;
#pragma unroll
        for (int f = 0; f < KP; ++f) {
            S[f] = hm::wave_sum_uniform(S[f]);
            pair += S[f] * S[f];
        }
        float p = lin + 0.5f * (pair - sq);
        const float w0v = P.use_w0 ? hm::wave_sum_uniform(w0part) : 0.f;
        p += w0v;
        float d;
        if (P.classification) {
            const float z = yy * p;
            d = -yy / (1.f + __expf(z));
            if (lane == 0) {
                if (pred) pred[row] = p;
                if (loss) loss[row] = hm::log1pexp(-z);
            }
        } else {
            const float pc = fminf(fmaxf(p, P.min_target), P.max_target);
            d = pc - yy;
            if (lane == 0) {
                if (pred) pred[row] = pc;
                if (loss) loss[row] = 0.5f * d * d;
            }
        }
        if (P.train) {
            const float eta = fm_eta(P, (float)(t0 + row + 1));
            const uint32_t rbase = P.seed ^ (uint32_t)(t0 + row) * 0x9E3779B9u;
            auto upd = [&](VRow<KP, BF16>& t, int ii, float xx, float ww) {
                const float nw = ww - eta * (d * xx + 2.f * P.lambda_w * ww);
#pragma unroll
                for (int f = 0; f < KP; ++f) {
                    const float g = d * xx * (S[f] - t.v[f] * xx) + 2.f * P.lambda_v * t.v[f];
                    t.v[f] = f < P.k ? t.v[f] - eta * g : 0.f;
                }
                if constexpr (WT > 0) {
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nw), wrs,
                                                          (uint32_t)((size_t)ii * P.wstride * 4), 0, CPOL_SC1);
                    t.store_sc1(vrs, ii, P.vstride, rbase);
                } else {
                    FW(ii) = nw;
                    t.store(V, ii, P.vstride, rbase);
                }
            };
            if (i >= 0) {
                if (hotf) {
                    // a hot feature (P.hot): the store leaves through to memory and drops the line
                    // from this XCD's L2, so the next read of it on this XCD fetches the other XCDs'
                    // updates instead of this XCD's stale copy (docs/perf_notes.md round 6)
                    const float nw = wi - eta * (d * x + 2.f * P.lambda_w * wi);
#pragma unroll
                    for (int f = 0; f < KP; ++f) {
                        const float g = d * x * (S[f] - vr.v[f] * x) + 2.f * P.lambda_v * vr.v[f];
                        vr.v[f] = f < P.k ? vr.v[f] - eta * g : 0.f;
                    }
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nw), wrs,
                                                          (uint32_t)((size_t)i * P.wstride * 4), 0, CPOL_SC1);
                    vr.store_sc1(vrs, i, P.vstride, rbase);
                } else {
                    upd(vr, i, x, wi);
                }
            }
            for (int base = 64; base < nnz; base += 64) {
                const int j = base + lane;
                if (j >= nnz) continue;
                const int i2 = idx[s + j];
                if (i2 < 0 || i2 >= P.dims) continue;
                const float x2 = val ? val[s + j] : 1.f;
                VRow<KP, BF16> t;
                t.load(V, i2, P.vstride);
                upd(t, i2, x2, FW(i2));
            }
            if (P.use_w0) {
                const float dw0 = -eta * (d + 2.f * P.lambda0 * w0v);
                if (lane == 0) {
                    atomicAdd(w0 + (int)(gw % P.w0_shards) * W0_STRIDE, dw0);
                    w0part += dw0;
                }
                acc += dw0;
            }
        }
        // rotate the pipeline
        s = ns; e = ne; ci = pi; cx = px; yy = py;
        if (w0_ref) { w0part = pw0; since = 0; acc = 0.f; } else { ++since; }
        ns = ns2; ne = ne2;
    }
}

template <int KP, bool BF16>
int launch(const FMParams& P, const int64_t* indptr, const int32_t* idx, const float* val,
           const float* y, int64_t n, int64_t t0, float* w, void* V, float* w0, float* pred,
           float* loss, int grid, int variant, int wpb, hipStream_t st) {
    // Default: 256 blocks x 4 waves.  With the global bias behind ONE atomic address every
    // grid topped out near 40 M rows/s (64 blocks was best; profiles/fm_sweep_r1.log); with 64
    // line-padded shards (profiles/fm_grid_probe_r1.log, 2M rows, 2^24 features, k=8 bf16):
    //   blocks  64: 58.7 M rows/s, held-out logloss 0.4749   128: 95.6 M, 0.4742
    //          256: 117.0 M, 0.4759                          512: 122.9 M, 0.4787
    // (single address, 64 blocks: 38.7 M, 0.4730).  256 keeps the logloss within 0.003 of the
    // single-address run at 3x the rows/s; more Hogwild concurrency costs more logloss than it
    // buys.  Round 5: against Hivemall's 8-mapper average on two boxes (3 + 5 reps,
    // profiles/r5/fm_grid_parity_yy.jsonl, fm_grid_parity_ab.jsonl; rates fm_grid_rate_yy.log):
    // 256 +2.9e-3 .. +4.1e-3 (218-234 M rows/s on config 2), 192 +2.4e-3 .. +3.6e-3 (199 M),
    // 160 +2.2e-3 .. +2.9e-3 (180 M), 128 +1.9e-3 .. +2.6e-3 (164 M).  128 (512 rows in flight)
    // is the largest grid that stays inside SURVEY's bf16 3e-3 tolerance on every box measured.
    // Round 6: the waves confined to 6 of the 8 XCDs (P.xcds, the auto default) take 256 inside it:
    // +2.06e-3 / +2.13e-3 at 188 M rows/s on config 2 (7 XCDs +2.65e-3 / +3.09e-3 at 191 M; 6 XCDs
    // at 320: +2.35e-3 / +3.26e-3, 195 M; 8 XCDs at 128: 161 M; profiles/r6/fm_xcd/).
    int64_t blocks = grid > 0 ? grid : (P.xcds < 8 ? 256 : 128);
    if (blocks > (n + 3) / 4) blocks = (n + 3) / 4;
    if (blocks > 256 * 8 * 4) blocks = 256 * 8 * 4;
    if (blocks < 1) blocks = 1;
    // `grid` counts 4-wave workgroups (the Hogwild rows in flight / 4); the waves are launched
    // wpb to a workgroup (1, 2 or 4), so the same rows in flight spread over more CUs
    int64_t lb = blocks * 4 / wpb;
    if (P.xcds < 8 && variant != 1) lb = (lb + P.xcds - 1) / P.xcds * 8;   // see fm_pipe_kernel
    if (variant == 1)
        hipLaunchKernelGGL((fm_kernel<KP, BF16>), dim3((int)lb), dim3(64 * wpb), 0, st, P, indptr, idx,
                           val, y, n, t0, w, V, w0, pred, loss);
    else if (variant == 2 || variant == 3) {
        // buffer offsets are 32-bit: the V table and the w array must stay below 4 GiB
        if ((size_t)P.dims * (size_t)P.vstride * (BF16 ? 2 : 4) >= ((size_t)1 << 32) ||
            (size_t)P.dims * (size_t)P.wstride * 4 >= ((size_t)1 << 32))
            return (int)hipErrorInvalidValue;
        if (variant == 2)
            hipLaunchKernelGGL((fm_pipe_kernel<KP, BF16, 1>), dim3((int)lb), dim3(64 * wpb), 0, st, P, indptr, idx,
                               val, y, n, t0, w, V, w0, pred, loss);
        else
            hipLaunchKernelGGL((fm_pipe_kernel<KP, BF16, 2>), dim3((int)lb), dim3(64 * wpb), 0, st, P, indptr, idx,
                               val, y, n, t0, w, V, w0, pred, loss);
    } else
        hipLaunchKernelGGL((fm_pipe_kernel<KP, BF16>), dim3((int)lb), dim3(64 * wpb), 0, st, P, indptr, idx,
                           val, y, n, t0, w, V, w0, pred, loss);
    HM_LAUNCH_RET();
}

}  // namespace

// ip: dims, k, KP, classification, train, eta_kind, use_w0, bf16, grid, seed, w0_shards, variant,
//     w0_every, vstride, wstride, wpb (waves per launched workgroup: 1, 2 or 4 = default)
//     (variant 0 = fm_pipe_kernel, 1 = fm_kernel; vstride = V elements per feature row (0: KP),
//     wstride = floats between consecutive w (0: 1); models/fm.py keeps w in the padding of each
//     feature's V row on the GPU)
// hp: eta0, power_t, total_steps, lambda0, lambda_w, lambda_v, min_target, max_target, w0_tol
HM_API int hm_fm_step(const int32_t* ip, const float* hp, int64_t n_rows, int64_t t0,
                      const int64_t* indptr, const int32_t* idx, const float* val, const float* y,
                      float* w, void* V, float* w0, float* pred, float* loss, const uint8_t* hot,
                      hipStream_t stream) {
    FMParams P;
    P.hot = hot;
    P.hot_mask = (uint32_t)ip[16];
    P.xcds = ip[17] >= 1 && ip[17] <= 8 ? ip[17] : 8;
    P.dims = ip[0]; P.k = ip[1];
    const int KP = ip[2];
    P.classification = ip[3]; P.train = ip[4]; P.eta_kind = ip[5]; P.use_w0 = ip[6];
    const int bf16 = ip[7], grid = ip[8];
    P.seed = (uint32_t)ip[9];
    P.w0_shards = ip[10];
    const int variant = ip[11];
    P.w0_every = ip[12] > 0 ? ip[12] : 1;
    if (P.w0_shards < 1 || P.w0_shards > 64) return (int)hipErrorInvalidValue;
    P.eta0 = hp[0]; P.power_t = hp[1]; P.total_steps = hp[2]; P.lambda0 = hp[3];
    P.lambda_w = hp[4]; P.lambda_v = hp[5]; P.min_target = hp[6]; P.max_target = hp[7];
    P.w0_tol = hp[8];
    const int wpb = ip[15] == 1 || ip[15] == 2 ? ip[15] : 4;
    P.vstride = ip[13] > 0 ? ip[13] : KP;
    P.wstride = ip[14] > 0 ? ip[14] : 1;
    // the hot stores use 32-bit buffer offsets: tables of 4 GiB and more keep plain stores
    if ((size_t)P.dims * (size_t)P.vstride * (bf16 ? 2 : 4) >= ((size_t)1 << 32) ||
        (size_t)P.dims * (size_t)P.wstride * 4 >= ((size_t)1 << 32))
        P.hot = nullptr;
    {
        // rows are read / written as 16-B (8-B for KP == 4 bf16) vectors
        const size_t es = bf16 ? 2 : 4, vec = (bf16 && KP == 4) ? 8 : 16;
        if (P.vstride < KP || ((size_t)P.vstride * es) % vec || reinterpret_cast<uintptr_t>(V) % vec)
            return (int)hipErrorInvalidValue;
    }
    if (n_rows <= 0) return 0;
#define HM_FM_CASE(K)                                                                            \
    case K:                                                                                      \
        return bf16 ? launch<K, true>(P, indptr, idx, val, y, n_rows, t0, w, V, w0, pred, loss, grid, variant, wpb, stream) \
                    : launch<K, false>(P, indptr, idx, val, y, n_rows, t0, w, V, w0, pred, loss, grid, variant, wpb, stream);
    switch (KP) {
        HM_FM_CASE(4)
        HM_FM_CASE(8)
        HM_FM_CASE(16)
        HM_FM_CASE(32)
        default: return (int)hipErrorInvalidValue;
    }
#undef HM_FM_CASE
}
