// Field-aware factorization machine (FFM) fused train / predict kernel for gfx950.
//
// Semantics follow Hivemall's FieldAwareFactorizationMachineUDTF (train_ffm) as pinned in
// docs/compat.md (reference @ apache/incubator-hivemall
// core/src/main/java/hivemall/fm/FieldAwareFactorizationMachineUDTF.java):
//
//   p = w0 + sum_a w[i_a] x_a + sum_{a<b} <V[i_a, f_b], V[i_b, f_a]> x_a x_b
//   classification: kappa = dloss/dp = -y / (1 + exp(y p)),  y in {-1, +1}
//   regression:     kappa = p - y
//   V   <- AdaGrad:  g = kappa x_a x_b V[i_b,f_a] + lambda_v V[i_a,f_b];  G += g^2;
//                    V -= eta0 * g / sqrt(G + eps)
//   w,w0 <- FTRL-proximal (alpha, beta, lambda1, lambda2) on g = kappa x
//
// Layout (MI355X-first):
//   * A "slot" is the (feature, field) pair; it owns the latent vector V[i, f] (Kp elements,
//     Kp = K rounded up to 4, padding stays 0) and its AdaGrad accumulator G[i, f].
//     Two layouts, selected per call by the strides of the V / G tensors:
//       - packed (default on the GPU): VG[feature][field] = {V[0..Kp) | G[0..Kp)}, slot stride
//         2*Kp.  One 16-B access (bf16, K=4) moves a slot's V and G together and a feature's
//         39-field block is 624 contiguous bytes.  gfx950 serves 8-B lanes at 0.54-0.70x the
//         16-B rate (MI355X_MICROARCH.md, global_load flavours) and the split layout needs four
//         8-B accesses per slot (V read, G read, V write, G write) against two 16-B ones here.
//       - split: V and G are separate [feature][field][Kp] tables, slot stride Kp.
//   * State is stored fp32, or bf16 (``-bf16_state``) with stochastic rounding on every write:
//     the kernel is bound by HBM / memory instructions, so halving the state bytes is the
//     throughput lever; stochastic rounding keeps the sub-ulp AdaGrad steps and G increments
//     unbiased.
//   * batch  : padded-ELL [B][F] (idx, fld, val), idx < 0 marks padding.
//   * One 256-thread block per row (grid-stride over rows).  Ordered slot s = a*F + b owns
//     the vector V[i_a, f_b]; consecutive threads read consecutive slot vectors of the same
//     feature block, so every gather is coalesced.  The row's F*F slot vectors are staged in
//     LDS in the storage format (12 KB at F=39, K=4, bf16 -> 8 blocks/CU) so the partner read
//     for the pair dot and for the gradient never goes back to L2.
//   * Updates are Hogwild across rows (no atomics); each slot vector has a single writer
//     within a row.  ``reload`` re-reads the own slot right before its update (shorter
//     read-modify-write window -> fewer lost updates on hot features).
#include <type_traits>

#include "common.h"

namespace {

struct FFMParams {
    int B, F;              // rows, slots per row (ELL width)
    int num_features, num_fields, Kp;
    int classification;    // 1: logistic loss on y in {-1,+1}; 0: squared loss
    int train;             // 0: predict only
    int use_linear, use_bias, norm;
    int reload;
    int gstride;           // per-slot G: floats between consecutive features of G
    int vpad;              // per-slot G block layout: V slots per feature block (0: separate tables)
    int tail16;            // per-slot G block layout: zero 16-B chunks after each G region
    int gfstride;          // per-slot G: floats between consecutive fields (1, or 3 in 12-B slots)
    int sstride;           // elements between consecutive slots: Kp (split) or 2*Kp (packed)
    int fstride;           // slots between consecutive features (>= num_fields; the packed GPU
                           // table pads each feature block to whole 128-B lines)
    long long vfe;         // generic kernel: V elements between consecutive features (fstride *
                           // sstride, or the 12-B slot blocks' bytes / 2)
    uint32_t seed;
    float eta0, eps, lambda_v;
    float alpha, beta, lambda1, lambda2;
    float min_target, max_target;  // regression clipping of the prediction
    const uint8_t* hot;            // per-feature flags (ffm_pipe_sg32_kernel ATOM = 2), or null
    // Multi-hot rows (two features of one field, or one feature twice: two slots of the row are
    // the same (feature, field) address).  A row updates each address once with its summed
    // gradient (docs/compat.md).  The pipelined kernels detect such rows in their forward pass
    // and, instead of updating, append them to defer = {count, rows...}; ffm_row_kernel then
    // trains them in list mode (it implements the grouped update).  null: no deferral.
    int32_t* defer;
    int list_mode;
    int lin_defer;                 // sg32: the W_LIN wave waits for the linear DMA at its first use
    // Linear FTRL state addressing: w / wz / wn of feature i at [i * lstride].  lpack: wz = w + 1,
    // wn = w + 2, 16-B aligned records (the GPU block layouts keep {w, z, n} in the 16-B chunk
    // after each feature's G region, a line the row reads and writes anyway): one 16-B DMA and
    // one 16-B store per feature instead of three scattered 4-B ones into three more lines.
    long long lstride;
    int lpack;
    // lin_atomic (lpack records, ATOM = 0 pipelined kernels, grid > 1): each row ADDS its FTRL
    // steps dz, g^2 to the record's (z, n) with float atomics instead of storing {w, z, n}, and w is
    // derived as f(z, n) where it is read (ffm_lin_derive_kernel refreshes the stored w after the
    // launch).  Round 6: a host model of W rows in flight (benchmarks/ffm_hogwild_sim.py) put 79 %
    // of the same-stream gap on lost linear updates (+3.86e-3 -> +0.81e-3 at W = 1024 with only
    // the linear (z, n) added, nothing else changed; the V / G slots' lost updates the rest).
    int lin_atomic;
    const int32_t* hidx;           // lin_atomic 4: hot index of each feature (-1: cold), [num_features]
    const int32_t* hot_id;         // lin_atomic 4: feature of each hot index, [nhot]
    float* hacc;                   // lin_atomic 4: {z, n, 0, 0} per hot index, [nhot][HACC_STRIDE]
    int nhot;                      // <= HD_SIZE
    int hacc_on;                   // set by the dispatch for a launch that uses the side table
    // Global-bias FTRL state sharded over bias_s 128-B lines during a training launch (sg32 /
    // sg12): z0 = sum of bias_sh[32 s], n0 = sum of bias_sh[32 s + 1]; a row adds its step to
    // shard (block % bias_s).  Null: the single {w0, z0, n0} address (every row's two atomics
    // and a same-address reload serialised the whole chip: 5.5 M rows/s with -w0).
    float* bias_sh;
    int bias_s;
    int bias_every;                // rows between a block's re-reads of the bias shards
};

// the linear state of feature i (FFMParams.lstride)
#define LW(p, i) ((p)[(size_t)(i) * (size_t)P.lstride])

__device__ __forceinline__ float ftrl_weight(float z, float n, float alpha, float beta,
                                             float l1, float l2) {
    if (fabsf(z) <= l1) return 0.f;
    const float s = z > 0.f ? 1.f : -1.f;
    return -(z - s * l1) / ((beta + sqrtf(n)) / alpha + l2);
}

// FTRL-proximal update of one coordinate; returns the new weight.
__device__ __forceinline__ float ftrl_update(float* __restrict__ z, float* __restrict__ n,
                                             float w, float g, float alpha, float beta,
                                             float l1, float l2) {
    const float n0 = *n;
    const float n1 = n0 + g * g;
    const float sigma = (sqrtf(n1) - sqrtf(n0)) / alpha;
    const float z1 = *z + g - sigma * w;
    *z = z1;
    *n = n1;
    return ftrl_weight(z1, n1, alpha, beta, l1, l2);
}

// Global bias w0 (-w0): bias = {w0, z0, n0, _}.  Every block updates it, so its FTRL state
// (z0, n0) is accumulated with atomics and w0 is derived from (z0, n0) where it is read;
// bias[0] is only a cached copy for the host.  Sequentially this is exactly ftrl_update.
__device__ __forceinline__ float bias_w0(const FFMParams& P, const float* bias) {
    const float z = __hip_atomic_load(bias + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float n = __hip_atomic_load(bias + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return ftrl_weight(z, n, P.alpha, P.beta, 0.f, 0.f);
}

__device__ __forceinline__ void bias_update(const FFMParams& P, float g, float* bias) {
    const float z0 = __hip_atomic_load(bias + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float n0 = __hip_atomic_load(bias + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float w = ftrl_weight(z0, n0, P.alpha, P.beta, 0.f, 0.f);
    const float sigma = (sqrtf(n0 + g * g) - sqrtf(n0)) / P.alpha;
    const float dz = g - sigma * w;
    atomicAdd(bias + 1, dz);
    atomicAdd(bias + 2, g * g);
    bias[0] = ftrl_weight(z0 + dz, n0 + g * g, P.alpha, P.beta, 0.f, 0.f);
}

// bias_update on the sharded state: (z0, n0) is the row's snapshot of the shard sums
// (adds the step to acc[0..1]: the block's own steps its copy of the shard sums lacks)
__device__ __forceinline__ void bias_update_sh(const FFMParams& P, float g, float z0, float n0, float* sh,
                                               float* acc) {
    const float w = ftrl_weight(z0, n0, P.alpha, P.beta, 0.f, 0.f);
    const float sigma = (sqrtf(n0 + g * g) - sqrtf(n0)) / P.alpha;
    const float dz = g - sigma * w;
    atomicAdd(sh, dz);
    atomicAdd(sh + 1, g * g);
    acc[0] += dz;
    acc[1] += g * g;
}

// lin_atomic: the weight of a DMA'd {w, z, n, _} record is f(z, n) (its stored w lags: rows add
// to (z, n) only); a record never stepped (n = 0) keeps its stored w
__device__ __forceinline__ float lin_w(const FFMParams& P, float4 r) {
    return r.z > 0.f ? ftrl_weight(r.y, r.z, P.alpha, P.beta, P.lambda1, P.lambda2) : r.x;
}

// lin_atomic: the row's FTRL step of feature i as two no-return float atomics on its record's
// (z, n): dz = g - sigma w (the host engine's association: z + (g - sigma w)), dn = g^2
__device__ __forceinline__ void lin_add(const FFMParams& P, float* w, int i, float g, float n0,
                                        float n1, float wcur) {
    atomicAdd(&LW(w, i) + 1, g - (sqrtf(n1) - sqrtf(n0)) / P.alpha * wcur);
    atomicAdd(&LW(w, i) + 2, g * g);
}

// lin_atomic 4 (template LT of the pipelined kernels): the linear FTRL state (z, n) of the
// P.nhot hot features lives in a dense side table P.hacc[h] = {z, n, 0, 0} (h = P.hidx[feature],
// -1: cold) for the duration of a launch (ffm_hacc_kernel copies it out of / back into the
// records around the launch).  A block sums its rows' steps of hot features in LDS, s_hd[h], and
// adds them to P.hacc by float atomics when it ends; a row reads hacc[h] (DMA'd one row ahead,
// like the record) plus the block's own sums.  Nothing is lost to a concurrent row, and the
// atomics land in the side table, not in the hot features' blocks: atomics on the records
// themselves drop those lines from L2, which every row reads (per-row atomics on the records: 8.7 M
// rows/s, block sums flushed onto the records: 28 M, vs 93 M with plain stores;
// profiles/r6/linhot/).  Cold features keep the plain record stores.
constexpr int HD_SIZE = 2048;
constexpr int HD12_SIZE = 1024;   // ffm_pipe_sg12_kernel (bf16 12-B slots)
// one side-table entry per 128-B line (16-B entries, 8 to a line: 73.6 vs 76.0 M rows/s)
constexpr int HACC_STRIDE = 32;
// default grid of a side-table launch: a block's sums are flushed when it ends, so fewer, longer-
// lived blocks add fewer atomics per row (distinct hot features per block grow slower than its
// rows).  Measured (profiles/r6/linhot/): 8,192 blocks 76.0 M rows/s, 4,096 82.4 M (+0.90e-3),
// 2,048 84.2-84.8 M at +0.96e-3 .. +1.01e-3; 1,024 (256 rows per block) diverges (+0.06 .. +0.11): every block walks
// its own copy of a hot feature's weight toward the target for 256 rows and the sum of those walks
// overshoots.
constexpr int HACC_GRID = 2048;
// The bf16 kernel holds 3 blocks per CU (768 resident), so 2,048 blocks leave its last round 2/3
// full: 2,304 (3 full rounds) 128.1-128.9 M bf16 rows/s at +1.58e-3 .. +1.67e-3 vs 125.8-125.9 M at
// 2,048; 3,072 126.5-126.9 M; 1,536 (171 rows per block) 131.2-131.7 M but diverging (+8e-3 ..
// +1.0e-2).  The fp32 kernel's 2 blocks per CU make 2,048 four full rounds (2,304: 81.5-81.8 M vs
// 84.8-85.0 M).  profiles/r6/hacc_grid/.  More fp32 blocks do not buy a safer gap either:
// 2,048 84.4-84.8 M at +0.95e-3 / +0.97e-3, 3,072 83.0-83.6 M at +0.90e-3 / +0.97e-3, 4,096
// 81.5-82.2 M at +0.90e-3 / +0.96e-3 (one box, interleaved; profiles/r6/hacc_grid/fp32/).
constexpr int HACC_GRID12 = 2304;

__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ c * 0xC2B2AE3Du;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    return h;
}

// 4-element chunk of a slot vector, at element offset `off` (a multiple of 4).
template <bool BF>
__device__ __forceinline__ float4 ld_chunk(const void* base, size_t off) {
    if constexpr (BF) {
        const uint2 q = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(base) + off);
        return make_float4(__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xFFFF0000u),
                           __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xFFFF0000u));
    } else {
        return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(base) + off);
    }
}

// Raw storage-format chunk (no conversion) and its fp32 view.
template <bool BF>
__device__ __forceinline__ typename std::conditional<BF, uint2, float4>::type ld_raw(const void* base, size_t off) {
    if constexpr (BF) return *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(base) + off);
    else return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(base) + off);
}

template <bool BF, typename T>
__device__ __forceinline__ float4 to_f4(const T& q) {
    if constexpr (BF) {
        return make_float4(__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xFFFF0000u),
                           __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xFFFF0000u));
    } else {
        return q;
    }
}

template <bool BF>
__device__ __forceinline__ void st_chunk(void* base, size_t off, float4 v, uint32_t rnd) {
    if constexpr (BF) {
        const uint32_t r2 = rnd * 0x9E3779B1u + 0x632BE5ABu;
        const uint32_t lo = hm::pack_bf16x2_sr(v.x, rnd, v.y, rnd >> 16);
        const uint32_t hi = hm::pack_bf16x2_sr(v.z, r2, v.w, r2 >> 16);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(base) + off) = make_uint2(lo, hi);
    } else {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(base) + off) = v;
    }
}

// Row metadata of one slot (thread tid < F) from the padded-ELL batch.
struct SlotMeta {
    int i, f;
    float x;
};

__device__ __forceinline__ SlotMeta fetch_row_meta(const FFMParams& P, int row,
                                                   const int32_t* __restrict__ idx,
                                                   const int32_t* __restrict__ fld,
                                                   const float* __restrict__ val) {
    SlotMeta m{-1, 0, 0.f};
    const int tid = threadIdx.x;
    if (tid < P.F && row < P.B) {
        const size_t o = (size_t)row * P.F + tid;
        m.i = idx[o];
        m.f = fld ? fld[o] : tid;
        m.x = val ? val[o] : 1.f;
    }
    return m;
}

// Metadata -> LDS and the instance-wise L2 normalisation factor (contains the block barrier
// that publishes s_idx / s_fld / s_x).
__device__ __forceinline__ float publish_row_meta(const FFMParams& P, SlotMeta m, int* s_idx,
                                                  int* s_fld, float* s_x, float* s_red) {
    const int tid = threadIdx.x;
    float sq = 0.f;
    if (tid < P.F) {
        int i = m.i, f = m.f;
        float x = m.x;
        if (i < 0 || i >= P.num_features || f < 0 || f >= P.num_fields) { i = -1; x = 0.f; }
        s_idx[tid] = i;
        s_fld[tid] = f < 0 ? 0 : (f >= P.num_fields ? P.num_fields - 1 : f);
        s_x[tid] = x;
        sq = x * x;
    }
    if (P.norm) {
        const float tot = hm::block_sum(sq, s_red);
        return tot > 0.f ? rsqrtf(tot) : 1.f;
    }
    __syncthreads();
    return 1.f;
}

__device__ __forceinline__ float load_row_meta(const FFMParams& P, int row,
                                               const int32_t* __restrict__ idx,
                                               const int32_t* __restrict__ fld,
                                               const float* __restrict__ val, int* s_idx,
                                               int* s_fld, float* s_x, float* s_red) {
    return publish_row_meta(P, fetch_row_meta(P, row, idx, fld, val), s_idx, s_fld, s_x, s_red);
}

// Loss of the row's score p; writes pred/loss (thread 0) and returns kappa = dloss/dp.
__device__ __forceinline__ float row_loss(const FFMParams& P, int row, float p,
                                          const float* __restrict__ y,
                                          float* __restrict__ pred_out,
                                          float* __restrict__ loss_out) {
    const float yy = y ? y[row] : 0.f;
    float kappa;
    if (P.classification) {
        const float e = yy * p;
        kappa = -yy / (1.f + __expf(e));
        if (threadIdx.x == 0) {
            if (loss_out) loss_out[row] = hm::log1pexp(-e);
            if (pred_out) pred_out[row] = p;
        }
    } else {
        const float pc = fminf(fmaxf(p, P.min_target), P.max_target);
        kappa = pc - yy;
        if (threadIdx.x == 0) {
            if (loss_out) loss_out[row] = 0.5f * kappa * kappa;
            if (pred_out) pred_out[row] = pc;
        }
    }
    return kappa;
}

// Multi-hot detection in the pipelined kernels: slot (a, b), a < b, of a row shares an address
// with another slot when the two positions hold the same feature or the same field.
__device__ __forceinline__ bool slot_repeats(int a, int b, int4 ma, int4 mb) {
    return a < b && (ma.x | mb.x) >= 0 && (ma.x == mb.x || ma.y == mb.y);
}

// Appends a multi-hot row to the deferred list (thread 0; the block skips the row's updates).
__device__ __forceinline__ void defer_row(const FFMParams& P, int row) {
    if (threadIdx.x == 0) {
        const int k = atomicAdd(P.defer, 1);
        P.defer[1 + k] = row;
    }
}

// ---------------------------------------------------------------------------------------------
// Generic kernel: any K, either per-element layout (slot stride P.sstride) or per-slot G
// (SG: one fp32 accumulator per slot at G[i * P.gstride + f]), LDS staging when it fits.
template <int KC, bool STAGE, bool BF, bool SG>
__global__ __launch_bounds__(256) void ffm_row_kernel(
    FFMParams P, const int32_t* __restrict__ idx, const int32_t* __restrict__ fld,
    const float* __restrict__ val, const float* __restrict__ y,
    void* __restrict__ V, void* __restrict__ G,
    float* __restrict__ w, float* __restrict__ wz, float* __restrict__ wn,
    float* __restrict__ bias,        // [4] = {w0, z0, n0, _}
    float* __restrict__ pred_out,    // [B] or null: raw score p
    float* __restrict__ loss_out)    // [B] or null: per-row loss
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int F = P.F;
    const int FF = F * F;
    // The LDS image keeps the storage format (bf16 state -> 8 B per 4-vector): half the LDS per
    // block at bf16, so up to 8 blocks fit per CU.  Measured variants (profiles/ffm_kernel_ab*):
    // J-slot batched gathers and a register-only pair-ownership kernel were both slower.
    using SV = typename std::conditional<BF, uint2, float4>::type;
    SV* s_v = reinterpret_cast<SV*>(smem);                               // STAGE: FF*KC
    const size_t vbytes = STAGE ? (size_t)FF * KC * sizeof(SV) : 0;
    int* s_idx = reinterpret_cast<int*>(smem + vbytes);                  // F
    int* s_fld = s_idx + F;                                              // F
    float* s_x = reinterpret_cast<float*>(s_fld + F);                    // F
    int* s_ni = reinterpret_cast<int*>(s_x + F);                         // F: next position, same feature
    int* s_nf = s_ni + F;                                                // F: next position, same field
    int* s_first = s_nf + F;                                             // F: bit 0 first of feature, 1 of field
    float* s_red = reinterpret_cast<float*>(s_first + F);                // 16 (+pad)

    const int tid = threadIdx.x;
    const size_t ss = (size_t)P.sstride;
    auto slot_off = [&](int i, int f) -> size_t { return (size_t)i * (size_t)P.vfe + (size_t)f * ss; };
    float* Gs = reinterpret_cast<float*>(G);
    // list mode: the rows the pipelined kernel deferred (count written by the previous launch)
    const int nrows = P.list_mode ? P.defer[0] : P.B;

    for (int k = blockIdx.x; k < nrows; k += gridDim.x) {
        const int row = P.list_mode ? P.defer[1 + k] : k;
        // ---- 1. row metadata -> LDS (+ instance-wise L2 normalisation) ----
        const float scale = load_row_meta(P, row, idx, fld, val, s_idx, s_fld, s_x, s_red);
        // ---- 1b. repeated features / fields: chains to the next position of the same feature
        //      and field, owner flags; multi = the row has any (one block-wide OR) ----
        int rep = 0;
        if (tid < F) {
            const int ia = s_idx[tid], fa = s_fld[tid];
            int ni = -1, nf = -1, first = 3;
            if (ia >= 0) {
                for (int b = 0; b < F; ++b) {
                    if (b == tid || s_idx[b] < 0) continue;
                    if (s_idx[b] == ia) { if (b < tid) first &= ~1; else if (ni < 0) ni = b; rep = 1; }
                    if (s_fld[b] == fa) { if (b < tid) first &= ~2; else if (nf < 0) nf = b; rep = 1; }
                }
            }
            s_ni[tid] = ni;
            s_nf[tid] = nf;
            s_first[tid] = first;
        }
        const bool multi = __syncthreads_or(rep) != 0;

        // ---- 2. gather the row's slot vectors (coalesced; the diagonal too in multi-hot rows,
        //      where it can be the owner of an address) ----
        if (STAGE) {
            for (int s = tid; s < FF; s += blockDim.x) {
                const int a = s / F, b = s - (s / F) * F;
                const int ia = s_idx[a];
                const bool live = (a != b || multi) && ia >= 0 && s_idx[b] >= 0;
                const size_t off = live ? slot_off(ia, s_fld[b]) : 0;
#pragma unroll
                for (int c = 0; c < KC; ++c)
                    s_v[s * KC + c] = live ? ld_raw<BF>(V, off + 4 * c) : SV{};
            }
            __syncthreads();
        }

        // ---- 3. forward ----
        float part = 0.f;
        for (int s = tid; s < FF; s += blockDim.x) {
            const int a = s / F, b = s - (s / F) * F;
            if (a >= b) continue;
            const int ia = s_idx[a], ib = s_idx[b];
            if (ia < 0 || ib < 0) continue;
            float4 u[KC], v[KC];
            if (STAGE) {
#pragma unroll
                for (int c = 0; c < KC; ++c) {
                    u[c] = to_f4<BF>(s_v[s * KC + c]);
                    v[c] = to_f4<BF>(s_v[(b * F + a) * KC + c]);
                }
            } else {
                const size_t ou = slot_off(ia, s_fld[b]);
                const size_t ov = slot_off(ib, s_fld[a]);
#pragma unroll
                for (int c = 0; c < KC; ++c) { u[c] = ld_chunk<BF>(V, ou + 4 * c); v[c] = ld_chunk<BF>(V, ov + 4 * c); }
            }
            float d = 0.f;
#pragma unroll
            for (int c = 0; c < KC; ++c) d += u[c].x * v[c].x + u[c].y * v[c].y + u[c].z * v[c].z + u[c].w * v[c].w;
            part += d * s_x[a] * s_x[b];
        }
        part *= scale * scale;
        if (P.use_linear && tid < F && s_idx[tid] >= 0) part += LW(w, s_idx[tid]) * s_x[tid] * scale;
        float p = hm::block_sum(part, s_red);
        if (P.use_bias) p += bias_w0(P, bias);

        // ---- 4. loss ----
        const float kappa = row_loss(P, row, p, y, pred_out, loss_out);

        // ---- 5. updates (Hogwild across rows; each address of the row written once) ----
        if (P.train) {
            const float ks = kappa * scale * scale;
            const uint32_t rrow = P.seed ^ ((uint32_t)row * 0x85EBCA77u);
            for (int s = tid; s < FF; s += blockDim.x) {
                const int a = s / F, b = s - (s / F) * F;
                if (a == b && !multi) continue;
                const int ia = s_idx[a], ib = s_idx[b];
                if (ia < 0 || ib < 0) continue;
                // multi-hot row: the slot (first position of the feature, first of the field)
                // owns the address (i_a, f_b) and sums the partner terms of every pair mapping
                // to it; the other slots of the address do not write
                if (multi && (!(s_first[a] & 1) || !(s_first[b] & 2))) continue;
                const size_t ov = slot_off(ia, s_fld[b]);
                float4 own[KC], gg[KC], g[KC];
                if (!SG) {
#pragma unroll
                    for (int c = 0; c < KC; ++c) gg[c] = ld_chunk<BF>(G, ov + 4 * c);
                }
#pragma unroll
                for (int c = 0; c < KC; ++c) {
                    own[c] = (STAGE && !P.reload) ? to_f4<BF>(s_v[s * KC + c]) : ld_chunk<BF>(V, ov + 4 * c);
                    g[c] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
                bool any = false;
                for (int a2 = a; a2 >= 0; a2 = multi ? s_ni[a2] : -1) {
                    for (int b2 = b; b2 >= 0; b2 = multi ? s_nf[b2] : -1) {
                        if (a2 == b2) continue;
                        any = true;
                        const float coef = ks * s_x[a2] * s_x[b2];
                        const size_t op = STAGE ? 0 : slot_off(s_idx[b2], s_fld[a2]);
#pragma unroll
                        for (int c = 0; c < KC; ++c) {
                            const float4 par = STAGE ? to_f4<BF>(s_v[(b2 * F + a2) * KC + c]) : ld_chunk<BF>(V, op + 4 * c);
                            g[c].x += coef * par.x;
                            g[c].y += coef * par.y;
                            g[c].z += coef * par.z;
                            g[c].w += coef * par.w;
                        }
                    }
                }
                if (!any) continue;       // a diagonal address no pair of the row reads
#pragma unroll
                for (int c = 0; c < KC; ++c) {
                    g[c].x += P.lambda_v * own[c].x;
                    g[c].y += P.lambda_v * own[c].y;
                    g[c].z += P.lambda_v * own[c].z;
                    g[c].w += P.lambda_v * own[c].w;
                }
                if constexpr (SG) {
                    // one accumulator per slot: G += sum of the k squared gradients (factor
                    // order), then every factor steps with 1 / sqrt(G + eps)
                    float* pg = Gs + (size_t)ia * P.gstride + (size_t)s_fld[b] * P.gfstride;
                    float gs = *pg;
#pragma unroll
                    for (int c = 0; c < KC; ++c)
                        gs = (((gs + g[c].x * g[c].x) + g[c].y * g[c].y) + g[c].z * g[c].z) + g[c].w * g[c].w;
                    *pg = gs;
                    const float r = rsqrtf(gs + P.eps);
#pragma unroll
                    for (int c = 0; c < KC; ++c) {
                        own[c].x -= P.eta0 * g[c].x * r;
                        own[c].y -= P.eta0 * g[c].y * r;
                        own[c].z -= P.eta0 * g[c].z * r;
                        own[c].w -= P.eta0 * g[c].w * r;
                        const uint32_t rnd = BF ? hash3(rrow, (uint32_t)s, (uint32_t)c) : 0u;
                        st_chunk<BF>(V, ov + 4 * c, own[c], rnd);
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < KC; ++c) {
                        gg[c].x += g[c].x * g[c].x; gg[c].y += g[c].y * g[c].y;
                        gg[c].z += g[c].z * g[c].z; gg[c].w += g[c].w * g[c].w;
                        own[c].x -= P.eta0 * g[c].x * rsqrtf(gg[c].x + P.eps);
                        own[c].y -= P.eta0 * g[c].y * rsqrtf(gg[c].y + P.eps);
                        own[c].z -= P.eta0 * g[c].z * rsqrtf(gg[c].z + P.eps);
                        own[c].w -= P.eta0 * g[c].w * rsqrtf(gg[c].w + P.eps);
                        const uint32_t rnd = BF ? hash3(rrow, (uint32_t)s, (uint32_t)c) : 0u;
                        st_chunk<BF>(V, ov + 4 * c, own[c], rnd);
                        st_chunk<BF>(G, ov + 4 * c, gg[c], rnd ^ 0xA5A5A5A5u);
                    }
                }
            }
            // FTRL: one step per distinct feature of the row, with the summed gradient
            if (P.use_linear && tid < F && s_idx[tid] >= 0 && (!multi || (s_first[tid] & 1))) {
                const int i = s_idx[tid];
                float xs = s_x[tid];
                if (multi)
                    for (int a2 = s_ni[tid]; a2 >= 0; a2 = s_ni[a2]) xs += s_x[a2];
                if (P.lpack) {
                    // the {w, z, n} record: one 16-B read and one 16-B store (never a torn record)
                    float4* rp = reinterpret_cast<float4*>(&LW(w, i));
                    const float4 r = *rp;
                    float z = r.y, n = r.z;
                    const float nw = ftrl_update(&z, &n, r.x, kappa * xs * scale, P.alpha, P.beta, P.lambda1, P.lambda2);
                    *rp = make_float4(nw, z, n, r.w);
                } else {
                    LW(w, i) = ftrl_update(&LW(wz, i), &LW(wn, i), LW(w, i), kappa * xs * scale, P.alpha, P.beta,
                                           P.lambda1, P.lambda2);
                }
            }
            if (P.use_bias && tid == 0) bias_update(P, kappa, bias);
        }
        __syncthreads();  // LDS reuse by the next row
    }
}


// ---------------------------------------------------------------------------------------------
// Lean packed kernel (K <= 4, packed V|G slots): the shipped kernel for the headline shape.
//
// Counters of ffm_packed_kernel on MI355X (profiles/ffm_pmc_packed_r2b.json) show the row loop
// is bound by vector-instruction ISSUE, not by memory: 3,976 VALU wave-instructions per row
// (~166 per slot and wave), 22 % of wave-cycles issuing with 4 waves/SIMD (the SIMDs ~90 %
// busy), HBM-side traffic only 3.7 TB/s.  The VALU went to bf16 unpacking, 13 quarter-rate
// v_mul_lo_u32 per slot for the stochastic-rounding hash chain, 64-bit address math and
// register shuffles around the per-slot branches.  This kernel does the same arithmetic with:
//   * the forward pair dot as two v_dot2c_f32_bf16 on the raw bf16 words (no unpack);
//   * the update in packed fp32 (v_pk_mul/fma/add_f32: two elements per instruction);
//   * ONE 32-bit hash per slot (row seed + a per-thread constant, one multiply) whose rotated
//     16-bit windows feed all eight v_cvt_sr_bf16_f32 (each window uniform -> unbiased);
//   * a transposed LDS image: slot s = (a, b) writes its own V to T[b*F + a], so the partner
//     V[i_b, f_a] of slot s is T[s] — both partner reads (forward, update) are contiguous;
//   * 32-bit slot byte offsets (tables < 4 GiB) from one uniform base;
//   * x_a * x_b per slot cached in a register for the forward and the update.
// Arithmetic order matches the CPU engine up to fp32 contraction / dot2 association.
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 bf2_to_f2(uint32_t u) {
    return f2{__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u)};
}

__device__ __forceinline__ float dot2_bf16(uint32_t a, uint32_t b, float c) {
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
    bf16x2_t va, vb;
    __builtin_memcpy(&va, &a, 4);
    __builtin_memcpy(&vb, &b, 4);
    return __builtin_amdgcn_fdot2_f32_bf16(va, vb, c, false);
}

// Two floats -> bf16x2 with stochastic rounding; ra / rb are used as is (the instruction adds
// the HIGH 16 bits of its random operand, see hm::pack_bf16x2_sr).
__device__ __forceinline__ uint32_t pack_sr_hi(f2 v, uint32_t ra, uint32_t rb) {
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
    bf16x2_t o = __builtin_bit_cast(bf16x2_t, ra);   // both halves are overwritten
    o = __builtin_amdgcn_cvt_sr_bf16_f32(o, v.x, ra, false);
    o = __builtin_amdgcn_cvt_sr_bf16_f32(o, v.y, rb, true);
    uint32_t u;
    __builtin_memcpy(&u, &o, 4);
    return u;
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return __builtin_amdgcn_alignbit(x, x, 32 - r); }

template <bool BF>
struct LeanIO {
    // raw slot: bf16 -> uint4 {v01, v23, g01, g23}; fp32 -> V float4 + G float4
    using Raw = typename std::conditional<BF, uint4, float4[2]>::type;
    using Img = typename std::conditional<BF, uint2, float4>::type;   // V in the LDS image
};

template <bool BF, int NS>
__global__ __launch_bounds__(256) void ffm_lean_kernel(
    FFMParams P, const int32_t* __restrict__ idx, const int32_t* __restrict__ fld,
    const float* __restrict__ val, const float* __restrict__ y, void* __restrict__ VG,
    float* __restrict__ w, float* __restrict__ wz, float* __restrict__ wn,
    float* __restrict__ bias, float* __restrict__ pred_out, float* __restrict__ loss_out)
{
    using Img = typename LeanIO<BF>::Img;
    constexpr uint32_t SLOT_B = BF ? 16u : 32u;          // bytes per packed slot
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int F = P.F;
    const int FF = F * F;
    Img* s_t = reinterpret_cast<Img*>(smem);                                     // FF (transposed)
    int4* s_m = reinterpret_cast<int4*>(smem + (size_t)FF * sizeof(Img));      // F x {i, f, x, -}
    float* s_red = reinterpret_cast<float*>(s_m + F);                           // 16
    const int tid = threadIdx.x;
    const uint32_t nfld = (uint32_t)P.fstride;
    char* vg = reinterpret_cast<char*>(VG);

    // row-invariant slot decode; slots past F*F become (0, 0): a diagonal slot, i.e. dead
    int sa[NS], sb[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        const int s = tid + j * 256;
        sa[j] = s < FF ? s / F : 0;
        sb[j] = s < FF ? s % F : 0;
    }
    const uint32_t tid_h = (uint32_t)tid * 0x9E3779B1u;

    for (int row = blockIdx.x; row < P.B; row += gridDim.x) {
        // ---- row metadata -> LDS {i, f, x}; instance-wise L2 norm (the block sum's barrier
        //      publishes s_m).  Padding / out-of-range entries get i = -1, x = 0. ----
        float sq = 0.f;
        int mi = -1;
        float mx = 0.f;
        if (tid < F) {
            const size_t o = (size_t)row * F + tid;
            int i = idx[o];
            int f = fld ? fld[o] : tid;
            float x = val ? val[o] : 1.f;
            if (i < 0 || i >= P.num_features || f < 0 || f >= P.num_fields) { i = -1; x = 0.f; f = 0; }
            s_m[tid] = make_int4(i, f, __float_as_int(x), 0);
            mi = i;
            mx = x;
            sq = x * x;
        }
        float scale = 1.f;
        if (P.norm) {
            const float tot = hm::block_sum(sq, s_red);
            scale = tot > 0.f ? rsqrtf(tot) : 1.f;
        } else {
            __syncthreads();
        }
        float lw = 0.f;
        if (P.use_linear && mi >= 0) lw = LW(w, mi);

        // ---- gather (branch-free): own raw slot -> registers, own V -> transposed LDS image.
        //      Dead slots (a == b, padding) load slot 0 and get x_a x_b = 0. ----
        uint4 q[NS];
        float4 qv[NS], qg[NS];
        uint32_t off[NS];
        float xab[NS];
        bool live[NS];
        int rep = 0;
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const int4 ma = s_m[sa[j]], mb = s_m[sb[j]];
            if (P.defer) rep |= (int)slot_repeats(sa[j], sb[j], ma, mb);
            live[j] = sa[j] != sb[j] && ma.x >= 0 && mb.x >= 0;
            off[j] = live[j] ? ((uint32_t)ma.x * nfld + (uint32_t)mb.y) * SLOT_B : 0u;
            xab[j] = live[j] ? __int_as_float(ma.z) * __int_as_float(mb.z) : 0.f;
            if constexpr (BF) {
                q[j] = *reinterpret_cast<const uint4*>(vg + off[j]);
                s_t[sb[j] * F + sa[j]] = make_uint2(q[j].x, q[j].y);
            } else {
                qv[j] = *reinterpret_cast<const float4*>(vg + off[j]);
                qg[j] = *reinterpret_cast<const float4*>(vg + off[j] + 16u);
                s_t[sb[j] * F + sa[j]] = qv[j];
            }
        }
        const bool rdup = __syncthreads_or(rep) != 0;

        // ---- forward: every slot (a, b) adds its pair dot weighted by x_a x_b (0 if dead); the
        //      sum over ordered pairs counts each unordered pair twice -> halved ----
        float part = 0.f;
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const int s = tid + j * 256;
            float d;
            if constexpr (BF) {
                const uint2 pv = s_t[s < FF ? s : 0];
                d = dot2_bf16(q[j].x, pv.x, dot2_bf16(q[j].y, pv.y, 0.f));
            } else {
                const float4 pv = s_t[s < FF ? s : 0];
                d = qv[j].x * pv.x + qv[j].y * pv.y + qv[j].z * pv.z + qv[j].w * pv.w;
            }
            part += d * xab[j];
        }
        part *= 0.5f * scale * scale;
        part += lw * mx * scale;                       // mx = 0 for tid >= F / padding
        float p = hm::block_sum(part, s_red);
        if (P.use_bias) p += bias_w0(P, bias);
        const float kappa = row_loss(P, row, p, y, pred_out, loss_out);

        // ---- AdaGrad(V) update (Hogwild), packed fp32 math; only the store is predicated ----
        if (P.train && rdup && P.defer) {
            defer_row(P, row);                  // multi-hot row: ffm_row_kernel trains it
        } else if (P.train) {
            float lz = 0.f, ln = 0.f;
            if (P.use_linear && mi >= 0) { lz = LW(wz, mi); ln = LW(wn, mi); }
            const float ks = kappa * scale * scale;
            const f2 lam = {P.lambda_v, P.lambda_v}, eps = {P.eps, P.eps};
            const f2 meta = {-P.eta0, -P.eta0};
            const uint32_t hrow = P.seed ^ ((uint32_t)row * 0x85EBCA77u);
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                const int s = tid + j * 256;
                const f2 coef = {ks * xab[j], ks * xab[j]};
                f2 o0, o1, g0, g1, p0, p1;
                if constexpr (BF) {
                    const uint2 pv = s_t[s < FF ? s : 0];
                    o0 = bf2_to_f2(q[j].x); o1 = bf2_to_f2(q[j].y);
                    g0 = bf2_to_f2(q[j].z); g1 = bf2_to_f2(q[j].w);
                    p0 = bf2_to_f2(pv.x);   p1 = bf2_to_f2(pv.y);
                } else {
                    const float4 pv = s_t[s < FF ? s : 0];
                    o0 = f2{qv[j].x, qv[j].y}; o1 = f2{qv[j].z, qv[j].w};
                    g0 = f2{qg[j].x, qg[j].y}; g1 = f2{qg[j].z, qg[j].w};
                    p0 = f2{pv.x, pv.y};       p1 = f2{pv.z, pv.w};
                }
                const f2 d0 = coef * p0 + lam * o0, d1 = coef * p1 + lam * o1;
                g0 = g0 + d0 * d0;
                g1 = g1 + d1 * d1;
                const f2 t0 = g0 + eps, t1 = g1 + eps;
                const f2 r0 = {__builtin_amdgcn_rsqf(t0.x), __builtin_amdgcn_rsqf(t0.y)};
                const f2 r1 = {__builtin_amdgcn_rsqf(t1.x), __builtin_amdgcn_rsqf(t1.y)};
                o0 = o0 + meta * d0 * r0;
                o1 = o1 + meta * d1 * r1;
                if constexpr (BF) {
                    // one hash per slot, full-rate 24-bit multiply; 8 rotated 16-bit windows
                    uint32_t h = hrow + tid_h + (uint32_t)j * 0x6A09E667u;
                    h ^= h >> 16;
                    h = __umul24(h, 0x2C1B3Du) ^ (h >> 11);
                    h ^= h >> 15;
                    const uint4 st = make_uint4(pack_sr_hi(o0, h, rotl32(h, 16)),
                                                pack_sr_hi(o1, rotl32(h, 8), rotl32(h, 24)),
                                                pack_sr_hi(g0, rotl32(h, 4), rotl32(h, 20)),
                                                pack_sr_hi(g1, rotl32(h, 12), rotl32(h, 28)));
                    if (live[j]) *reinterpret_cast<uint4*>(vg + off[j]) = st;
                } else {
                    if (live[j]) {
                        *reinterpret_cast<float4*>(vg + off[j]) = make_float4(o0.x, o0.y, o1.x, o1.y);
                        *reinterpret_cast<float4*>(vg + off[j] + 16u) = make_float4(g0.x, g0.y, g1.x, g1.y);
                    }
                }
            }
            if (P.use_linear && mi >= 0) {
                const float g = kappa * mx * scale;
                const float n1 = ln + g * g;
                const float z1 = lz + g - (sqrtf(n1) - sqrtf(ln)) / P.alpha * lw;
                LW(wz, mi) = z1;
                LW(wn, mi) = n1;
                LW(w, mi) = ftrl_weight(z1, n1, P.alpha, P.beta, P.lambda1, P.lambda2);
            }
            if (P.use_bias && tid == 0) bias_update(P, kappa, bias);
        }
        __syncthreads();
    }
}


// ---------------------------------------------------------------------------------------------
// Pipelined kernel (packed per-element V|G, K <= 4; bf16 or fp32 state): the next row's 1,482
// slot gathers fly into LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR destination) while the
// current row computes.
//
// The lean kernel above still waits on two dependent global round trips per row (row metadata,
// then the slot gather) with nothing else to do: per CU only ~4 rows' gathers are ever in flight,
// and only during their gather phase (HBM-side 3.7-3.9 TB/s).  Here a block's loop iteration
// for row r is
//   A  wait for DMA(r) (own wave: vmcnt(0)), barrier
//   B  own raw slots LDS -> registers, own V -> transposed image T; publish meta(r+G) (loaded
//      into registers one iteration earlier) and its L2-norm scale; barrier
//   C  issue DMA(r+G) from meta(r+G) (offsets, x_a x_b, linear-term ids kept in registers);
//      issue the loads of meta(r+2G)
//   D  forward(r), block sum (raw s_barrier: a __syncthreads() fence would drain the DMA)
//   E  AdaGrad / FTRL updates of r (stores)
//   F  load w, z, n of r+G's linear terms (after E's stores: same-thread order keeps the FTRL
//      read-modify-write of a feature shared by consecutive rows exact)
// so each block keeps one row's 24 KB gather in flight behind its compute (4 blocks/CU: ~96 KB
// in flight per CU).  Staleness: row r+G's slots are read before row r's updates land — the
// same one-row Hogwild window the other ~1,000 rows in flight already impose.
// Polling the DMA targets instead of vmcnt(0) (so no wave waits on the previous row's stores),
// with an LDS hand-over of slots shared by consecutive rows, was measured no faster (101.1-101.6 M
// rows/s default vs 98.8-100.8 M polled, profiles/ffm_poll_r2/bench_ab_corrected.log) and removed.
// BF = false: the same pipeline over fp32 packed slots (32 B: V float4 | G float4; two 16-B DMAs
// per slot; LDS 77.6 KB at NS = 6 -> 2 blocks/CU; opt-in HM_FFM_VARIANT=3).
__device__ __forceinline__ void bar_raw() {
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's LDS writes are done
    __builtin_amdgcn_s_barrier();
    __asm__ __volatile__("" ::: "memory");
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* glb_ptr_t;


template <int NS, bool BF = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BF ? 4 : 2))) void ffm_pipe_kernel(
    FFMParams P, const int32_t* __restrict__ idx, const int32_t* __restrict__ fld,
    const float* __restrict__ val, const float* __restrict__ y, void* __restrict__ VG,
    float* __restrict__ w, float* __restrict__ wz, float* __restrict__ wn,
    float* __restrict__ bias, float* __restrict__ pred_out, float* __restrict__ loss_out)
{
    constexpr uint32_t SLOT_B = BF ? 16u : 32u;                        // bytes per packed slot
    using Img = typename std::conditional<BF, uint2, float4>::type;   // V in the transposed image
    __shared__ __attribute__((aligned(16))) uint4 s_raw[NS * 256 * (BF ? 1 : 2)];   // slot DMA landing zone
    __shared__ __attribute__((aligned(16))) Img s_t[NS * 256];        // transposed V image
    // F <= 45 (F*F <= 2048): per-field arrays of 48; total LDS 40,736 B at NS = 6 -> 4 blocks/CU
    __shared__ __attribute__((aligned(16))) int4 s_m[2][48];          // validated meta {i, f, x}
    __shared__ __attribute__((aligned(16))) int s_mr[2][3][48];       // raw meta DMA {idx, fld, val}
    __shared__ __attribute__((aligned(16))) float s_lin[2][3][48];    // DMA of w, z, n [mi]
    __shared__ float s_red[8];                                        // [0..3] sums, [4+b] scale
    __shared__ int s_rep[4];                                          // per wave: a multi-hot slot
    const int F = P.F;
    const int FF = F * F;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    // per-row bookkeeping is spread over the waves so no wave works alone before a barrier:
    // wave 1 validates / publishes meta, wave 2 owns the linear (FTRL) terms, wave 3 DMAs meta
    constexpr int W_META = 1, W_LIN = 2, W_DMA = 3;
    const uint32_t nfld = (uint32_t)P.fstride;
    const int G = gridDim.x;
    char* vg = reinterpret_cast<char*>(VG);

    // row-invariant slot decode, packed a | b << 8 (one register per slot; F <= 45)
    int ab[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        const int s = tid + j * 256;
        ab[j] = s < FF ? (s / F) | ((s % F) << 8) : 0;
    }
#define SA(j) (ab[j] & 0xFF)
#define SB(j) (ab[j] >> 8)
    const uint32_t tid_h = (uint32_t)tid * 0x9E3779B1u;

    // wave W_DMA, lanes < F: DMA of one row's raw meta into s_mr[bf] (no registers held)
    auto dma_meta = [&](int bf, int row) {
        if (wave == W_DMA && lane < F && row < P.B) {
            const size_t o = (size_t)row * F + lane;
            __builtin_amdgcn_global_load_lds((glb_ptr_t)(idx + o), (lds_ptr_t)&s_mr[bf][0][0], 4, 0, 0);
            if (fld) __builtin_amdgcn_global_load_lds((glb_ptr_t)(fld + o), (lds_ptr_t)&s_mr[bf][1][0], 4, 0, 0);
            if (val) __builtin_amdgcn_global_load_lds((glb_ptr_t)(val + o), (lds_ptr_t)&s_mr[bf][2][0], 4, 0, 0);
        }
    };
    // wave W_META: raw meta of buffer bf (landed) -> validated s_m[bf] + the L2-norm scale
    auto publish_meta = [&](int bf) {
        if (wave == W_META) {
            float sq = 0.f;
            if (lane < F) {
                int ri = s_mr[bf][0][lane];
                int rf = fld ? s_mr[bf][1][lane] : lane;
                float rx = val ? __int_as_float(s_mr[bf][2][lane]) : 1.f;
                if (ri < 0 || ri >= P.num_features || rf < 0 || rf >= P.num_fields) { ri = -1; rx = 0.f; rf = 0; }
                s_m[bf][lane] = make_int4(ri, rf, __float_as_int(rx), 0);
                sq = rx * rx;
            }
            const float tot = hm::wave_sum_uniform(sq);
            if (lane == 0) s_red[4 + bf] = (P.norm && tot > 0.f) ? rsqrtf(tot) : 1.f;
        }
    };
    // slot j of the row in buffer bf: byte offset, x_a x_b; returns 1 = live (updated),
    // 2 = diagonal (a == b: written back unchanged, so a row rewrites whole 128-B lines of its
    // features' line-padded blocks), 0 = dead (padding, past F*F)
    auto slot = [&](int bf, int j, uint32_t& off, float& xab) -> uint32_t {
        const int4 ma = s_m[bf][SA(j)], mb = s_m[bf][SB(j)];
        const bool ok = (ma.x | mb.x) >= 0 && tid + j * 256 < FF;
        const bool live = ok && SA(j) != SB(j);
        const uint32_t o = ((uint32_t)ma.x * nfld + (uint32_t)mb.y) * SLOT_B;   // branch-free
        const float x = __int_as_float(ma.z) * __int_as_float(mb.z);
        off = ok ? o : 0u;
        xab = live ? x : 0.f;
        return live ? 1u : (ok ? 2u : 0u);
    };
    // DMA of the slots of the row in buffer bf (dead slots fetch slot 0; never read back)
    auto dma_slots = [&](int bf) {
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            uint32_t off;
            float xab;
            slot(bf, j, off, xab);
            if constexpr (BF) {
                __builtin_amdgcn_global_load_lds((glb_ptr_t)(vg + off),
                                                 (lds_ptr_t)(s_raw + j * 256 + wave * 64), 16, 0, 0);
            } else {   // V half, then G half: rows 2j and 2j + 1 of the landing zone
                __builtin_amdgcn_global_load_lds((glb_ptr_t)(vg + off),
                                                 (lds_ptr_t)(s_raw + (2 * j) * 256 + wave * 64), 16, 0, 0);
                __builtin_amdgcn_global_load_lds((glb_ptr_t)(vg + off + 16u),
                                                 (lds_ptr_t)(s_raw + (2 * j + 1) * 256 + wave * 64), 16, 0, 0);
            }
        }
    };
    // wave W_LIN, lanes < F with a valid feature: DMA of w, z, n of the row in buffer bf
    // (issued after this wave's FTRL stores: same-wave order keeps a shared feature's update exact)
    auto dma_lin = [&](int bf) {
        if (P.use_linear && wave == W_LIN && lane < F) {
            const int i = s_m[bf][lane].x;
            if (i >= 0) {
                __builtin_amdgcn_global_load_lds((glb_ptr_t)&LW(w, i), (lds_ptr_t)&s_lin[bf][0][0], 4, 0, 0);
                if (P.train) {
                    __builtin_amdgcn_global_load_lds((glb_ptr_t)&LW(wz, i), (lds_ptr_t)&s_lin[bf][1][0], 4, 0, 0);
                    __builtin_amdgcn_global_load_lds((glb_ptr_t)&LW(wn, i), (lds_ptr_t)&s_lin[bf][2][0], 4, 0, 0);
                }
            }
        }
    };

    int row = blockIdx.x;
    if (row >= P.B) return;
    // ---- prologue: meta(row) -> s_m[0]; DMA of its slots and linear state; meta(row + G) ----
    dma_meta(0, row);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    bar_raw();
    publish_meta(0);
    bar_raw();
    dma_slots(0);
    dma_lin(0);
    dma_meta(1, row + G);

    for (int cur = 0; row < P.B; row += G, cur ^= 1) {
        const int nxt = cur ^ 1;
        const bool more = row + G < P.B;

        // ---- A: every DMA of this wave has landed (slots + lin of this row, meta of the
        //      next), then every wave's ----
        __builtin_amdgcn_s_waitcnt(0x0F70);                                     // vmcnt(0)
        bar_raw();
        // ---- B: raw -> registers, V -> transposed image; meta(row + G) -> s_m[nxt] ----
        uint4 q[NS];
        float4 qv[NS], qg[NS];   // fp32 state
        if constexpr (!BF) {
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                const uint4 a = s_raw[(2 * j) * 256 + tid], b = s_raw[(2 * j + 1) * 256 + tid];
                qv[j] = make_float4(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z), __uint_as_float(a.w));
                qg[j] = make_float4(__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z), __uint_as_float(b.w));
            }
#pragma unroll
            for (int j = 0; j < NS; ++j) s_t[SB(j) * F + SA(j)] = qv[j];
        } else {
#pragma unroll
            for (int j = 0; j < NS; ++j) q[j] = s_raw[j * 256 + tid];
#pragma unroll
            for (int j = 0; j < NS; ++j) s_t[SB(j) * F + SA(j)] = make_uint2(q[j].x, q[j].y);
        }
        uint32_t off[NS];
        float xab[NS];
        uint32_t live = 0u, wr = 0u;
        int rep = 0;
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const uint32_t k = slot(cur, j, off[j], xab[j]);
            live |= (k & 1u) << j;
            wr |= (uint32_t)(k != 0u) << j;
            if (P.defer) rep |= (int)slot_repeats(SA(j), SB(j), s_m[cur][SA(j)], s_m[cur][SB(j)]);
        }
        if (more) publish_meta(nxt);
        bar_raw();
        // ---- C: next row's slot DMA, then the raw meta of the row after it ----
        if (more) {
            dma_slots(nxt);
            dma_meta(cur, row + 2 * G);    // s_mr[cur] was consumed at this row's B
        }
        const float scale = s_red[4 + cur];
        int mi = -1;
        float mx = 0.f, lw = 0.f;
        if (wave == W_LIN && lane < F) {
            const int4 m = s_m[cur][lane];
            mi = m.x;
            mx = __int_as_float(m.z);
            lw = s_lin[cur][0][lane];
        }
        // ---- D: forward ----
        float part = 0.f;
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const int s = tid + j * 256;
            float d;
            if constexpr (BF) {
                const uint2 pv = s_t[s < FF ? s : 0];
                d = dot2_bf16(q[j].x, pv.x, dot2_bf16(q[j].y, pv.y, 0.f));
            } else {
                const float4 pv = s_t[s < FF ? s : 0];
                d = qv[j].x * pv.x + qv[j].y * pv.y + qv[j].z * pv.z + qv[j].w * pv.w;
            }
            part += d * xab[j];
        }
        part *= 0.5f * scale * scale;
        part += lw * mx * scale;
        part = hm::wave_sum_uniform(part);
        const int wrep = __any(rep);
        if (lane == 0) { s_red[wave] = part; s_rep[wave] = wrep; }
        bar_raw();
        float p = s_red[0] + s_red[1] + s_red[2] + s_red[3];
        const bool rdup = (s_rep[0] | s_rep[1] | s_rep[2] | s_rep[3]) != 0;
        if (P.use_bias) p += bias_w0(P, bias);
        const float kappa = row_loss(P, row, p, y, pred_out, loss_out);

        // ---- E: updates (a multi-hot row is deferred to ffm_row_kernel) ----
        if (P.train && rdup && P.defer) {
            defer_row(P, row);
        } else if (P.train) {
            const float ks = kappa * scale * scale;
            const f2 eps = {P.eps, P.eps};
            const f2 meta = {-P.eta0, -P.eta0};
            uint32_t hrow = (P.seed ^ ((uint32_t)row * 0x85EBCA77u)) + tid_h;
            hrow ^= hrow >> 16;
            hrow *= 0x7FEB352Du;
            hrow ^= hrow >> 15;
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                const int s = tid + j * 256;
                const f2 coef = {ks * xab[j], ks * xab[j]};
                f2 o0, o1, g0, g1, p0, p1;
                if constexpr (BF) {
                    const uint2 pv = s_t[s < FF ? s : 0];
                    o0 = bf2_to_f2(q[j].x); o1 = bf2_to_f2(q[j].y);
                    g0 = bf2_to_f2(q[j].z); g1 = bf2_to_f2(q[j].w);
                    p0 = bf2_to_f2(pv.x);   p1 = bf2_to_f2(pv.y);
                } else {
                    const float4 pv = s_t[s < FF ? s : 0];
                    o0 = f2{qv[j].x, qv[j].y}; o1 = f2{qv[j].z, qv[j].w};
                    g0 = f2{qg[j].x, qg[j].y}; g1 = f2{qg[j].z, qg[j].w};
                    p0 = f2{pv.x, pv.y};       p1 = f2{pv.z, pv.w};
                }
                // diagonal slots: coef = 0 and lambda = 0 -> d = 0, V and G unchanged, and the
                // stochastic rounding of a value already in bf16 is exact
                const float lj = (live >> j & 1u) ? P.lambda_v : 0.f;
                const f2 lamj = {lj, lj};
                const f2 d0 = coef * p0 + lamj * o0, d1 = coef * p1 + lamj * o1;
                g0 = g0 + d0 * d0;
                g1 = g1 + d1 * d1;
                const f2 t0 = g0 + eps, t1 = g1 + eps;
                const f2 r0 = {__builtin_amdgcn_rsqf(t0.x), __builtin_amdgcn_rsqf(t0.y)};
                const f2 r1 = {__builtin_amdgcn_rsqf(t1.x), __builtin_amdgcn_rsqf(t1.y)};
                o0 = o0 + meta * d0 * r0;
                o1 = o1 + meta * d1 * r1;
                if constexpr (!BF) {
                    if (wr >> j & 1u) {
                        *reinterpret_cast<float4*>(vg + off[j]) = make_float4(o0.x, o0.y, o1.x, o1.y);
                        *reinterpret_cast<float4*>(vg + off[j] + 16u) = make_float4(g0.x, g0.y, g1.x, g1.y);
                    }
                    continue;
                }
                // this thread's row hash, re-keyed per slot: each 16-bit window stays uniform
                const uint32_t h = rotl32(hrow, 5 * j + 1) ^ (0x9E3779B9u * (uint32_t)(j + 1));
                const uint4 st = make_uint4(pack_sr_hi(o0, h, rotl32(h, 16)),
                                            pack_sr_hi(o1, rotl32(h, 8), rotl32(h, 24)),
                                            pack_sr_hi(g0, rotl32(h, 4), rotl32(h, 20)),
                                            pack_sr_hi(g1, rotl32(h, 12), rotl32(h, 28)));
                if (wr >> j & 1u) *reinterpret_cast<uint4*>(vg + off[j]) = st;
            }
            // the feature blocks' pad slots (never read): zeros, completing their last lines;
            // written by wave 0 (wave W_LIN has the FTRL updates: one wave doing both was the
            // last to reach the barrier, cf. ffm_pipe_sg32_kernel)
            if (wave == 0 && lane < F) {
                const int pi = s_m[cur][lane].x;
                if (pi >= 0) {
                    for (int f = P.num_fields; f < (int)nfld; ++f) {
                        *reinterpret_cast<uint4*>(vg + ((uint32_t)pi * nfld + (uint32_t)f) * SLOT_B) = make_uint4(0u, 0u, 0u, 0u);
                        if (!BF) *reinterpret_cast<uint4*>(vg + ((uint32_t)pi * nfld + (uint32_t)f) * SLOT_B + 16u) = make_uint4(0u, 0u, 0u, 0u);
                    }
                }
            }
            if (mi >= 0) {
                if (P.use_linear) {   // FTRL-proximal on the DMA'd (w, z, n)
                    const float lz = s_lin[cur][1][lane];
                    const float ln = s_lin[cur][2][lane];
                    const float g = kappa * mx * scale;
                    const float n1 = ln + g * g;
                    const float z1 = lz + g - (sqrtf(n1) - sqrtf(ln)) / P.alpha * lw;
                    LW(wz, mi) = z1;
                    LW(wn, mi) = n1;
                    LW(w, mi) = ftrl_weight(z1, n1, P.alpha, P.beta, P.lambda1, P.lambda2);
                }
            }
            if (P.use_bias && tid == 0) bias_update(P, kappa, bias);
        }
        // ---- F: linear state of the next row (after this row's FTRL stores) ----
        if (more) dma_lin(nxt);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);       // no LDS-DMA outstanding at exit
#undef SA
#undef SB
}


// Coherent-cache variant (SC1 DMA loads that bypass L1, SC1 write-through stores that drop the
// line from the writer's L2) was measured and removed: 9.6 M rows/s vs 75.2 M, held-out logloss
// 0.44742 vs 0.4478 (sequential 0.44501) — the same-stream gap is the concurrency of Hogwild
// updates itself, not stale L1/L2 copies across XCDs (profiles/r4/ffm_coh_variant_parity.log).
typedef uint32_t u3v_t __attribute__((ext_vector_type(3)));

// ---------------------------------------------------------------------------------------------
// LDS-DMA pipelined kernel for per-slot AdaGrad with fp32 V in the block layout
// ([V: FS x 16 B | G: FS x fp32 | zero tail] per feature, 896 B): the schedule of
// ffm_pipe_kernel (A..F above) with two DMAs per slot (V 16 B, G 4 B) into separate landing
// zones.  A register-prefetch variant of this layout reached 66-68 M rows/s (70 % of the
// access-pattern ceiling, 97.5 M rows/s: profiles/ffm_r3/roofline_sg.log, ab_fp32_sg_reg_*.log;
// removed); here no VGPR holds the next row and the LDS image is the only staging (55 KB per
// block -> 2 blocks/CU).
// s_waitcnt immediate: vmcnt(n) (n <= 63), expcnt / lgkmcnt not waited on
#define VMCNT_ENC(n) ((((n) & 15) | (((n) >> 4) << 14)) | 0x0F70)
// KV = 16-B quads per slot: 1 for k <= 4 (the 896-B blocks above), 2 for k <= 8 (32-B V slots,
// 1,536-B blocks; the landing zone and the image double, 107 KB of LDS at 39 fields: one block
// per CU, launched with 512 threads so that each SIMD still holds two waves).
// KEEP >= 1 (round 6; the default is 2, variant 10 = 1, variant 9 = 0 for A/B): each slot's offsets, x_a x_b and live / written / repeat bits are derived
// from the row metadata ONCE, in phase C (next to that row's DMA issue), and kept in registers
// for the row's B / D / E phases; the other phases re-read both metadata entries of every slot from
// LDS, and the (b)-side reads of 16-B entries conflict where b wraps from F - 1 to 0 inside a
// 16-lane group (2.7 extra LDS cycles per such read at F = 39, profiles/r6/lds_conflict_model.txt).
// Measured (profiles/r6/keep_*): LDS bank-conflict cycles 210 M -> 30 M and LDS instructions 115 M
// -> 72 M per 262,144-row dispatch; bench 93.0-93.3 vs 89.2-89.4 M rows/s fp32, same box,
// interleaved x3; one block still equals the sequential engine to 3e-8 (k = 4) / 6e-8 (k = 8).
// KEEP = 2 also keeps the forward pass's two image reads per slot for the update phase (the image
// is not written between D and E): 94.2-97.6 vs 92.8-95.4 M rows/s fp32, 153.6-154.3 vs
// 149.6-150.6 M bf16, same box, interleaved x3 (profiles/r6/keep/bench_keep2_ab.log).
template <int NS, typename OT, int TPB = 256, int ATOM = 0, int KV = 1, int KEEP = 0, int LT = 0>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(TPB / 128))) void ffm_pipe_sg32_kernel(
    FFMParams P, const int32_t* __restrict__ idx, const int32_t* __restrict__ fld,
    const float* __restrict__ val, const float* __restrict__ y, void* __restrict__ Vt,
    float* __restrict__ Gt, float* __restrict__ w, float* __restrict__ wz, float* __restrict__ wn,
    float* __restrict__ bias, float* __restrict__ pred_out, float* __restrict__ loss_out)
{
    __shared__ __attribute__((aligned(16))) float4 s_rv[NS * TPB * KV]; // V DMA landing zone [q][j][tid]
    __shared__ __attribute__((aligned(16))) float s_rg[NS * TPB];     // G DMA landing zone
    __shared__ __attribute__((aligned(16))) float4 s_t[NS * TPB * KV];  // transposed V image [slot][q]
    __shared__ __attribute__((aligned(16))) int4 s_m[2][48];          // validated meta {i, f, x}
    __shared__ __attribute__((aligned(16))) int s_mr[2][3][48];       // raw meta DMA {idx, fld, val}
    __shared__ __attribute__((aligned(16))) float s_lin[2][3][48];    // DMA of w, z, n [mi]
    __shared__ __attribute__((aligned(16))) float4 s_lin4[2][48];     // ... as {w, z, n, _} (lpack)
    __shared__ float s_red[TPB / 64 + 2];                             // [0..NW) sums, [NW+b] scale
    __shared__ int s_rep[TPB / 64];                                   // per wave: a multi-hot slot
    __shared__ float s_bias[4];                                       // the row's {w0, z0, n0}
    __shared__ float s_bcur[2];                                       // own bias steps since the read
    // LT (lin_atomic 4, HD_SIZE above): the block's own linear steps of hot features, summed per
    // hot index, and the rows' DMA of the side table
    __shared__ float2 s_hd[LT ? HD_SIZE : 1];
    __shared__ __attribute__((aligned(16))) float4 s_hacc[LT ? 2 : 1][48];
    __shared__ __attribute__((aligned(16))) int s_nh[LT ? 2 : 1][48];   // DMA of the rows' hot indices
    const int F = P.F;
    const int FF = F * F;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    constexpr int W_META = 1, W_LIN = 2, W_DMA = 3;
    const OT vfs = (OT)P.fstride * (16u * KV);           // V bytes between features
    const OT gfs = (OT)P.gstride * 4u;                   // G bytes between features
    // (One table replica per XCD, averaged between launches, was measured and removed: +3.1e-3 ..
    // +5.4e-3 vs sequential on the bench stream instead of +2.4e-3; profiles/r5/ffm_xrep_probe.jsonl.)
    const int G = (int)gridDim.x;
    const int bid = (int)blockIdx.x;
    char* vb = reinterpret_cast<char*>(Vt);
    char* gb = reinterpret_cast<char*>(Gt);
    // linear (z, n) steps by float atomics (FFMParams.lin_atomic; 2 / 3: only the features P.hot
    // flags / does not flag, A/B); one block stores them (exact)
    const bool latom = ATOM == 0 && !LT && P.lin_atomic == 1 && G > 1;
    if constexpr (LT != 0) {
        for (int t = tid; t < HD_SIZE; t += TPB) s_hd[t] = make_float2(0.f, 0.f);
    }
    int nh = -1, kh = -1;            // LT, W_LIN lanes: hot index of the next / current row's feature

    int ab[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        const int s = tid + j * TPB;
        ab[j] = s < FF ? (s / F) | ((s % F) << 8) : 0;
    }
#define SA(j) (ab[j] & 0xFF)
#define SB(j) (ab[j] >> 8)

    auto dma_meta = [&](int bf, int row) {
        if (wave == W_DMA && lane < F && row < P.B) {
            const size_t o = (size_t)row * F + lane;
            __builtin_amdgcn_global_load_lds((glb_ptr_t)(idx + o), (lds_ptr_t)&s_mr[bf][0][0], 4, 0, 0);
            if (fld) __builtin_amdgcn_global_load_lds((glb_ptr_t)(fld + o), (lds_ptr_t)&s_mr[bf][1][0], 4, 0, 0);
            if (val) __builtin_amdgcn_global_load_lds((glb_ptr_t)(val + o), (lds_ptr_t)&s_mr[bf][2][0], 4, 0, 0);
        }
    };
    auto publish_meta = [&](int bf) {
        if (wave == W_META) {
            float sq = 0.f;
            if (lane < F) {
                int ri = s_mr[bf][0][lane];
                int rf = fld ? s_mr[bf][1][lane] : lane;
                float rx = val ? __int_as_float(s_mr[bf][2][lane]) : 1.f;
                if (ri < 0 || ri >= P.num_features || rf < 0 || rf >= P.num_fields) { ri = -1; rx = 0.f; rf = 0; }
                const int hb = ((ATOM == 2 || (latom && P.lin_atomic >= 2)) && ri >= 0) ? (int)P.hot[ri] : 0;
                s_m[bf][lane] = make_int4(ri, rf, __float_as_int(rx), hb);
                sq = rx * rx;
            }
            const float tot = hm::wave_sum_uniform(sq);
            if (lane == 0) s_red[TPB / 64 + bf] = (P.norm && tot > 0.f) ? rsqrtf(tot) : 1.f;
        }
    };
    // slot j of the row in s_m[bf]: V / G byte offsets, x_a x_b; 1 = live, 2 = diagonal, 0 = dead
    auto slot = [&](int bf, int j, OT& ov, OT& og, float& xab) -> uint32_t {
        const int4 ma = s_m[bf][SA(j)], mb = s_m[bf][SB(j)];
        const bool ok = (ma.x | mb.x) >= 0 && tid + j * TPB < FF;
        const bool live = ok && SA(j) != SB(j);
        const OT i = ok ? (OT)(uint32_t)ma.x : (OT)0, f = ok ? (OT)(uint32_t)mb.y : (OT)0;
        ov = i * vfs + f * (16u * KV);
        og = i * gfs + f * 4u;
        xab = live ? __int_as_float(ma.z) * __int_as_float(mb.z) : 0.f;
        return live ? 1u : (ok ? 2u : 0u);
    };
    // KEEP: the slot data of the row whose DMA was issued last (nov / nog / nxab / bits), handed to
    // the current-row registers (kov / kog / kxab / bits) at the end of each row
    OT kov[KEEP ? NS : 1], kog[KEEP ? NS : 1], nov[KEEP ? NS : 1], nog[KEEP ? NS : 1];
    float kxab[KEEP ? NS : 1], nxab[KEEP ? NS : 1];
    uint32_t klive = 0u, kwr = 0u, nlive = 0u, nwr = 0u;
    int krep = 0, nrep = 0;
    auto dma_slots = [&](int bf) {
        if constexpr (KEEP) { nlive = 0u; nwr = 0u; nrep = 0; }
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            OT ov, og;
            float xab;
            const uint32_t k = slot(bf, j, ov, og, xab);
            if constexpr (KEEP) {
                nov[j] = ov;
                nog[j] = og;
                nxab[j] = xab;
                nlive |= (k & 1u) << j;
                nwr |= (uint32_t)(k != 0u) << j;
                if (P.defer) nrep |= (int)slot_repeats(SA(j), SB(j), s_m[bf][SA(j)], s_m[bf][SB(j)]);
            }
#pragma unroll
            for (int q = 0; q < KV; ++q)
                __builtin_amdgcn_global_load_lds((glb_ptr_t)(vb + ov + 16u * q),
                                                 (lds_ptr_t)(s_rv + (q * NS + j) * TPB + wave * 64), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((glb_ptr_t)(gb + og), (lds_ptr_t)(s_rg + j * TPB + wave * 64), 4, 0, 0);
        }
    };
    auto keep_rotate = [&]() {
        if constexpr (KEEP) {
#pragma unroll
            for (int j = 0; j < NS; ++j) { kov[j] = nov[j]; kog[j] = nog[j]; kxab[j] = nxab[j]; }
            klive = nlive; kwr = nwr; krep = nrep;
        }
    };
    // The linear state of the next row is DMA'd after this row's FTRL stores (phase F), so it is
    // the W_LIN wave's youngest load at the next phase A.  That wave therefore waits there only for
    // its older slot DMAs (vmcnt(NLIN)), and for the linear DMA right before its first read in D
    // (vmcnt(2 NS): only the next row's slot DMAs, issued in C, may still be in flight).  Every
    // lane < F issues the DMAs (an invalid feature reads w[0], unused), so the counts are exact.
    const int nlin = (P.use_linear && P.lin_defer) ? ((P.lpack || !P.train) ? 1 + (LT != 0) : 3) : 0;
    auto dma_lin = [&](int bf) {
        if (P.use_linear && wave == W_LIN && lane < F) {
            const int i = max(s_m[bf][lane].x, 0);
            if (P.lpack) {
                __builtin_amdgcn_global_load_lds((glb_ptr_t)&LW(w, i), (lds_ptr_t)&s_lin4[bf][0], 16, 0, 0);
                if constexpr (LT != 0)   // every lane: the wave's DMA count stays exact
                    __builtin_amdgcn_global_load_lds((glb_ptr_t)(P.hacc + HACC_STRIDE * max(nh, 0)), (lds_ptr_t)&s_hacc[bf][0], 16, 0, 0);
                return;
            }
            __builtin_amdgcn_global_load_lds((glb_ptr_t)&LW(w, i), (lds_ptr_t)&s_lin[bf][0][0], 4, 0, 0);
            if (P.train) {
                __builtin_amdgcn_global_load_lds((glb_ptr_t)&LW(wz, i), (lds_ptr_t)&s_lin[bf][1][0], 4, 0, 0);
                __builtin_amdgcn_global_load_lds((glb_ptr_t)&LW(wn, i), (lds_ptr_t)&s_lin[bf][2][0], 4, 0, 0);
            }
        }
    };

    int row = bid;
    if (row >= P.B) return;
    if (tid == 0) { s_bcur[0] = 0.f; s_bcur[1] = 0.f; }
    dma_meta(0, row);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    bar_raw();
    publish_meta(0);
    bar_raw();
    dma_slots(0);
    keep_rotate();
    if constexpr (LT != 0) {
        if (wave == W_LIN && lane < F) nh = s_m[0][lane].x >= 0 ? P.hidx[s_m[0][lane].x] : -1;
    }
    dma_lin(0);
    kh = nh;
    dma_meta(1, row + G);

    // Forwarding of the block's own updates into its next row: the next row's slots are DMA'd
    // (phase C) before this row's updates land (phase E), so a slot both rows hold — the same
    // (feature, field), hence the same slot index and thread when the rows share a feature at one
    // position — would be read one update stale.  The updating thread keeps the new V / G and
    // their offset, and phase B of the next row takes them instead of the landing zone.
    float4 fv[NS][KV];
    float fg[NS];
    OT fo[NS];
    uint32_t fwd = 0u;
    const bool bsh = P.use_bias && P.bias_sh;
    // A block re-reads the 64 shard lines every bias_every rows (loads of lines the other blocks'
    // atomics keep updating are slow: every row took -w0 from 75 to 40 M rows/s) and adds its own
    // steps since that read (s_bcur) in between; the other blocks' steps arrive with the next read.
    int bit = 0;                    // rows of this block so far
    float bz = 0.f, bn = 0.f;       // the W_META lanes' copy of the shard sums, loaded a row ahead
    if (bsh && wave == W_META && lane < P.bias_s) {
        bz = __hip_atomic_load(P.bias_sh + lane * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bn = __hip_atomic_load(P.bias_sh + lane * 32 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int cur = 0; row < P.B; row += G, cur ^= 1) {
        const int nxt = cur ^ 1;
        const bool more = row + G < P.B;
        // ---- A: this wave's DMAs have landed, then every wave's ----
        if (wave == W_LIN && nlin == 3) __builtin_amdgcn_s_waitcnt(0x0F73);      // vmcnt(3)
        else if (wave == W_LIN && nlin == 2) __builtin_amdgcn_s_waitcnt(0x0F72); // vmcnt(2)
        else if (wave == W_LIN && nlin == 1) __builtin_amdgcn_s_waitcnt(0x0F71); // vmcnt(1)
        else __builtin_amdgcn_s_waitcnt(0x0F70);                                // vmcnt(0)
        bar_raw();
        // the bias shards for the NEXT row (one row of extra staleness on one parameter, as
        // train_fm's w0): issued here, landed by the next phase A's vmcnt(0), used in its D
        // this row re-reads (block-uniform); not the block's first row: the shards were just read
        const bool bre = bsh && bit > 0 && (bit % P.bias_every) == 0;
        float nbz = bz, nbn = bn;
        if (bre && wave == W_META && lane < P.bias_s) {
            nbz = __hip_atomic_load(P.bias_sh + lane * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            nbn = __hip_atomic_load(P.bias_sh + lane * 32 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // ---- B: landing zone -> registers (G) and the transposed image (V); meta(row + G) ----
        if constexpr (LT != 0) {
            // the next row's hot indices by LDS-DMA from its raw meta (landed at A): older than the
            // slot DMAs of phase C, so C's wait covers them and phase F reads them from LDS
            if (more && wave == W_LIN && lane < F) {
                const int ri = s_mr[nxt][0][lane];
                __builtin_amdgcn_global_load_lds((glb_ptr_t)(P.hidx + (ri >= 0 && ri < P.num_features ? ri : 0)),
                                                 (lds_ptr_t)&s_nh[nxt][0], 4, 0, 0);
            }
        }
        float cg[NS];
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            cg[j] = s_rg[j * TPB + tid];
            float4 v[KV];
#pragma unroll
            for (int q = 0; q < KV; ++q) v[q] = s_rv[(q * NS + j) * TPB + tid];
            if (fwd >> j & 1u) {
                bool same;
                if constexpr (KEEP) {
                    same = (kwr >> j & 1u) && kov[j] == fo[j];
                } else {
                    OT ov, og;
                    float xq;
                    same = slot(cur, j, ov, og, xq) != 0u && ov == fo[j];
                }
                if (same) {
#pragma unroll
                    for (int q = 0; q < KV; ++q) v[q] = fv[j][q];
                    cg[j] = fg[j];
                }
            }
            if (tid + j * TPB < FF) {
#pragma unroll
                for (int q = 0; q < KV; ++q) s_t[(SB(j) * F + SA(j)) * KV + q] = v[q];
            }
        }
        fwd = 0u;
        if (more) publish_meta(nxt);
        bar_raw();
        // ---- C: next row's slot DMA (the landing zones are free: read in B), its meta after ----
        if (more) {
            dma_slots(nxt);
            dma_meta(cur, row + 2 * G);
        }
        const float scale = s_red[TPB / 64 + cur];
        int mi = -1;
        float mx = 0.f, lw = 0.f;
        int hot = 0;                     // LT: this lane's feature is hot (kh >= 0)
        float hz = 0.f, hn = 0.f;        // LT: its (z, n) as this block sees them
        if (wave == W_LIN && nlin) {
            // the linear DMA of this row has landed (older than the C-phase slot DMAs)
            if (more) __builtin_amdgcn_s_waitcnt(VMCNT_ENC((KV + 1) * NS));
            else __builtin_amdgcn_s_waitcnt(0x0F70);
        }
        if (wave == W_LIN && lane < F) {
            const int4 m = s_m[cur][lane];
            mi = m.x;
            mx = __int_as_float(m.z);
            lw = P.lpack ? s_lin4[cur][lane].x : s_lin[cur][0][lane];
            if (latom) lw = lin_w(P, s_lin4[cur][lane]);
            if constexpr (LT != 0) {
                if (P.hacc_on && mi >= 0 && kh >= 0) {
                    // hot: the side table as DMA'd (the other blocks' flushed steps) + this block's own
                    const float4 a = s_hacc[cur][lane];
                    const float2 d = s_hd[kh];
                    hz = a.x + d.x;
                    hn = a.y + d.y;
                    hot = 1;
                    lw = hn > 0.f ? ftrl_weight(hz, hn, P.alpha, P.beta, P.lambda1, P.lambda2) : lw;
                }
            }
        }
        // ---- D: forward ----
        uint32_t live = 0u, wr = 0u;
        float xab[NS];
        float4 kpv[KEEP >= 2 ? NS : 1][KEEP >= 2 ? KV : 1], kcv[KEEP >= 2 ? NS : 1][KEEP >= 2 ? KV : 1];
        float part = 0.f;
        int rep = 0;
        if constexpr (KEEP) { live = klive; wr = kwr; rep = krep; }
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            if constexpr (KEEP) {
                xab[j] = kxab[j];
            } else {
                OT ov, og;
                const uint32_t k = slot(cur, j, ov, og, xab[j]);
                live |= (k & 1u) << j;
                wr |= (uint32_t)(k != 0u) << j;
                if (P.defer) rep |= (int)slot_repeats(SA(j), SB(j), s_m[cur][SA(j)], s_m[cur][SB(j)]);
            }
            const int s = tid + j * TPB;
            float dot = 0.f;
#pragma unroll
            for (int q = 0; q < KV; ++q) {
                const float4 pv = s_t[(s < FF ? s : 0) * KV + q];
                const float4 cv = s_t[(SB(j) * F + SA(j)) * KV + q];
                if constexpr (KEEP >= 2) { kpv[j][q] = pv; kcv[j][q] = cv; }
                dot += cv.x * pv.x + cv.y * pv.y + cv.z * pv.z + cv.w * pv.w;
            }
            part += dot * xab[j];
        }
        part *= 0.5f * scale * scale;
        part += lw * mx * scale;
        part = hm::wave_sum_uniform(part);
        const int wrep = __any(rep);
        if (bsh && wave == W_META) {
            const float z = hm::wave_sum_uniform(bz) + s_bcur[0], n = hm::wave_sum_uniform(bn) + s_bcur[1];
            if (lane == 0) { s_bias[0] = ftrl_weight(z, n, P.alpha, P.beta, 0.f, 0.f); s_bias[1] = z; s_bias[2] = n; }
        }
        if (lane == 0) { s_red[wave] = part; s_rep[wave] = wrep; }
        bar_raw();
        float p = 0.f;
        int rdup = 0;
#pragma unroll
        for (int q = 0; q < TPB / 64; ++q) { p += s_red[q]; rdup |= s_rep[q]; }
        if (P.use_bias) p += bsh ? s_bias[0] : bias_w0(P, bias);
        const float kappa = row_loss(P, row, p, y, pred_out, loss_out);

        // ---- E: updates (a multi-hot row is deferred to ffm_row_kernel) ----
        // the shards read at this row's B lack only this row's own step (wave 0 waits for its
        // atomics at every phase A, so all earlier ones had landed)
        if (bre && tid == 0) { s_bcur[0] = 0.f; s_bcur[1] = 0.f; }
        if (P.train && rdup && P.defer) {
            defer_row(P, row);
        } else if (P.train) {
            const float ks = kappa * scale * scale;
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                if (!(wr >> j & 1u)) continue;
                OT ov, og;
                if constexpr (KEEP) {
                    ov = kov[j];
                    og = kog[j];
                } else {
                    float xj;
                    slot(cur, j, ov, og, xj);
                }
                const int s = tid + j * TPB;
                const float c = ks * xab[j];
                const float lj = (live >> j & 1u) ? P.lambda_v : 0.f;   // diagonal: zero step
                const f2 cc = {c, c}, ll = {lj, lj};
                f2 o0[KV], o1[KV], d0[KV], d1[KV];
                float gs = cg[j];
#pragma unroll
                for (int q = 0; q < KV; ++q) {
                    // KEEP >= 2: the two image reads of the forward pass, kept in registers (the
                    // image is not written between D and E)
                    const float4 pv = KEEP >= 2 ? kpv[j][q] : s_t[s * KV + q];
                    const float4 cv = KEEP >= 2 ? kcv[j][q] : s_t[(SB(j) * F + SA(j)) * KV + q];
                    o0[q] = f2{cv.x, cv.y};
                    o1[q] = f2{cv.z, cv.w};
                    const f2 p0 = f2{pv.x, pv.y}, p1 = f2{pv.z, pv.w};
                    d0[q] = cc * p0 + ll * o0[q];
                    d1[q] = cc * p1 + ll * o1[q];
                    gs = (((gs + d0[q].x * d0[q].x) + d0[q].y * d0[q].y) + d1[q].x * d1[q].x) + d1[q].y * d1[q].y;
                }
                const float r = __builtin_amdgcn_rsqf(gs + P.eps) * -P.eta0;
                const f2 rr = {r, r};
#pragma unroll
                for (int q = 0; q < KV; ++q) {
                    const f2 n0 = o0[q] + rr * d0[q], n1 = o1[q] + rr * d1[q];
                    fv[j][q] = make_float4(n0.x, n0.y, n1.x, n1.y);
                }
                fg[j] = gs;
                fo[j] = ov;
                fwd |= 1u << j;
                if (ATOM == 1 || (ATOM == 2 && s_m[cur][SA(j)].w != 0)) {
                    // concurrent rows' updates of one slot all land (no read-modify-write race)
                    if (live >> j & 1u) {
                        float* vp = reinterpret_cast<float*>(vb + ov);
#pragma unroll
                        for (int q = 0; q < KV; ++q) {
                            const f2 e0 = rr * d0[q], e1 = rr * d1[q];
                            atomicAdd(vp + 4 * q + 0, e0.x);
                            atomicAdd(vp + 4 * q + 1, e0.y);
                            atomicAdd(vp + 4 * q + 2, e1.x);
                            atomicAdd(vp + 4 * q + 3, e1.y);
                        }
                        atomicAdd(reinterpret_cast<float*>(gb + og), gs - cg[j]);
                    }
                    continue;
                }
#pragma unroll
                for (int q = 0; q < KV; ++q) *reinterpret_cast<float4*>(vb + ov + 16u * q) = fv[j][q];
                *reinterpret_cast<float*>(gb + og) = fg[j];
            }
            // (The pad slots and block tails are never read.  Zeroing them so that every line a
            // row touches is written whole cost 1.5 %: 73.7-74.0 vs 75.0-75.2 M rows/s, same
            // held-out logloss, profiles/r4/ffm_no_pad_stores_ab.log.  Skipping the DMA and the
            // store of the diagonal / dead slots too was slower: 72.4-72.7 vs 74.9-75.5 M,
            // profiles/r4/ffm_skip_diagonal_ab.log.)
            if (mi >= 0) {
                if (P.use_linear) {   // FTRL-proximal on the DMA'd (w, z, n)
                    const float lz = hot ? hz : (P.lpack ? s_lin4[cur][lane].y : s_lin[cur][1][lane]);
                    const float ln = hot ? hn : (P.lpack ? s_lin4[cur][lane].z : s_lin[cur][2][lane]);
                    const float g = kappa * mx * scale;
                    const float n1 = ln + g * g;
                    const float z1 = lz + g - (sqrtf(n1) - sqrtf(ln)) / P.alpha * lw;
                    const float w1 = ftrl_weight(z1, n1, P.alpha, P.beta, P.lambda1, P.lambda2);
                    if (LT && hot) {
                        const float2 d = s_hd[kh];
                        s_hd[kh] = make_float2(d.x + (g - (sqrtf(n1) - sqrtf(ln)) / P.alpha * lw), d.y + g * g);
                    } else if (ATOM == 1 || (ATOM == 2 && s_m[cur][lane].w != 0)) {
                        atomicAdd(&LW(wz, mi), z1 - lz);
                        atomicAdd(&LW(wn, mi), g * g);
                        LW(w, mi) = w1;
                    } else if (latom && (P.lin_atomic == 1 || (P.lin_atomic == 2) == (s_m[cur][lane].w != 0))) {
                        lin_add(P, w, mi, g, ln, n1, lw);
                    } else if (P.lpack) {
                        *reinterpret_cast<float4*>(&LW(w, mi)) = make_float4(w1, z1, n1, s_lin4[cur][lane].w);
                    } else {
                        LW(wz, mi) = z1;
                        LW(wn, mi) = n1;
                        LW(w, mi) = w1;
                    }
                }
            }
            if (P.use_bias && tid == 0) {
                if (bsh) bias_update_sh(P, kappa, s_bias[1], s_bias[2], P.bias_sh + (blockIdx.x % P.bias_s) * 32, s_bcur);
                else bias_update(P, kappa, bias);
            }
        }
        // ---- F: linear state of the next row (after this row's FTRL stores) ----
        if constexpr (LT != 0) {
            if (more && wave == W_LIN && lane < F) nh = s_nh[nxt][lane];
        }
        if (more) dma_lin(nxt);
        kh = nh;
        keep_rotate();
        bz = nbz;
        bn = nbn;
        ++bit;
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);       // no LDS-DMA outstanding at exit
    if constexpr (LT != 0) {
        // the block's summed hot steps -> the side table (every wave; the W_LIN wave's LDS adds
        // are published by the barrier).  No-return atomics, not waited for: a wait here for their
        // completion under every block's contention cost 89 -> 68 M rows/s (profiles/r6/linhot/)
        bar_raw();
        // Lanes 2e, 2e + 1 add z, n of entry e (one 8-B run per entry and instruction: 67 -> 76 M
        // rows/s against one lane adding both)
        if (P.hacc_on)
            for (int t = tid; t < 2 * P.nhot; t += TPB) {
                const float2 d = s_hd[t >> 1];
                if (d.y != 0.f || d.x != 0.f) atomicAdd(P.hacc + HACC_STRIDE * (t >> 1) + (t & 1), (t & 1) ? d.y : d.x);
            }
    }
#undef SA
#undef SB
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA pipelined kernel for per-slot AdaGrad with bf16 V in 12-B slots {V bf16 x 4 | G fp32}:
// 40 slots per feature = 480 B + a 32-B zero tail = one 512-B block (4 lines; the 16-B
// {V | G | 0} slots need 5).  One 12-B LDS-DMA (global_load_lds_dwordx3) and one 12-B store
// per slot; otherwise the schedule of ffm_pipe_sg32_kernel.  Access-pattern ceiling of this
// footprint: 182 M rows/s (profiles/ffm_r3/roofline_sg.log, mode 6), 16-B slots 138 M.
// KEEP (round 6; default 2, variant 10 = 1, variant 9 = 0): the slot data kept in registers from
// phase C, and with 2 the forward's image reads kept for the update, as in ffm_pipe_sg32_kernel
// (the 16-B metadata reads of the b-side conflict where b wraps).
template <int NS, typename OT, int KEEP = 0, int LT = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void ffm_pipe_sg12_kernel(
    FFMParams P, const int32_t* __restrict__ idx, const int32_t* __restrict__ fld,
    const float* __restrict__ val, const float* __restrict__ y, void* __restrict__ Vt,
    float* __restrict__ w, float* __restrict__ wz, float* __restrict__ wn,
    float* __restrict__ bias, float* __restrict__ pred_out, float* __restrict__ loss_out)
{
    // 12-B slot landing zone: global_load_lds_dwordx3 lands each lane at a 16-B stride
    // (measured: benchmarks/lds_dma12_probe.py, profiles/ffm_r3/lds_dma12_probe.log)
    __shared__ __attribute__((aligned(16))) uint32_t s_raw[NS * 256 * 4];
    __shared__ __attribute__((aligned(16))) uint2 s_t[NS * 256];            // transposed V image
    __shared__ __attribute__((aligned(16))) int4 s_m[2][48];
    __shared__ __attribute__((aligned(16))) int s_mr[2][3][48];
    __shared__ __attribute__((aligned(16))) float s_lin[2][3][48];
    __shared__ __attribute__((aligned(16))) float4 s_lin4[2][48];     // ... as {w, z, n, _} (lpack)
    __shared__ float s_red[8];
    __shared__ int s_rep[4];                                                  // per wave: a multi-hot slot
    __shared__ float s_bias[4];                                       // the row's {w0, z0, n0}
    __shared__ float s_bcur[2];                                       // own bias steps since the read
    // LT: the side table of ffm_pipe_sg32_kernel with at most HD12_SIZE hot features (8 KB of sums:
    // 3 blocks per CU still fit)
    __shared__ float2 s_hd[LT ? HD12_SIZE : 1];
    __shared__ __attribute__((aligned(16))) float4 s_hacc[LT ? 2 : 1][48];
    __shared__ __attribute__((aligned(16))) int s_nh[LT ? 2 : 1][48];
    const int F = P.F;
    const int FF = F * F;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    constexpr int W_META = 1, W_LIN = 2, W_DMA = 3;
    const OT bs = (OT)P.gstride * 4u;                    // block bytes per feature
    const int G = gridDim.x;
    char* vb = reinterpret_cast<char*>(Vt);
    const bool latom = !LT && P.lin_atomic == 1 && G > 1;   // as in ffm_pipe_sg32_kernel
    if constexpr (LT != 0) {
        for (int t = tid; t < HD12_SIZE; t += 256) s_hd[t] = make_float2(0.f, 0.f);
    }
    int nh = -1, kh = -1;            // LT, W_LIN lanes: hot index of the next / current row's feature
    // linear records inside the blocks (the first 16-B chunk after the 12-B slots), whether they
    // are accessed as one 16-B record (lpack) or as three 4-B words: the tail zeroing skips them
    const bool lin_in_tail = reinterpret_cast<const char*>(w) == vb + (size_t)P.vpad * 12;
    typedef uint32_t u3v __attribute__((ext_vector_type(3)));

    int ab[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        const int s = tid + j * 256;
        ab[j] = s < FF ? (s / F) | ((s % F) << 8) : 0;
    }
#define SA(j) (ab[j] & 0xFF)
#define SB(j) (ab[j] >> 8)
    const uint32_t tid_h = (uint32_t)tid * 0x9E3779B1u;

    auto dma_meta = [&](int bf, int row) {
        if (wave == W_DMA && lane < F && row < P.B) {
            const size_t o = (size_t)row * F + lane;
            __builtin_amdgcn_global_load_lds((glb_ptr_t)(idx + o), (lds_ptr_t)&s_mr[bf][0][0], 4, 0, 0);
            if (fld) __builtin_amdgcn_global_load_lds((glb_ptr_t)(fld + o), (lds_ptr_t)&s_mr[bf][1][0], 4, 0, 0);
            if (val) __builtin_amdgcn_global_load_lds((glb_ptr_t)(val + o), (lds_ptr_t)&s_mr[bf][2][0], 4, 0, 0);
        }
    };
    auto publish_meta = [&](int bf) {
        if (wave == W_META) {
            float sq = 0.f;
            if (lane < F) {
                int ri = s_mr[bf][0][lane];
                int rf = fld ? s_mr[bf][1][lane] : lane;
                float rx = val ? __int_as_float(s_mr[bf][2][lane]) : 1.f;
                if (ri < 0 || ri >= P.num_features || rf < 0 || rf >= P.num_fields) { ri = -1; rx = 0.f; rf = 0; }
                s_m[bf][lane] = make_int4(ri, rf, __float_as_int(rx), 0);
                sq = rx * rx;
            }
            const float tot = hm::wave_sum_uniform(sq);
            if (lane == 0) s_red[4 + bf] = (P.norm && tot > 0.f) ? rsqrtf(tot) : 1.f;
        }
    };
    auto slot = [&](int bf, int j, OT& off, float& xab) -> uint32_t {
        const int4 ma = s_m[bf][SA(j)], mb = s_m[bf][SB(j)];
        const bool ok = (ma.x | mb.x) >= 0 && tid + j * 256 < FF;
        const bool live = ok && SA(j) != SB(j);
        off = ok ? (OT)(uint32_t)ma.x * bs + (OT)(uint32_t)mb.y * 12u : (OT)0;
        xab = live ? __int_as_float(ma.z) * __int_as_float(mb.z) : 0.f;
        return live ? 1u : (ok ? 2u : 0u);
    };
    OT koff[KEEP ? NS : 1], noff[KEEP ? NS : 1];
    float kxab[KEEP ? NS : 1], nxab[KEEP ? NS : 1];
    uint32_t klive = 0u, kwr = 0u, nlive = 0u, nwr = 0u;
    int krep = 0, nrep = 0;
    auto dma_slots = [&](int bf) {
        if constexpr (KEEP) { nlive = 0u; nwr = 0u; nrep = 0; }
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            OT off;
            float xab;
            const uint32_t k = slot(bf, j, off, xab);
            if constexpr (KEEP) {
                noff[j] = off;
                nxab[j] = xab;
                nlive |= (k & 1u) << j;
                nwr |= (uint32_t)(k != 0u) << j;
                if (P.defer) nrep |= (int)slot_repeats(SA(j), SB(j), s_m[bf][SA(j)], s_m[bf][SB(j)]);
            }
            __builtin_amdgcn_global_load_lds((glb_ptr_t)(vb + off), (lds_ptr_t)(s_raw + (j * 256 + wave * 64) * 4),
                                             12, 0, 0);
        }
    };
    auto keep_rotate = [&]() {
        if constexpr (KEEP) {
#pragma unroll
            for (int j = 0; j < NS; ++j) { koff[j] = noff[j]; kxab[j] = nxab[j]; }
            klive = nlive; kwr = nwr; krep = nrep;
        }
    };
    auto dma_lin = [&](int bf) {
        if (P.use_linear && wave == W_LIN && lane < F) {
            const int i = s_m[bf][lane].x;
            if (i >= 0 && P.lpack) {
                __builtin_amdgcn_global_load_lds((glb_ptr_t)&LW(w, i), (lds_ptr_t)&s_lin4[bf][0], 16, 0, 0);
                if (LT && nh >= 0)
                    __builtin_amdgcn_global_load_lds((glb_ptr_t)(P.hacc + HACC_STRIDE * nh), (lds_ptr_t)&s_hacc[bf][0], 16, 0, 0);
            } else if (i >= 0) {
                __builtin_amdgcn_global_load_lds((glb_ptr_t)&LW(w, i), (lds_ptr_t)&s_lin[bf][0][0], 4, 0, 0);
                if (P.train) {
                    __builtin_amdgcn_global_load_lds((glb_ptr_t)&LW(wz, i), (lds_ptr_t)&s_lin[bf][1][0], 4, 0, 0);
                    __builtin_amdgcn_global_load_lds((glb_ptr_t)&LW(wn, i), (lds_ptr_t)&s_lin[bf][2][0], 4, 0, 0);
                }
            }
        }
    };

    int row = blockIdx.x;
    if (row >= P.B) return;
    if (tid == 0) { s_bcur[0] = 0.f; s_bcur[1] = 0.f; }
    dma_meta(0, row);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    bar_raw();
    publish_meta(0);
    bar_raw();
    dma_slots(0);
    keep_rotate();
    if constexpr (LT != 0) {
        if (P.hacc_on && wave == W_LIN && lane < F) nh = s_m[0][lane].x >= 0 ? P.hidx[s_m[0][lane].x] : -1;
    }
    dma_lin(0);
    kh = nh;
    dma_meta(1, row + G);

    const bool bsh = P.use_bias && P.bias_sh;
    // A block re-reads the 64 shard lines every bias_every rows (loads of lines the other blocks'
    // atomics keep updating are slow: every row took -w0 from 75 to 40 M rows/s) and adds its own
    // steps since that read (s_bcur) in between; the other blocks' steps arrive with the next read.
    int bit = 0;                    // rows of this block so far
    float bz = 0.f, bn = 0.f;       // the W_META lanes' copy of the shard sums, loaded a row ahead
    if (bsh && wave == W_META && lane < P.bias_s) {
        bz = __hip_atomic_load(P.bias_sh + lane * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bn = __hip_atomic_load(P.bias_sh + lane * 32 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int cur = 0; row < P.B; row += G, cur ^= 1) {
        const int nxt = cur ^ 1;
        const bool more = row + G < P.B;
        __builtin_amdgcn_s_waitcnt(0x0F70);                                     // vmcnt(0)
        bar_raw();
        // the bias shards for the NEXT row (one row of extra staleness on one parameter, as
        // train_fm's w0): issued here, landed by the next phase A's vmcnt(0), used in its D
        // this row re-reads (block-uniform); not the block's first row: the shards were just read
        const bool bre = bsh && bit > 0 && (bit % P.bias_every) == 0;
        float nbz = bz, nbn = bn;
        if (bre && wave == W_META && lane < P.bias_s) {
            nbz = __hip_atomic_load(P.bias_sh + lane * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            nbn = __hip_atomic_load(P.bias_sh + lane * 32 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // ---- B: landing zone -> G registers + transposed V image ----
        if constexpr (LT != 0) {
            // the next row's hot indices (as in ffm_pipe_sg32_kernel; waited for in C)
            if (P.hacc_on && more && wave == W_LIN && lane < F) {
                const int ri = s_mr[nxt][0][lane];
                __builtin_amdgcn_global_load_lds((glb_ptr_t)(P.hidx + (ri >= 0 && ri < P.num_features ? ri : 0)),
                                                 (lds_ptr_t)&s_nh[nxt][0], 4, 0, 0);
            }
        }
        float cg[NS];
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            // one 16-B read per lane (contiguous: conflict-free); separate 4-B and 8-B reads at a
            // 16-B lane stride were 4-way / 2-way bank conflicts
            const uint4 q = *reinterpret_cast<const uint4*>(s_raw + (j * 256 + tid) * 4);
            // q.w is not needed, and without this use the compiler narrows the read back to the
            // conflicting ds_read_b64 + ds_read_b32 pair
            asm volatile("" :: "v"(q.w));
            cg[j] = __uint_as_float(q.z);
            if (tid + j * 256 < FF) s_t[SB(j) * F + SA(j)] = make_uint2(q.x, q.y);
        }
        if (more) publish_meta(nxt);
        bar_raw();
        if (more) {
            dma_slots(nxt);
            dma_meta(cur, row + 2 * G);
        }
        if constexpr (LT != 0) {
            if (P.hacc_on && more && wave == W_LIN) {
                __builtin_amdgcn_s_waitcnt(VMCNT_ENC(NS));   // the B-phase DMA (older than the NS slot DMAs)
                if (lane < F) nh = s_nh[nxt][lane];
            }
        }
        const float scale = s_red[4 + cur];
        int mi = -1;
        float mx = 0.f, lw = 0.f;
        int hot = 0;
        float hz = 0.f, hn = 0.f;
        if (wave == W_LIN && lane < F) {
            const int4 m = s_m[cur][lane];
            mi = m.x;
            mx = __int_as_float(m.z);
            lw = P.lpack ? s_lin4[cur][lane].x : s_lin[cur][0][lane];
            if (latom) lw = lin_w(P, s_lin4[cur][lane]);
            if constexpr (LT != 0) {
                if (P.hacc_on && mi >= 0 && kh >= 0) {
                    const float4 a = s_hacc[cur][lane];
                    const float2 d = s_hd[kh];
                    hz = a.x + d.x;
                    hn = a.y + d.y;
                    hot = 1;
                    lw = hn > 0.f ? ftrl_weight(hz, hn, P.alpha, P.beta, P.lambda1, P.lambda2) : lw;
                }
            }
        }
        // ---- D: forward ----
        uint32_t live = 0u, wr = 0u;
        float xab[NS];
        uint2 kpv[KEEP >= 2 ? NS : 1], kcv[KEEP >= 2 ? NS : 1];
        float part = 0.f;
        int rep = 0;
        if constexpr (KEEP) { live = klive; wr = kwr; rep = krep; }
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            if constexpr (KEEP) {
                xab[j] = kxab[j];
            } else {
                OT off;
                const uint32_t k = slot(cur, j, off, xab[j]);
                live |= (k & 1u) << j;
                wr |= (uint32_t)(k != 0u) << j;
                if (P.defer) rep |= (int)slot_repeats(SA(j), SB(j), s_m[cur][SA(j)], s_m[cur][SB(j)]);
            }
            const int s = tid + j * 256;
            const uint2 pv = s_t[s < FF ? s : 0];
            const uint2 cv = s_t[SB(j) * F + SA(j)];
            if constexpr (KEEP >= 2) { kpv[j] = pv; kcv[j] = cv; }
            part += dot2_bf16(cv.x, pv.x, dot2_bf16(cv.y, pv.y, 0.f)) * xab[j];
        }
        part *= 0.5f * scale * scale;
        part += lw * mx * scale;
        part = hm::wave_sum_uniform(part);
        const int wrep = __any(rep);
        if (bsh && wave == W_META) {
            const float z = hm::wave_sum_uniform(bz) + s_bcur[0], n = hm::wave_sum_uniform(bn) + s_bcur[1];
            if (lane == 0) { s_bias[0] = ftrl_weight(z, n, P.alpha, P.beta, 0.f, 0.f); s_bias[1] = z; s_bias[2] = n; }
        }
        if (lane == 0) { s_red[wave] = part; s_rep[wave] = wrep; }
        bar_raw();
        float p = s_red[0] + s_red[1] + s_red[2] + s_red[3];
        const bool rdup = (s_rep[0] | s_rep[1] | s_rep[2] | s_rep[3]) != 0;
        if (P.use_bias) p += bsh ? s_bias[0] : bias_w0(P, bias);
        const float kappa = row_loss(P, row, p, y, pred_out, loss_out);

        // ---- E: updates (a multi-hot row is deferred to ffm_row_kernel) ----
        // the shards read at this row's B lack only this row's own step (wave 0 waits for its
        // atomics at every phase A, so all earlier ones had landed)
        if (bre && tid == 0) { s_bcur[0] = 0.f; s_bcur[1] = 0.f; }
        if (P.train && rdup && P.defer) {
            defer_row(P, row);
        } else if (P.train) {
            const float ks = kappa * scale * scale;
            uint32_t hrow = (P.seed ^ ((uint32_t)row * 0x85EBCA77u)) + tid_h;
            hrow ^= hrow >> 16;
            hrow *= 0x7FEB352Du;
            hrow ^= hrow >> 15;
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                if (!(wr >> j & 1u)) continue;
                OT off;
                if constexpr (KEEP) {
                    off = koff[j];
                } else {
                    float xj;
                    slot(cur, j, off, xj);
                }
                const int s = tid + j * 256;
                const uint2 pv = KEEP >= 2 ? kpv[j] : s_t[s];
                const uint2 cv = KEEP >= 2 ? kcv[j] : s_t[SB(j) * F + SA(j)];
                const float c = ks * xab[j];
                const float lj = (live >> j & 1u) ? P.lambda_v : 0.f;   // diagonal: zero step
                const f2 cc = {c, c}, ll = {lj, lj};
                f2 o0 = bf2_to_f2(cv.x), o1 = bf2_to_f2(cv.y);
                const f2 p0 = bf2_to_f2(pv.x), p1 = bf2_to_f2(pv.y);
                const f2 d0 = cc * p0 + ll * o0, d1 = cc * p1 + ll * o1;
                const float gs = (((cg[j] + d0.x * d0.x) + d0.y * d0.y) + d1.x * d1.x) + d1.y * d1.y;
                const float r = __builtin_amdgcn_rsqf(gs + P.eps) * -P.eta0;
                const f2 rr = {r, r};
                o0 = o0 + rr * d0;
                o1 = o1 + rr * d1;
                const uint32_t h = rotl32(hrow, 5 * j + 1) ^ (0x9E3779B9u * (uint32_t)(j + 1));
                *reinterpret_cast<u3v*>(vb + off) = u3v{pack_sr_hi(o0, h, rotl32(h, 16)),
                                                        pack_sr_hi(o1, rotl32(h, 8), rotl32(h, 24)),
                                                        __float_as_uint(gs)};
            }
            // pad slots + block tails of the row's features, spread over all threads (here they
            // pay: without them 117.3-117.6 vs 118.1-118.6 M rows/s, profiles/r4/ffm_no_pad_stores_ab.log;
            // the fp32 kernel is faster without)
            {
                const int npad = P.vpad - P.num_fields;
                const int per = npad + P.tail16;
                for (int q = tid; q < F * per; q += 256) {
                    const int a = q / per, kk = q - a * per;
                    const int i = s_m[cur][a].x;
                    if (i < 0) continue;
                    char* blk = vb + (OT)(uint32_t)i * bs;
                    if (kk < npad) *reinterpret_cast<u3v*>(blk + (P.num_fields + kk) * 12) = u3v{0u, 0u, 0u};
                    else if (!(lin_in_tail && kk == npad))   // the first tail chunk holds {w, z, n}
                        *reinterpret_cast<uint4*>(blk + P.vpad * 12 + 16 * (kk - npad)) = make_uint4(0u, 0u, 0u, 0u);
                }
            }
            if (mi >= 0 && P.use_linear) {   // FTRL-proximal on the DMA'd (w, z, n)
                const float lz = hot ? hz : (P.lpack ? s_lin4[cur][lane].y : s_lin[cur][1][lane]);
                const float ln = hot ? hn : (P.lpack ? s_lin4[cur][lane].z : s_lin[cur][2][lane]);
                const float g = kappa * mx * scale;
                const float n1 = ln + g * g;
                const float z1 = lz + g - (sqrtf(n1) - sqrtf(ln)) / P.alpha * lw;
                const float w1 = ftrl_weight(z1, n1, P.alpha, P.beta, P.lambda1, P.lambda2);
                if (LT && hot) {
                    const float2 d = s_hd[kh];
                    s_hd[kh] = make_float2(d.x + (g - (sqrtf(n1) - sqrtf(ln)) / P.alpha * lw), d.y + g * g);
                } else if (latom) {
                    lin_add(P, w, mi, g, ln, n1, lw);
                } else if (P.lpack) {
                    *reinterpret_cast<float4*>(&LW(w, mi)) = make_float4(w1, z1, n1, 0.f);
                } else {
                    LW(wz, mi) = z1;
                    LW(wn, mi) = n1;
                    LW(w, mi) = w1;
                }
            }
            if (P.use_bias && tid == 0) {
                if (bsh) bias_update_sh(P, kappa, s_bias[1], s_bias[2], P.bias_sh + (blockIdx.x % P.bias_s) * 32, s_bcur);
                else bias_update(P, kappa, bias);
            }
        }
        if (more) dma_lin(nxt);
        kh = nh;
        keep_rotate();
        bz = nbz;
        bn = nbn;
        ++bit;
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);       // no LDS-DMA outstanding at exit
    if constexpr (LT != 0) {
        bar_raw();   // (as in ffm_pipe_sg32_kernel)
        if (P.hacc_on)
            for (int t = tid; t < 2 * P.nhot; t += 256) {
                const float2 d = s_hd[t >> 1];
                if (d.y != 0.f || d.x != 0.f) atomicAdd(P.hacc + HACC_STRIDE * (t >> 1) + (t & 1), (t & 1) ? d.y : d.x);
            }
    }
#undef SA
#undef SB
}


// 8,192 blocks (8 per CU, 4 resident at a time) unless the batch is smaller or a grid is given.
// The bf16 12-B-slot kernel takes 16,384 (16 rows per block at the bench batch).  Round 3 measured
// 32,768 best (+1.5 %, profiles/ffm_r3/grid_sweep_*.log); with the linear records in the feature
// blocks 8-16 K lead: 129.5-129.8 M rows/s vs 127.6 M at 32 K (profiles/r5/bench_grid_sweep_linrec.log;
// the fp32 kernel is flat from 2 K to 16 K, logloss unchanged for both).
int default_blocks(int B, int grid, int cap = 256 * 8 * 4) {
    return grid > 0 ? grid : (B < cap ? B : cap);
}

// Per-element pipelined / lean dispatch (Kp == 4, packed, table < 4 GiB, F*F <= 2048); -1 when
// the shape needs the generic kernel.
template <bool BF>
int dispatch_lean(const FFMParams& P, const int32_t* idx, const int32_t* fld, const float* val,
                  const float* y, void* VG, float* w, float* wz, float* wn, float* bias,
                  float* pred, float* loss, int grid, int variant, hipStream_t stream) {
    const size_t slot_b = BF ? 16 : 32;
    if (P.Kp != 4 || P.F > 45) return -1;
    if ((size_t)P.num_features * (size_t)P.fstride * slot_b >= ((size_t)1 << 32)) return -1;
    const size_t meta = (size_t)P.F * 16 + 16 * 4;
    const size_t sh = (size_t)P.F * P.F * (BF ? 8 : 16) + meta;
    const int need = (P.F * P.F + 255) / 256;
    const int blocks = default_blocks(P.B, grid);
    if (blocks <= 0) return 0;
    // bf16: the LDS-DMA pipeline unless variant 2; fp32: the lean kernel unless variant 3
    // (measured same-box, profiles/ffm_r2/fp32_pipe_ab.log: 52.5 M rows/s vs 51.2 M (+2.6 %),
    // while the pipeline's extra row of staleness cost held-out logloss at 500 K rows: +0.019 vs
    // sequential, lean +0.010)
    if ((BF && variant != 2) || (!BF && variant == 3)) {
#define HM_PIPE(NSV) hipLaunchKernelGGL((ffm_pipe_kernel<NSV, BF>), dim3(blocks), dim3(256), 0, stream, P, idx, \
                                        fld, val, y, VG, w, wz, wn, bias, pred, loss)
        if (need <= 2) { HM_PIPE(2); }
        else if (need <= 4) { HM_PIPE(4); }
        else if (need <= 6) { HM_PIPE(6); }
        else { HM_PIPE(8); }
#undef HM_PIPE
        HM_LAUNCH_RET();
    }
#define HM_LEAN(NSV)                                                                                \
    hipLaunchKernelGGL((ffm_lean_kernel<BF, NSV>), dim3(blocks), dim3(256), sh, stream, P, idx, fld, \
                       val, y, VG, w, wz, wn, bias, pred, loss)
    if (need <= 2) HM_LEAN(2);
    else if (need <= 4) HM_LEAN(4);
    else if (need <= 6) HM_LEAN(6);
    else HM_LEAN(8);
#undef HM_LEAN
    HM_LAUNCH_RET();
}

// lin_atomic 4: dir 0 copies the hot features' (z, n) from their records into the side table
// before a launch, dir 1 writes them back (w = f(z, n)) after it.
__global__ __launch_bounds__(256) void ffm_hacc_kernel(FFMParams P, float* __restrict__ w, int dir) {
    const int h = blockIdx.x * 256 + threadIdx.x;
    if (h >= P.nhot) return;
    float4* rp = reinterpret_cast<float4*>(&LW(w, P.hot_id[h]));
    float4* ap = reinterpret_cast<float4*>(P.hacc + HACC_STRIDE * h);
    const float4 r = *rp;
    if (dir == 0) {
        *ap = make_float4(r.y, r.z, 0.f, 0.f);
    } else {
        const float4 a = *ap;
        const float nw = a.y > 0.f ? ftrl_weight(a.x, a.y, P.alpha, P.beta, P.lambda1, P.lambda2) : r.x;
        *rp = make_float4(nw, a.x, a.y, r.w);
    }
}

// lin_atomic: w <- f(z, n) for every feature record a row stepped (n > 0; a record never stepped
// keeps its w, e.g. an imported model's).
__global__ __launch_bounds__(256) void ffm_lin_derive_kernel(FFMParams P, float* __restrict__ w) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P.num_features) return;
    const float4 r = *reinterpret_cast<const float4*>(&LW(w, i));
    if (r.z > 0.f) LW(w, i) = ftrl_weight(r.y, r.z, P.alpha, P.beta, P.lambda1, P.lambda2);
}

// Per-slot-G in 12-B bf16 slots {V | G}, 512-B feature blocks (Kp == 4, F <= 45, table < 4 GiB).
int dispatch_sg12(const FFMParams& P, const int32_t* idx, const int32_t* fld, const float* val,
                  const float* y, void* VG, float* w, float* wz, float* wn, float* bias,
                  float* pred, float* loss, int grid, int variant, hipStream_t stream) {
    if (P.Kp != 4 || P.F > 45) return -1;
    // tables of 4 GiB and more (-feature_hashing >= 23 at 512-B blocks): 64-bit slot offsets
    const bool wide = (size_t)P.num_features * (size_t)P.gstride * 4 >= ((size_t)1 << 32);
    const int need = (P.F * P.F + 255) / 256;
    int blocks = default_blocks(P.B, grid, 256 * 8 * 8);
    if (blocks <= 0) return 0;
    FFMParams Q = P;
    Q.hacc_on = P.lin_atomic == 4 && P.nhot <= HD12_SIZE && blocks > 1 && !wide && variant != 9 && variant != 10;
    if (Q.hacc_on && grid <= 0) blocks = default_blocks(P.B, grid, HACC_GRID12);
    if (Q.hacc_on) {
        hipLaunchKernelGGL(ffm_hacc_kernel, dim3((P.nhot + 255) / 256), dim3(256), 0, stream, Q, w, 0);
        HM_LAUNCH_RET_IF_ERR();
    }
#define HM_P12(NSV) do { \
        if (wide) hipLaunchKernelGGL((ffm_pipe_sg12_kernel<NSV, uint64_t>), dim3(blocks), dim3(256), 0, stream, \
                                     P, idx, fld, val, y, VG, w, wz, wn, bias, pred, loss); \
        else if (Q.hacc_on) hipLaunchKernelGGL((ffm_pipe_sg12_kernel<NSV, uint32_t, 2, 1>), dim3(blocks), dim3(256), 0, \
                                               stream, Q, idx, fld, val, y, VG, w, wz, wn, bias, pred, loss); \
        else if (variant == 9) hipLaunchKernelGGL((ffm_pipe_sg12_kernel<NSV, uint32_t>), dim3(blocks), dim3(256), 0, \
                                                  stream, P, idx, fld, val, y, VG, w, wz, wn, bias, pred, loss); \
        else if (variant == 10) hipLaunchKernelGGL((ffm_pipe_sg12_kernel<NSV, uint32_t, 1>), dim3(blocks), dim3(256), 0, \
                                                   stream, P, idx, fld, val, y, VG, w, wz, wn, bias, pred, loss); \
        else hipLaunchKernelGGL((ffm_pipe_sg12_kernel<NSV, uint32_t, 2>), dim3(blocks), dim3(256), 0, stream, \
                                P, idx, fld, val, y, VG, w, wz, wn, bias, pred, loss); } while (0)
    if (need <= 2) { HM_P12(2); }
    else if (need <= 4) { HM_P12(4); }
    else if (need <= 6) { HM_P12(6); }
    else { HM_P12(8); }
#undef HM_P12
    if (Q.hacc_on) {
        HM_LAUNCH_RET_IF_ERR();
        hipLaunchKernelGGL(ffm_hacc_kernel, dim3((P.nhot + 255) / 256), dim3(256), 0, stream, Q, w, 1);
    }
    HM_LAUNCH_RET();
}

// Per-slot-G fp32 pipelined dispatch (Kp == 4 or 8, F <= 45, block layout, tables < 4 GiB): the
// LDS-DMA ffm_pipe_sg32_kernel; -1 otherwise (bf16 V in this layout: the generic kernel; the
// bf16 default is the 12-B slot layout of dispatch_sg12).
int dispatch_sg32(const FFMParams& P, const int32_t* idx, const int32_t* fld, const float* val,
                  const float* y, void* V, float* G, float* w, float* wz, float* wn, float* bias,
                  float* pred, float* loss, int grid, int variant, hipStream_t stream) {
    if ((P.Kp != 4 && P.Kp != 8) || P.F > 45 || P.vpad <= 0) return -1;
    // tables of 4 GiB and more (-feature_hashing >= 23 at 896-B blocks): 64-bit slot offsets
    const bool wide = (size_t)P.num_features * (size_t)P.fstride * (size_t)(P.Kp * 4) >= ((size_t)1 << 32) ||
                      (size_t)P.num_features * (size_t)P.gstride * 4 >= ((size_t)1 << 32);
    if (P.Kp == 8) {
        // 32-B slots: 512-thread blocks, one per CU (107 KB of LDS at 39 fields)
        if (variant == 8) return -1;
        const int need = (P.F * P.F + 511) / 512;
        int blocks = default_blocks(P.B, grid);
        if (blocks <= 0) return 0;
        // lin_atomic 4 as for k = 4 below (the 16 KB of block sums still leave one block per CU)
        FFMParams Q = P;
        Q.hacc_on = P.lin_atomic == 4 && blocks > 1 && !wide && variant != 6 && variant != 9;
        if (Q.hacc_on && grid <= 0) blocks = default_blocks(P.B, grid, HACC_GRID);
        if (Q.hacc_on) {
            hipLaunchKernelGGL(ffm_hacc_kernel, dim3((P.nhot + 255) / 256), dim3(256), 0, stream, Q, w, 0);
            HM_LAUNCH_RET_IF_ERR();
        }
#define HM_P32K8(NSV) do { \
        if (wide) hipLaunchKernelGGL((ffm_pipe_sg32_kernel<NSV, uint64_t, 512, 0, 2>), dim3(blocks), dim3(512), 0, stream, \
                                     P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss); \
        else if (Q.hacc_on) hipLaunchKernelGGL((ffm_pipe_sg32_kernel<NSV, uint32_t, 512, 0, 2, 1, 1>), dim3(blocks), \
                                               dim3(512), 0, stream, Q, idx, fld, val, y, V, G, w, wz, wn, \
                                               bias, pred, loss); \
        else if (variant == 6) hipLaunchKernelGGL((ffm_pipe_sg32_kernel<NSV, uint32_t, 512, 1, 2>), dim3(blocks), \
                                                  dim3(512), 0, stream, P, idx, fld, val, y, V, G, w, wz, wn, \
                                                  bias, pred, loss); \
        else if (variant == 9) hipLaunchKernelGGL((ffm_pipe_sg32_kernel<NSV, uint32_t, 512, 0, 2>), dim3(blocks), \
                                                  dim3(512), 0, stream, P, idx, fld, val, y, V, G, w, wz, wn, \
                                                  bias, pred, loss); \
        else hipLaunchKernelGGL((ffm_pipe_sg32_kernel<NSV, uint32_t, 512, 0, 2, 1>), dim3(blocks), dim3(512), 0, stream, \
                                P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss); } while (0)
        if (need <= 2) { HM_P32K8(2); }
        else if (need <= 3) { HM_P32K8(3); }
        else { HM_P32K8(4); }
#undef HM_P32K8
        if (Q.hacc_on) {
            HM_LAUNCH_RET_IF_ERR();
            hipLaunchKernelGGL(ffm_hacc_kernel, dim3((P.nhot + 255) / 256), dim3(256), 0, stream, Q, w, 1);
        }
        HM_LAUNCH_RET();
    }
    const int need = (P.F * P.F + 255) / 256;
    int blocks = default_blocks(P.B, grid);
    if (blocks <= 0) return 0;
    // lin_atomic 4: the side table for a launch of more than one block (one block stores the
    // records in row order: the sequential engine)
    FFMParams Q = P;
    Q.hacc_on = P.lin_atomic == 4 && blocks > 1 && !wide && variant != 6 && variant != 8 && variant != 9 && variant != 10;
    if (Q.hacc_on && grid <= 0) blocks = default_blocks(P.B, grid, HACC_GRID);
    if (Q.hacc_on) {
        hipLaunchKernelGGL(ffm_hacc_kernel, dim3((P.nhot + 255) / 256), dim3(256), 0, stream, Q, w, 0);
        HM_LAUNCH_RET_IF_ERR();
    }
#define HM_P32(NSV) do { \
        if (wide) hipLaunchKernelGGL((ffm_pipe_sg32_kernel<NSV, uint64_t>), dim3(blocks), dim3(256), 0, stream, \
                                     P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss); \
        else if (variant == 6) hipLaunchKernelGGL((ffm_pipe_sg32_kernel<NSV, uint32_t, 256, 1>), dim3(blocks), \
                                                  dim3(256), 0, stream, P, idx, fld, val, y, V, G, w, wz, wn, \
                                                  bias, pred, loss); \
        else if (variant == 8 && P.hot) hipLaunchKernelGGL((ffm_pipe_sg32_kernel<NSV, uint32_t, 256, 2>), dim3(blocks), \
                                                  dim3(256), 0, stream, P, idx, fld, val, y, V, G, w, wz, wn, \
                                                  bias, pred, loss); \
        else if (variant == 9) hipLaunchKernelGGL((ffm_pipe_sg32_kernel<NSV, uint32_t>), dim3(blocks), dim3(256), 0, \
                                                  stream, P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss); \
        else if (variant == 10) hipLaunchKernelGGL((ffm_pipe_sg32_kernel<NSV, uint32_t, 256, 0, 1, 1>), dim3(blocks), \
                                                   dim3(256), 0, stream, P, idx, fld, val, y, V, G, w, wz, wn, \
                                                   bias, pred, loss); \
        else if (Q.hacc_on) hipLaunchKernelGGL((ffm_pipe_sg32_kernel<NSV, uint32_t, 256, 0, 1, 2, 1>), dim3(blocks), \
                                               dim3(256), 0, stream, Q, idx, fld, val, y, V, G, w, wz, wn, \
                                               bias, pred, loss); \
        else hipLaunchKernelGGL((ffm_pipe_sg32_kernel<NSV, uint32_t, 256, 0, 1, 2>), dim3(blocks), dim3(256), 0, stream, \
                                P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss); } while (0)
    if (need <= 2) { HM_P32(2); }
    else if (need <= 4) { HM_P32(4); }
    else if (need <= 6) { HM_P32(6); }
    else { HM_P32(8); }
#undef HM_P32
    if (Q.hacc_on) {
        HM_LAUNCH_RET_IF_ERR();
        hipLaunchKernelGGL(ffm_hacc_kernel, dim3((P.nhot + 255) / 256), dim3(256), 0, stream, Q, w, 1);
    }
    HM_LAUNCH_RET();
}

template <int KC, bool BF, bool SG>
int launch_ffm(const FFMParams& P, const int32_t* idx, const int32_t* fld, const float* val,
               const float* y, void* V, void* G, float* w, float* wz, float* wn, float* bias,
               float* pred, float* loss, int grid, hipStream_t stream) {
    const size_t meta = (size_t)6 * P.F * 4 + 16 * 4;
    const size_t stage = (size_t)P.F * P.F * KC * (BF ? 8 : 16);
    const bool use_stage = stage + meta <= 64 * 1024;
    const int blocks = default_blocks(P.B, grid);
    if (blocks <= 0) return 0;
    if (use_stage) {
        hipLaunchKernelGGL((ffm_row_kernel<KC, true, BF, SG>), dim3(blocks), dim3(256), stage + meta, stream,
                           P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss);
    } else {
        hipLaunchKernelGGL((ffm_row_kernel<KC, false, BF, SG>), dim3(blocks), dim3(256), meta, stream,
                           P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss);
    }
    HM_LAUNCH_RET();
}

template <bool BF, bool SG>
int launch_generic(const FFMParams& P, const int32_t* idx, const int32_t* fld, const float* val,
                   const float* y, void* V, void* G, float* w, float* wz, float* wn, float* bias,
                   float* pred, float* loss, int grid, hipStream_t stream) {
    switch (P.Kp / 4) {
        case 1: return launch_ffm<1, BF, SG>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
        case 2: return launch_ffm<2, BF, SG>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
        case 3: return launch_ffm<3, BF, SG>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
        case 4: return launch_ffm<4, BF, SG>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
        case 8: return launch_ffm<8, BF, SG>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
        default: return (int)hipErrorInvalidValue;
    }
}

// *fast = 1 when a pipelined / lean kernel ran (it defers multi-hot rows when P.defer is set).
template <bool BF>
int dispatch(const FFMParams& P, const int32_t* idx, const int32_t* fld, const float* val,
             const float* y, void* V, void* G, float* w, float* wz, float* wn, float* bias,
             float* pred, float* loss, int grid, int packed, int slot_g, int variant, hipStream_t stream,
             int* fast) {
    *fast = 1;
    if (slot_g) {
        if (P.gfstride == 3) {
            // 12-B {V | G} slots: the pipelined kernel; rows wider than 45 features or tables of
            // 4 GiB and more (32-bit offsets there) take the generic kernel with 64-bit offsets
            // (slot stride 6 bf16, feature stride = the block)
            if (!BF) return (int)hipErrorInvalidValue;
            const int rc = variant == 1 ? -1 : dispatch_sg12(P, idx, fld, val, y, V, w, wz, wn, bias, pred, loss, grid, variant, stream);
            if (rc != -1) return rc;
            *fast = 0;
            return launch_generic<true, true>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
        }
        if (variant != 1 && !BF && P.gfstride == 1) {
            const int rc = dispatch_sg32(P, idx, fld, val, y, V, reinterpret_cast<float*>(G), w, wz, wn,
                                         bias, pred, loss, grid, variant, stream);
            if (rc != -1) return rc;
        }
        *fast = 0;
        return launch_generic<BF, true>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
    }
    if (packed && variant != 1) {
        const int rc = dispatch_lean<BF>(P, idx, fld, val, y, V, w, wz, wn, bias, pred, loss, grid, variant, stream);
        if (rc != -1) return rc;
        // other shapes: the generic kernel handles the packed strides too (G = V + Kp)
    }
    *fast = 0;
    return launch_generic<BF, false>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
}

// The deferred multi-hot rows of a pipelined launch: ffm_row_kernel over the list (grid of
// DEFER_BLOCKS blocks; each exits at once when the count is 0).
constexpr int DEFER_BLOCKS = 512;

template <bool BF>
int launch_deferred(FFMParams P, const int32_t* idx, const int32_t* fld, const float* val,
                    const float* y, void* V, void* G, float* w, float* wz, float* wn, float* bias,
                    float* pred, float* loss, int slot_g, int grid_req, hipStream_t stream) {
    P.list_mode = 1;
    // an explicit grid bounds the deferred rows' concurrency too (grid = 1: one block trains
    // them in list order, after the batch's other rows)
    const int cap = grid_req > 0 && grid_req < DEFER_BLOCKS ? grid_req : DEFER_BLOCKS;
    const int grid = P.B < cap ? P.B : cap;
    return slot_g ? launch_generic<BF, true>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream)
                  : launch_generic<BF, false>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
}

}  // namespace

// hp layout (floats): eta0, eps, lambda_v, alpha, beta, lambda1, lambda2, min_target, max_target
// ip layout (ints)  : B, F, num_features, num_fields, Kp, classification, train, use_linear,
//                     use_bias, norm, grid, reload, bf16_state, seed, packed, variant, fstride,
//                     slot_g, gstride, vpad, tail16, gfstride, lin_defer, bias_every, lstride, lpack,
//                     lin_atomic
// lstride = floats between consecutive features' w / wz / wn (1: separate arrays; the records of
//           ops/ffm.py lin_record_views: the feature block's size); lpack = 1: {w, z, n} are one
//           16-B record (wz = w + 1, wn = w + 2), DMA'd and stored as one 16-B access
// slot_g = 1: one fp32 AdaGrad accumulator per (feature, field) slot, G[i * gstride + f * gfstride];
//             bf16 V in 12-B slots {V | G} (G = V + 8 B, gfstride 3): ffm_pipe_sg12_kernel; fp32 V
//             in the block layout (G = V + vpad * Kp * 4 B, vpad > 0): ffm_pipe_sg32_kernel (Kp 4:
//             256-thread blocks; Kp 8: 32-B slots, 512-thread blocks; F <= 45); anything else the
//             generic kernel.  tail16 = zero 16-B chunks after each
//             feature's G region (line completion).
// slot_g = 0 (per-element G shaped like V): packed = 1: V and G are the two halves of one
//             [num_features][fstride][2][Kp] table (G == V + Kp elements, slot stride 2*Kp); 0:
//             separate [.][.][Kp] tables.
// variant (A/B): 0 = auto (per-slot: the sg12 / sg32 pipelines; per-element bf16:
// ffm_pipe_kernel, fp32: ffm_lean_kernel), 1 = the generic ffm_row_kernel, 2 = ffm_lean_kernel
// for bf16, 3 = ffm_pipe_kernel for fp32 (per-element G), 6 = ffm_pipe_sg32_kernel with every
// slot update added by float atomics (no lost update; the learner's early-training ramp,
// models/ffm.py RAMP_*; G-only atomics were measured as variant 7 and removed: the full gap at
// 12 M rows/s, profiles/r4/ffm_g_atomic_bench_ab.log).  Measured and removed: 512-thread sg32
// blocks (75.7-76.1 vs 75.6 M rows/s, profiles/r4/ffm_512_thread_ab.log); a paired-slot sg32
// kernel holding each (a, b) / (b, a) slot pair in one thread's registers instead of a transposed
// LDS image (4 rows in flight per CU instead of 2): 58.1-58.4 vs 74.9-75.5 M rows/s — the (b, a)
// halves of a wave's pairs are V[i_b][f_a] for 64 different features, 16-B loads from 64
// feature blocks where the row-major order reads whole runs of one block
// (profiles/r4/ffm_paired_slots_ab.log); the sg32 kernel with the next row's G prefetched into
// registers instead of an LDS landing zone (53 KB per block: 3 rows in flight per CU instead of
// 2): 73.6-73.8 vs 73.9-74.2 M rows/s (profiles/r4/ffm_register_g_ab.log) — more rows in flight
// per CU does not move this kernel.  Round 5 re-tried it after the linear records (53.4 KB of LDS
// with the 4-B linear zone aliased onto the 16-B one, forced to 3 waves per SIMD): 168 VGPRs with
// 21 spilled, 63.2 vs 89.6 M rows/s (profiles/r5/bench_rg_ab.log).
// aux (host array of 4 pointer-sized entries, or null): aux[0] = per-feature hot flags (variant 8)
// or null; aux[1] = the multi-hot deferral buffer int32 [1 + B] or null (then a multi-hot row is
// updated slot by slot by the pipelined kernels: racing stores of one address, one wins);
// aux[2] = the global-bias shards fp32 [S][32] (training with -w0) or null; aux[3] = S, the
// shard count (1 .. 64), as an integer.
// Measured and removed in round 5 (docs/perf_notes.md "where the fp32 same-stream gap comes
// from"): reload-delta stores, SC1 DMA loads, write-through (device-scope) stores, agent / system
// acquires, a coherent re-read, 512-thread and one-block-per-CU launches, one table replica per
// XCD, and the one-XCD probe switch.
HM_API int hm_ffm_step(const int32_t* ip, const float* hp, const int32_t* idx, const int32_t* fld,
                       const float* val, const float* y, void* V, void* G, float* w, float* wz,
                       float* wn, float* bias, float* pred, float* loss, void* const* aux,
                       hipStream_t stream) {
    FFMParams P;
    P.hot = aux ? reinterpret_cast<const uint8_t*>(aux[0]) : nullptr;
    P.defer = aux ? reinterpret_cast<int32_t*>(aux[1]) : nullptr;
    P.list_mode = 0;
    P.B = ip[0]; P.F = ip[1]; P.num_features = ip[2]; P.num_fields = ip[3]; P.Kp = ip[4];
    P.classification = ip[5]; P.train = ip[6]; P.use_linear = ip[7]; P.use_bias = ip[8];
    P.norm = ip[9];
    const int grid = ip[10];
    P.reload = ip[11];
    const int bf16 = ip[12];
    P.seed = (uint32_t)ip[13];
    const int packed = ip[14];
    const int variant = ip[15];
    P.sstride = packed ? 2 * P.Kp : P.Kp;
    P.fstride = ip[16] > 0 ? ip[16] : P.num_fields;
    const int slot_g = ip[17];
    P.gstride = ip[18];
    P.vpad = ip[19];
    P.tail16 = ip[20];
    P.gfstride = ip[21] > 0 ? ip[21] : 1;
    P.lin_defer = ip[22];
    P.lstride = ip[24] > 0 ? ip[24] : 1;
    P.lpack = ip[25];
    P.lin_atomic = P.lpack ? ip[26] : 0;
    P.hidx = nullptr; P.hot_id = nullptr; P.hacc = nullptr; P.nhot = 0; P.hacc_on = 0;

    if (P.lin_atomic == 4) {
        // aux[4..6] = hidx, hot_id, hacc; ip[27] = nhot
        P.nhot = ip[27];
        if (aux) {
            P.hidx = reinterpret_cast<const int32_t*>(aux[4]);
            P.hot_id = reinterpret_cast<const int32_t*>(aux[5]);
            P.hacc = reinterpret_cast<float*>(aux[6]);
        }
        if (!P.hidx || !P.hot_id || !P.hacc || P.nhot <= 0 || P.nhot > HD_SIZE || !P.train || !P.use_linear)
            P.lin_atomic = 0;
    }
    if (P.lpack && (wz != w + 1 || wn != w + 2 || (P.lstride & 3) || (reinterpret_cast<uintptr_t>(w) & 15)))
        return (int)hipErrorInvalidValue;
    P.bias_sh = aux ? reinterpret_cast<float*>(aux[2]) : nullptr;
    P.bias_s = aux ? (int)reinterpret_cast<intptr_t>(aux[3]) : 0;
    if (!P.bias_sh || P.bias_s < 1 || P.bias_s > 64 || !P.train) { P.bias_sh = nullptr; P.bias_s = 0; }
    P.bias_every = ip[23] > 0 ? ip[23] : 16;
    if (P.fstride < P.num_fields) return (int)hipErrorInvalidValue;
    P.vfe = (long long)P.fstride * P.sstride;
    P.eta0 = hp[0]; P.eps = hp[1]; P.lambda_v = hp[2]; P.alpha = hp[3]; P.beta = hp[4];
    P.lambda1 = hp[5]; P.lambda2 = hp[6]; P.min_target = hp[7]; P.max_target = hp[8];
    if (P.F <= 0 || P.F > 256 || (P.Kp & 3)) return (int)hipErrorInvalidValue;
    if (slot_g) {
        if (packed || P.gstride < P.num_fields || P.tail16 < 0) return (int)hipErrorInvalidValue;
        if (P.gfstride == 3) {
            // 12-B {V | G} slots: G = V + 8 B, vpad slots of 12 B then a zero tail per block
            if (!bf16 || P.Kp != 4 || reinterpret_cast<char*>(G) != reinterpret_cast<char*>(V) + 8 ||
                P.vpad < P.num_fields || (size_t)P.vpad * 12 + (size_t)P.tail16 * 16 != (size_t)P.gstride * 4)
                return (int)hipErrorInvalidValue;
            P.sstride = 6;                           // bf16 elements per 12-B slot
            P.vfe = (long long)P.gstride * 2;        // bf16 elements per feature block
        } else if (P.vpad > 0) {
            // block layout: G right after the V region of the same feature block
            const size_t es = bf16 ? 2 : 4;
            if (reinterpret_cast<char*>(G) != reinterpret_cast<char*>(V) + (size_t)P.vpad * P.Kp * es ||
                (size_t)P.fstride * P.Kp * es != (size_t)P.gstride * 4 || P.vpad < P.num_fields ||
                P.gfstride != 1)
                return (int)hipErrorInvalidValue;
        }
    } else if (packed) {
        // G must be the second half of every packed slot
        const size_t es = bf16 ? 2 : 4;
        if (reinterpret_cast<char*>(G) != reinterpret_cast<char*>(V) + (size_t)P.Kp * es)
            return (int)hipErrorInvalidValue;
        // 32-bit slot indices in the packed kernel
        if ((size_t)P.num_features * (size_t)P.fstride >= ((size_t)1 << 32)) return (int)hipErrorInvalidValue;
    }
    if (!P.train || P.B <= 0) P.defer = nullptr;
    if (P.defer) {
        const hipError_t e = hipMemsetAsync(P.defer, 0, sizeof(int32_t), stream);
        if (e != hipSuccess) return (int)e;
    }
    int fast = 0;
    const int rc = bf16 ? dispatch<true>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, packed, slot_g, variant, stream, &fast)
                        : dispatch<false>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, packed, slot_g, variant, stream, &fast);
    if (rc != 0) return rc;
    if (fast && P.train && P.use_linear && P.lin_atomic == 1) {
        // the stored w of every record a row stepped: w = f(z, n) (before the deferred rows, whose
        // generic kernel reads w)
        hipLaunchKernelGGL(ffm_lin_derive_kernel, dim3((P.num_features + 255) / 256), dim3(256), 0, stream, P, w);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    if (!fast || !P.defer) return rc;
    return bf16 ? launch_deferred<true>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, slot_g, grid, stream)
                : launch_deferred<false>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, slot_g, grid, stream);
}
