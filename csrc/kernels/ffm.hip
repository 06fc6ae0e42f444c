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
//   * V, G   : [num_features][num_fields][Kp], Kp = K rounded up to 4 (padding stays 0).
//              Stored fp32, or bf16 (BF = true, ``-bf16_state``) with stochastic rounding on
//              every write: the kernel is HBM-bound (~95 KB of V/G traffic per Criteo row in
//              fp32), so halving the state bytes is the throughput lever; stochastic rounding
//              keeps the sub-ulp AdaGrad steps and G increments unbiased.
//   * batch  : padded-ELL [B][F] (idx, fld, val), idx < 0 marks padding.
//   * One 256-thread block per row (grid-stride over rows).  Ordered slot s = a*F + b owns
//     the vector V[i_a, f_b]; consecutive threads read consecutive slot vectors of the same
//     feature block, so every gather is coalesced.  The row's F*F*Kp slot vectors are staged
//     in LDS as fp32 (24 KB at F=39, K=4) so the partner read for the pair dot and for the
//     gradient never goes back to L2.
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
    uint32_t seed;
    float eta0, eps, lambda_v;
    float alpha, beta, lambda1, lambda2;
    float min_target, max_target;  // regression clipping of the prediction
};

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

__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ c * 0xC2B2AE3Du;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    return h;
}

__device__ __forceinline__ uint32_t bf16_sr(float f, uint32_t rnd) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7F800000u) == 0x7F800000u) return u >> 16;
    return (u + (rnd & 0xFFFFu)) >> 16;
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
        const uint32_t lo = bf16_sr(v.x, rnd) | (bf16_sr(v.y, rnd >> 16) << 16);
        const uint32_t hi = bf16_sr(v.z, r2) | (bf16_sr(v.w, r2 >> 16) << 16);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(base) + off) = make_uint2(lo, hi);
    } else {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(base) + off) = v;
    }
}

template <int KC, bool STAGE, bool BF>
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
    float* s_red = s_x + F;                                              // 16 (+pad)

    const int tid = threadIdx.x;
    const int Kp = P.Kp;
    const size_t fstride = (size_t)P.num_fields * Kp;  // elements per feature block

    for (int row = blockIdx.x; row < P.B; row += gridDim.x) {
        // ---- 1. row metadata -> LDS (+ instance-wise L2 normalisation) ----
        float sq = 0.f;
        if (tid < F) {
            const size_t o = (size_t)row * F + tid;
            int i = idx[o];
            int f = fld ? fld[o] : tid;
            float x = val ? val[o] : 1.f;
            if (i < 0 || i >= P.num_features || f < 0 || f >= P.num_fields) { i = -1; x = 0.f; }
            s_idx[tid] = i;
            s_fld[tid] = f < 0 ? 0 : (f >= P.num_fields ? P.num_fields - 1 : f);
            s_x[tid] = x;
            sq = x * x;
        }
        float scale = 1.f;
        if (P.norm) {
            const float tot = hm::block_sum(sq, s_red);
            scale = tot > 0.f ? rsqrtf(tot) : 1.f;
        } else {
            __syncthreads();
        }

        // ---- 2. gather the row's slot vectors (coalesced) ----
        if (STAGE) {
            for (int s = tid; s < FF; s += blockDim.x) {
                const int a = s / F, b = s - (s / F) * F;
                const int ia = s_idx[a];
                const bool live = a != b && ia >= 0 && s_idx[b] >= 0;
                const size_t off = live ? (size_t)ia * fstride + (size_t)s_fld[b] * Kp : 0;
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
                const size_t ou = (size_t)ia * fstride + (size_t)s_fld[b] * Kp;
                const size_t ov = (size_t)ib * fstride + (size_t)s_fld[a] * Kp;
#pragma unroll
                for (int c = 0; c < KC; ++c) { u[c] = ld_chunk<BF>(V, ou + 4 * c); v[c] = ld_chunk<BF>(V, ov + 4 * c); }
            }
            float d = 0.f;
#pragma unroll
            for (int c = 0; c < KC; ++c) d += u[c].x * v[c].x + u[c].y * v[c].y + u[c].z * v[c].z + u[c].w * v[c].w;
            part += d * s_x[a] * s_x[b];
        }
        part *= scale * scale;
        if (P.use_linear && tid < F && s_idx[tid] >= 0) part += w[s_idx[tid]] * s_x[tid] * scale;
        float p = hm::block_sum(part, s_red);
        if (P.use_bias) p += bias[0];

        // ---- 4. loss ----
        const float yy = y ? y[row] : 0.f;
        float kappa;
        if (P.classification) {
            const float e = yy * p;
            kappa = -yy / (1.f + __expf(e));
            if (tid == 0) {
                if (loss_out) loss_out[row] = hm::log1pexp(-e);
                if (pred_out) pred_out[row] = p;
            }
        } else {
            const float pc = fminf(fmaxf(p, P.min_target), P.max_target);
            kappa = pc - yy;
            if (tid == 0) {
                if (loss_out) loss_out[row] = 0.5f * kappa * kappa;
                if (pred_out) pred_out[row] = pc;
            }
        }

        // ---- 5. updates (Hogwild) ----
        if (P.train) {
            const float ks = kappa * scale * scale;
            const uint32_t rrow = P.seed ^ ((uint32_t)row * 0x85EBCA77u);
            for (int s = tid; s < FF; s += blockDim.x) {
                const int a = s / F, b = s - (s / F) * F;
                if (a == b) continue;
                const int ia = s_idx[a], ib = s_idx[b];
                if (ia < 0 || ib < 0) continue;
                const float coef = ks * s_x[a] * s_x[b];
                const size_t ov = (size_t)ia * fstride + (size_t)s_fld[b] * Kp;
                float4 own[KC], par[KC], gg[KC];
#pragma unroll
                for (int c = 0; c < KC; ++c) gg[c] = ld_chunk<BF>(G, ov + 4 * c);
                if (STAGE) {
#pragma unroll
                    for (int c = 0; c < KC; ++c) {
                        own[c] = P.reload ? ld_chunk<BF>(V, ov + 4 * c) : to_f4<BF>(s_v[s * KC + c]);
                        par[c] = to_f4<BF>(s_v[(b * F + a) * KC + c]);
                    }
                } else {
                    const size_t op = (size_t)ib * fstride + (size_t)s_fld[a] * Kp;
#pragma unroll
                    for (int c = 0; c < KC; ++c) { own[c] = ld_chunk<BF>(V, ov + 4 * c); par[c] = ld_chunk<BF>(V, op + 4 * c); }
                }
#pragma unroll
                for (int c = 0; c < KC; ++c) {
                    float4 g;
                    g.x = coef * par[c].x + P.lambda_v * own[c].x;
                    g.y = coef * par[c].y + P.lambda_v * own[c].y;
                    g.z = coef * par[c].z + P.lambda_v * own[c].z;
                    g.w = coef * par[c].w + P.lambda_v * own[c].w;
                    gg[c].x += g.x * g.x; gg[c].y += g.y * g.y; gg[c].z += g.z * g.z; gg[c].w += g.w * g.w;
                    own[c].x -= P.eta0 * g.x * rsqrtf(gg[c].x + P.eps);
                    own[c].y -= P.eta0 * g.y * rsqrtf(gg[c].y + P.eps);
                    own[c].z -= P.eta0 * g.z * rsqrtf(gg[c].z + P.eps);
                    own[c].w -= P.eta0 * g.w * rsqrtf(gg[c].w + P.eps);
                    const uint32_t rnd = BF ? hash3(rrow, (uint32_t)s, (uint32_t)c) : 0u;
                    st_chunk<BF>(V, ov + 4 * c, own[c], rnd);
                    st_chunk<BF>(G, ov + 4 * c, gg[c], rnd ^ 0xA5A5A5A5u);
                }
            }
            if (P.use_linear && tid < F) {
                const int i = s_idx[tid];
                if (i >= 0) {
                    const float g = kappa * s_x[tid] * scale;
                    w[i] = ftrl_update(wz + i, wn + i, w[i], g, P.alpha, P.beta, P.lambda1, P.lambda2);
                }
            }
            if (P.use_bias && tid == 0) {
                bias[0] = ftrl_update(bias + 1, bias + 2, bias[0], kappa, P.alpha, P.beta, 0.f, 0.f);
            }
        }
        __syncthreads();  // LDS reuse by the next row
    }
}

template <int KC, bool BF>
int launch_ffm(const FFMParams& P, const int32_t* idx, const int32_t* fld, const float* val,
               const float* y, void* V, void* G, float* w, float* wz, float* wn, float* bias,
               float* pred, float* loss, int grid, hipStream_t stream) {
    const size_t meta = (size_t)3 * P.F * 4 + 16 * 4;
    const size_t stage = (size_t)P.F * P.F * KC * (BF ? 8 : 16);
    const bool use_stage = stage + meta <= 64 * 1024;
    const int blocks = grid > 0 ? grid : (P.B < 256 * 8 * 4 ? P.B : 256 * 8 * 4);
    if (blocks <= 0) return 0;
    if (use_stage) {
        hipLaunchKernelGGL((ffm_row_kernel<KC, true, BF>), dim3(blocks), dim3(256), stage + meta, stream,
                           P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss);
    } else {
        hipLaunchKernelGGL((ffm_row_kernel<KC, false, BF>), dim3(blocks), dim3(256), meta, stream,
                           P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss);
    }
    HM_LAUNCH_RET();
}

template <bool BF>
int dispatch(const FFMParams& P, const int32_t* idx, const int32_t* fld, const float* val,
             const float* y, void* V, void* G, float* w, float* wz, float* wn, float* bias,
             float* pred, float* loss, int grid, hipStream_t stream) {
    switch (P.Kp / 4) {
        case 1: return launch_ffm<1, BF>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
        case 2: return launch_ffm<2, BF>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
        case 3: return launch_ffm<3, BF>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
        case 4: return launch_ffm<4, BF>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
        case 8: return launch_ffm<8, BF>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
        default: return (int)hipErrorInvalidValue;
    }
}

}  // namespace

// hp layout (floats): eta0, eps, lambda_v, alpha, beta, lambda1, lambda2, min_target, max_target
// ip layout (ints)  : B, F, num_features, num_fields, Kp, classification, train, use_linear,
//                     use_bias, norm, grid, reload, bf16_state, seed
HM_API int hm_ffm_step(const int32_t* ip, const float* hp, const int32_t* idx, const int32_t* fld,
                       const float* val, const float* y, void* V, void* G, float* w, float* wz,
                       float* wn, float* bias, float* pred, float* loss, hipStream_t stream) {
    FFMParams P;
    P.B = ip[0]; P.F = ip[1]; P.num_features = ip[2]; P.num_fields = ip[3]; P.Kp = ip[4];
    P.classification = ip[5]; P.train = ip[6]; P.use_linear = ip[7]; P.use_bias = ip[8];
    P.norm = ip[9];
    const int grid = ip[10];
    P.reload = ip[11];
    const int bf16 = ip[12];
    P.seed = (uint32_t)ip[13];
    P.eta0 = hp[0]; P.eps = hp[1]; P.lambda_v = hp[2]; P.alpha = hp[3]; P.beta = hp[4];
    P.lambda1 = hp[5]; P.lambda2 = hp[6]; P.min_target = hp[7]; P.max_target = hp[8];
    if (P.F <= 0 || P.F > 256 || (P.Kp & 3)) return (int)hipErrorInvalidValue;
    return bf16 ? dispatch<true>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream)
                : dispatch<false>(P, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss, grid, stream);
}
