// Mini-batch FM on low-dimensional dense rows (train_fm -engine minibatch; models/fm_dense.py).
//
// One step of B rows is two launches: a gradient kernel and a parameter-parallel AdaGrad kernel.
// Default gradient kernel: fmd_mfma_kernel (below) — the two GEMM-shaped products on f32 MFMA.
// The VALU kernel (variant 1, the round-2 first version):
//   fmd_grad_kernel   — 64-row tiles (<= 128 workgroups, each looping over tiles): the tile X [64][d] (coalesced
//                       read), V [d][KP] and w are staged in LDS; 4 lanes per row form
//                       XV_r = x_r V, the prediction p_r = w0 + x_r w + 0.5 (|XV_r|^2 - sum_i x_ri^2 |V_i|^2)
//                       and g_r = dloss/dp_r; then every thread owns parameters and sums the tile's
//                       contributions  dV_ik = sum_r g_r x_ri (XV_rk - V_ik x_ri),  dw_i = sum_r g_r x_ri,
//                       dw0 = sum_r g_r  (and the tile's loss) into its workgroup's partial row —
//                       no atomics, deterministic;
//   fmd_update_kernel — one wave per parameter sums the <= 128 partial rows (workgroups loop
//                       over row tiles), adds the L2 term and applies AdaGrad to the mean gradient.
// Arithmetic intensity is ~4 (1 + k) FLOP per byte of X (d = 28, k = 8: ~36 FLOP/B) — below the
// VALU ridge of MI355X, so the tile math stays on VALU from LDS (the GEMM formulation on
// hipBLASLt MFMA kernels measured 9-56 M rows/s, launch- and skinny-GEMM-bound:
// profiles/fm_dense_r2/).  Upstream semantics are per-row SGD (hivemall/fm/
// FactorizationMachineUDTF); this engine is mini-batch AdaGrad by design (docs/compat.md).
#include "common.h"

namespace {

constexpr int FMD_RB = 64;       // rows per workgroup
constexpr int FMD_DMAX = 64;     // features
constexpr int FMD_KMAX = 32;     // padded factors
constexpr int FMD_GRID = 128;    // workgroups per step (each loops over row tiles)
constexpr int FMD_MFMA_BLK = 512;     // MFMA kernel: default workgroups per step
constexpr int FMD_MFMA_MAXBLK = 2048; // ... and the most the partial buffer is sized for
constexpr int FMD_PMAX = (FMD_DMAX * FMD_KMAX + FMD_DMAX + 2 + 255) / 256;   // parameters per thread

__global__ __launch_bounds__(256) void fmd_grad_kernel(const float* __restrict__ X, const float* __restrict__ y,
                                                       int64_t n, int d, int KP, const float* __restrict__ V,
                                                       const float* __restrict__ w, const float* __restrict__ w0,
                                                       int cls, float lo, float hi, float* __restrict__ partial) {
    __shared__ float s_x[FMD_RB * FMD_DMAX];
    __shared__ float s_V[FMD_DMAX * FMD_KMAX];
    __shared__ float s_xv[FMD_RB * FMD_KMAX];
    __shared__ float s_w[FMD_DMAX], s_vsq[FMD_DMAX];
    __shared__ float s_g[FMD_RB], s_loss[FMD_RB];
    const int tid = threadIdx.x;
    const int P = d * KP;
    const int NP = P + d + 2;
    for (int e = tid; e < d * KP; e += 256) s_V[e] = V[e];
    for (int i = tid; i < d; i += 256) s_w[i] = w[i];
    __syncthreads();
    for (int i = tid; i < d; i += 256) {
        float s = 0.f;
        for (int k = 0; k < KP; ++k) s += s_V[i * KP + k] * s_V[i * KP + k];
        s_vsq[i] = s;
    }
    float acc[FMD_PMAX];
#pragma unroll
    for (int j = 0; j < FMD_PMAX; ++j) acc[j] = 0.f;
    const int64_t n_tiles = (n + FMD_RB - 1) / FMD_RB;
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int64_t row0 = tile * FMD_RB;
        const int nr = (int)min((int64_t)FMD_RB, n - row0);
        const float* xt = X + row0 * d;
        __syncthreads();                 // the previous tile's phase 2 is done with s_x / s_g
        for (int e = tid; e < nr * d; e += 256) s_x[e] = xt[e];
        __syncthreads();
        // phase 1: 4 lanes per row
        const int r = tid >> 2, q = tid & 3;
        float part = 0.f;
        if (r < nr) {
            const float* xr = s_x + r * d;
            float sq = 0.f;
            for (int k = q; k < KP; k += 4) {
                float a = 0.f;
                for (int i = 0; i < d; ++i) a += xr[i] * s_V[i * KP + k];
                s_xv[r * KP + k] = a;
                sq += a * a;
            }
            float lin = 0.f;
            for (int i = q; i < d; i += 4) {
                const float x = xr[i];
                lin += x * s_w[i] - 0.5f * x * x * s_vsq[i];
            }
            part = 0.5f * sq + lin;
        }
        part += __shfl_xor(part, 1);
        part += __shfl_xor(part, 2);
        if (r < nr && q == 0) {
            const float p = w0[0] + part;
            const float t = y[row0 + r];
            float g, l;
            if (cls) {                   // t in {-1, +1}: loss = softplus(-t p)
                const float z = -t * p;
                g = -t / (1.f + __expf(-z));
                l = z > 0.f ? z + log1pf(__expf(-z)) : log1pf(__expf(z));
            } else {
                const float pc = fminf(fmaxf(p, lo), hi);
                g = pc - t;
                l = 0.5f * g * g;
            }
            s_g[r] = g;
            s_loss[r] = l;
        }
        __syncthreads();
        // phase 2: each thread owns parameters tid + 256 j and adds the tile's rows
#pragma unroll
        for (int j = 0; j < FMD_PMAX; ++j) {
            const int t2 = tid + 256 * j;
            if (t2 >= NP) break;
            float a = 0.f;
            if (t2 < P) {
                const int i = t2 / KP, k = t2 - i * KP;
                const float vik = s_V[t2];
                for (int rr = 0; rr < nr; ++rr) {
                    const float x = s_x[rr * d + i];
                    a += s_g[rr] * x * (s_xv[rr * KP + k] - vik * x);
                }
            } else if (t2 < P + d) {
                const int i = t2 - P;
                for (int rr = 0; rr < nr; ++rr) a += s_g[rr] * s_x[rr * d + i];
            } else if (t2 == P + d) {
                for (int rr = 0; rr < nr; ++rr) a += s_g[rr];
            } else {
                for (int rr = 0; rr < nr; ++rr) a += s_loss[rr];
            }
            acc[j] += a;
        }
    }
    float* out = partial + (size_t)blockIdx.x * NP;
#pragma unroll
    for (int j = 0; j < FMD_PMAX; ++j) {
        const int t2 = tid + 256 * j;
        if (t2 < NP) out[t2] = acc[j];
    }
}

struct FmdUpd {
    int nblk, d, KP, k;
    int64_t sb, st;                      // partial[b * sb + t * st]
    float inv_b, lr, eps, l0, lw, lv;
};

// one wave per parameter: lanes sum the workgroups' partials, a wave reduction, lane 0 updates
__global__ __launch_bounds__(256) void fmd_update_kernel(const float* __restrict__ partial, FmdUpd u,
                                                         float* __restrict__ V, float* __restrict__ w,
                                                         float* __restrict__ w0, float* __restrict__ GV,
                                                         float* __restrict__ Gw, float* __restrict__ Gw0,
                                                         double* __restrict__ loss_sum) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int P = u.d * u.KP;
    const int NP = P + u.d + 2;
    if (t >= NP) return;
    if (t < P && (t % u.KP) >= u.k) return;   // padded factor columns stay zero
    float s = 0.f;
    for (int b = lane; b < u.nblk; b += 64) s += partial[b * u.sb + t * u.st];
    s = hm::wave_sum(s);
    if (lane != 0) return;
    if (t == NP - 1) {                   // the step's summed loss
        loss_sum[0] += (double)s;
        return;
    }
    float grad = s * u.inv_b;
    float *p, *G;
    float lam;
    if (t < P) { p = V + t; G = GV + t; lam = u.lv; }
    else if (t < P + u.d) { p = w + (t - P); G = Gw + (t - P); lam = u.lw; }
    else { p = w0; G = Gw0; lam = u.l0; }
    grad += lam * p[0];
    const float g2 = G[0] + grad * grad;
    G[0] = g2;
    p[0] -= u.lr * grad / (sqrtf(g2) + u.eps);
}

// ---------------------------------------------------------------------------------------------
// f32 MFMA gradient kernel.  Per 64-row tile, wave w owns rows 16w .. 16w+15:
//   phase 1  C[r][c] = sum_i x_ri B1[i][c]  on v_mfma_f32_16x16x4_f32 (K = features), with the
//            B1 columns [V_0 .. V_{KP-1} | w | -vsq/2]: the last column is fed x^2 instead of x,
//            so p_r = w0 + 0.5 sum_{c<KP} C_rc^2 + C_r,KP + C_r,KP+1 (a 16-lane reduction);
//   phase 2  D[i][c] += sum_r (g_r x_ri) B2[r][c]  (K = the wave's 16 rows), B2 = [XV | 1 | 0]
//            taken straight from phase 1's accumulators: the C layout holds rows 4q + j of
//            column lane&15 in lane (q = lane >> 4), so step j uses K index q -> row 4q + j and
//            A and B agree on that row order with no data movement.  Row d of A is g_r (a bias
//            feature), so D[d][KP] = sum g; D[i][KP] = dw_i; D[i][c<KP] - V_ic sum_r g_r x_ri^2 = dV_ic.
// D stays in accumulator registers over all of the workgroup's tiles; the X tile for the next
// tile is prefetched into registers while the current one computes.  The four waves' D are
// summed in LDS in a fixed order (deterministic) into partial[t * nblk + block].
typedef float fmd_f4 __attribute__((ext_vector_type(4)));

template <int KT, int NB>
__global__ __launch_bounds__(256) void fmd_mfma_kernel(const float* __restrict__ X, const float* __restrict__ y,
                                                       int64_t n, int d, int KP, const float* __restrict__ V,
                                                       const float* __restrict__ w, const float* __restrict__ w0,
                                                       int cls, float lo, float hi, float* __restrict__ partial) {
    constexpr int MB = (4 * KT) / 16 + 1;         // output row blocks (features + the bias row)
    constexpr int U = (64 * KT + 255) / 256;       // float4 loads per thread per X tile
    __shared__ __attribute__((aligned(16))) float s_x[64 * 4 * KT];
    __shared__ float s_red[4][MB * NB * 256];
    __shared__ float s_sd[4][MB * 16];
    __shared__ float s_l[4];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, q = lane >> 4, c16 = lane & 15;
    const int P = d * KP, NP = P + d + 2;
    const int nblk = gridDim.x;
    const int NBS = (KP + 1) >> 4, CS = (KP + 1) & 15;   // block / column of the -vsq/2 column

    // B1 operands (constant over the step): lane holds B1[k = q + 4t][c = 16 nb + c16]
    // |V_k|^2 from the operands themselves: the 16 lanes of group q hold row k's columns
    float bV[NB][KT], bS[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) {
        const int k = q + 4 * t;
        float vsq = 0.f;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
            const int c = 16 * nb + c16;
            const float v = k < d ? (c < KP ? V[k * KP + c] : (c == KP ? w[k] : 0.f)) : 0.f;
            bV[nb][t] = v;
            if (c < KP) vsq += v * v;
        }
        vsq += __shfl_xor(vsq, 1);
        vsq += __shfl_xor(vsq, 2);
        vsq += __shfl_xor(vsq, 4);
        vsq += __shfl_xor(vsq, 8);
        bS[t] = (k < d && c16 == CS) ? -0.5f * vsq : 0.f;
    }
    const float w0v = w0[0];
    fmd_f4 acc[MB][NB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = fmd_f4{0.f, 0.f, 0.f, 0.f};
    float sd[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) sd[mb] = 0.f;
    float lsum = 0.f;

    const int64_t n_tiles = (n + 63) / 64;
    const int tile_elems = 64 * d;
    float4 pre[U];
    auto fetch = [&](int64_t tile) {
        const int64_t row0 = tile * 64;
        const int valid = (int)min((int64_t)64, n - row0) * d;
        const float* xt = X + row0 * d;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = 4 * (tid + 256 * u);
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (e + 3 < valid) {
                v = *reinterpret_cast<const float4*>(xt + e);
            } else if (e < valid) {
                v.x = xt[e];
                if (e + 1 < valid) v.y = xt[e + 1];
                if (e + 2 < valid) v.z = xt[e + 2];
            }
            pre[u] = v;
        }
    };
    if ((int64_t)blockIdx.x < n_tiles) fetch(blockIdx.x);
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += nblk) {
        const int64_t row0 = tile * 64;
        const int nr = (int)min((int64_t)64, n - row0);
        float yv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int rl = 16 * wv + 4 * q + j;
            yv[j] = rl < nr ? y[row0 + rl] : 0.f;
        }
        __syncthreads();                                  // the previous tile's reads of s_x are done
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = 4 * (tid + 256 * u);
            if (e < tile_elems) *reinterpret_cast<float4*>(s_x + e) = pre[u];
        }
        __syncthreads();
        if (tile + nblk < n_tiles) fetch(tile + nblk);   // lands while this tile computes

        // ---- phase 1: XV, x.w and -x^2.vsq/2 of the wave's 16 rows
        fmd_f4 c1[NB];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) c1[nb] = fmd_f4{0.f, 0.f, 0.f, 0.f};
        const float* xr = s_x + (16 * wv + c16) * d;
#pragma unroll
        for (int t = 0; t < KT; ++t) {
            const int k = q + 4 * t;
            const float a = k < d ? xr[k] : 0.f;
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) c1[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bV[nb][t], c1[nb], 0, 0, 0);
            // the -vsq/2 column takes x^2 (its B is zero in every other column)
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
                if (nb == NBS) c1[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a * a, bS[t], c1[nb], 0, 0, 0);
        }
        float g[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float part = 0.f;
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
                const int c = 16 * nb + c16;
                const float v = c1[nb][j];
                part += c < KP ? 0.5f * v * v : ((c == KP || c == KP + 1) ? v : 0.f);
            }
            part += __shfl_xor(part, 1);
            part += __shfl_xor(part, 2);
            part += __shfl_xor(part, 4);
            part += __shfl_xor(part, 8);
            const float p = w0v + part, tv = yv[j];
            float gj, l;
            if (cls) {                                     // t in {-1, +1}: loss = softplus(-t p)
                const float z = -tv * p;
                gj = -tv / (1.f + __expf(-z));
                l = z > 0.f ? z + log1pf(__expf(-z)) : log1pf(__expf(z));
            } else {
                const float pc = fminf(fmaxf(p, lo), hi);
                gj = pc - tv;
                l = 0.5f * gj * gj;
            }
            const bool ok = 16 * wv + 4 * q + j < nr;
            g[j] = ok ? gj : 0.f;
            if (ok && c16 == 0) lsum += l;
        }
        // ---- phase 2: D += (g x)^T [XV | 1 | 0] over the wave's rows
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float b2[NB];
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
                const int c = 16 * nb + c16;
                b2[nb] = c < KP ? c1[nb][j] : (c == KP ? 1.f : 0.f);
            }
            const float* xrow = s_x + (16 * wv + 4 * q + j) * d;
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) {
                const int i = 16 * mb + c16;
                const float x = i < d ? xrow[i] : (i == d ? 1.f : 0.f);
                const float a = g[j] * x;
                sd[mb] += a * x;
#pragma unroll
                for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b2[nb], acc[mb][nb], 0, 0, 0);
            }
        }
    }
    // ---- the four waves' partials, summed in LDS in wave order
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
        float v = sd[mb];
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        if (q == 0) s_sd[wv][mb * 16 + c16] = v;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int j = 0; j < 4; ++j) s_red[wv][(mb * NB + nb) * 256 + j * 64 + lane] = acc[mb][nb][j];
    }
    lsum = hm::wave_sum(lsum);
    if (lane == 0) s_l[wv] = lsum;
    __syncthreads();
    const int b = blockIdx.x;
    for (int e = tid; e < MB * NB * 256; e += 256) {
        const int blk = e >> 8, mb = blk / NB, nb = blk - mb * NB, rem = e & 255, j = rem >> 6, ln = rem & 63;
        const int i = 16 * mb + 4 * (ln >> 4) + j, c = 16 * nb + (ln & 15);
        const float D = ((s_red[0][e] + s_red[1][e]) + s_red[2][e]) + s_red[3][e];
        if (i < d && c < KP) {
            const int si = (i >> 4) * 16 + (i & 15);
            const float sdg = ((s_sd[0][si] + s_sd[1][si]) + s_sd[2][si]) + s_sd[3][si];
            partial[(int64_t)(i * KP + c) * nblk + b] = D - V[i * KP + c] * sdg;
        } else if (i < d && c == KP) {
            partial[(int64_t)(P + i) * nblk + b] = D;
        } else if (i == d && c == KP) {
            partial[(int64_t)(P + d) * nblk + b] = D;
        }
    }
    if (tid == 0) partial[(int64_t)(NP - 1) * nblk + b] = ((s_l[0] + s_l[1]) + s_l[2]) + s_l[3];
}

template <int KT>
hipError_t fmd_mfma_launch(int NB, int nblk, hipStream_t st, const float* X, const float* y, int64_t n, int d,
                           int KP, const float* V, const float* w, const float* w0, int cls, float lo, float hi,
                           float* partial) {
    if (NB == 1)
        hipLaunchKernelGGL((fmd_mfma_kernel<KT, 1>), dim3(nblk), dim3(256), 0, st, X, y, n, d, KP, V, w, w0, cls, lo, hi, partial);
    else if (NB == 2)
        hipLaunchKernelGGL((fmd_mfma_kernel<KT, 2>), dim3(nblk), dim3(256), 0, st, X, y, n, d, KP, V, w, w0, cls, lo, hi, partial);
    else
        hipLaunchKernelGGL((fmd_mfma_kernel<KT, 3>), dim3(nblk), dim3(256), 0, st, X, y, n, d, KP, V, w, w0, cls, lo, hi, partial);
    return hipGetLastError();
}

}  // namespace

// One mini-batch step over rows [0, n) of X (fp32 [n][d], row-major, 16-B aligned), targets y [n];
// V [d][KP], w [d], w0 [1] updated in place with AdaGrad state GV / Gw / Gw0; loss_sum[0] += summed loss.
// partial: >= hm_fmd_partial_floats(n, d, KP) floats of scratch.
// ip: n, d, KP, k, cls, variant (0 = MFMA, 1 = VALU kernel), nblk (0 = auto);
// hp: lr, eps, lambda0, lambda_w, lambda_v, min_target, max_target
HM_API int64_t hm_fmd_max_blocks() { return FMD_MFMA_MAXBLK; }

HM_API int hm_fmd_step(const int64_t* ip, const float* hp, const float* X, const float* y, float* V, float* w,
                       float* w0, float* GV, float* Gw, float* Gw0, float* partial, double* loss_sum,
                       hipStream_t stream) {
    const int64_t n = ip[0];
    const int d = (int)ip[1], KP = (int)ip[2], k = (int)ip[3], cls = (int)ip[4];
    const int variant = (int)ip[5];
    if (n <= 0) return 0;
    if (d <= 0 || d > FMD_DMAX || KP <= 0 || KP > FMD_KMAX || k > KP) return (int)hipErrorInvalidValue;
    const int NP = d * KP + d + 2;
    const int64_t n_tiles = (n + FMD_RB - 1) / FMD_RB;
    FmdUpd u;
    u.d = d; u.KP = KP; u.k = k;
    u.inv_b = 1.f / (float)n; u.lr = hp[0]; u.eps = hp[1]; u.l0 = hp[2]; u.lw = hp[3]; u.lv = hp[4];
    if (variant == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0) {
        int nblk = ip[6] > 0 ? (int)ip[6] : FMD_MFMA_BLK;
        nblk = (int)min((int64_t)min(nblk, FMD_MFMA_MAXBLK), n_tiles);
        const int NB = (KP + 2 + 15) / 16;
        hipError_t e;
        if (d <= 8) e = fmd_mfma_launch<2>(NB, nblk, stream, X, y, n, d, KP, V, w, w0, cls, hp[5], hp[6], partial);
        else if (d <= 16) e = fmd_mfma_launch<4>(NB, nblk, stream, X, y, n, d, KP, V, w, w0, cls, hp[5], hp[6], partial);
        else if (d <= 28) e = fmd_mfma_launch<7>(NB, nblk, stream, X, y, n, d, KP, V, w, w0, cls, hp[5], hp[6], partial);
        else if (d <= 32) e = fmd_mfma_launch<8>(NB, nblk, stream, X, y, n, d, KP, V, w, w0, cls, hp[5], hp[6], partial);
        else if (d <= 48) e = fmd_mfma_launch<12>(NB, nblk, stream, X, y, n, d, KP, V, w, w0, cls, hp[5], hp[6], partial);
        else e = fmd_mfma_launch<16>(NB, nblk, stream, X, y, n, d, KP, V, w, w0, cls, hp[5], hp[6], partial);
        if (e != hipSuccess) return (int)e;
        u.nblk = nblk; u.sb = 1; u.st = nblk;
    } else {
        const int nblk = (int)min((int64_t)FMD_GRID, n_tiles);
        hipLaunchKernelGGL(fmd_grad_kernel, dim3(nblk), dim3(256), 0, stream, X, y, n, d, KP, V, w, w0, cls, hp[5],
                           hp[6], partial);
        u.nblk = nblk; u.sb = NP; u.st = 1;
    }
    hipLaunchKernelGGL(fmd_update_kernel, dim3((NP + 3) / 4), dim3(256), 0, stream, partial, u, V, w, w0, GV,
                       Gw, Gw0, loss_sum);
    HM_LAUNCH_RET();
}
