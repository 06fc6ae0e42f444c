// Mini-batch FM on low-dimensional dense rows (train_fm -engine minibatch; models/fm_dense.py).
//
// One step of B rows is two launches:
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
    for (int b = lane; b < u.nblk; b += 64) s += partial[(size_t)b * NP + t];
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

}  // namespace

// One mini-batch step over rows [0, n) of X (fp32 [n][d], row-major), targets y [n]; V [d][KP],
// w [d], w0 [1] updated in place with AdaGrad state GV / Gw / Gw0; loss_sum[0] += summed loss.
// partial: >= min(128, ceil(n / 64)) * (d * KP + d + 2) floats of scratch.
// ip: n, d, KP, k, cls;  hp: lr, eps, lambda0, lambda_w, lambda_v, min_target, max_target
HM_API int hm_fmd_step(const int64_t* ip, const float* hp, const float* X, const float* y, float* V, float* w,
                       float* w0, float* GV, float* Gw, float* Gw0, float* partial, double* loss_sum,
                       hipStream_t stream) {
    const int64_t n = ip[0];
    const int d = (int)ip[1], KP = (int)ip[2], k = (int)ip[3], cls = (int)ip[4];
    if (n <= 0) return 0;
    if (d <= 0 || d > FMD_DMAX || KP <= 0 || KP > FMD_KMAX || k > KP) return (int)hipErrorInvalidValue;
    const int nblk = (int)min((int64_t)FMD_GRID, (n + FMD_RB - 1) / FMD_RB);
    hipLaunchKernelGGL(fmd_grad_kernel, dim3(nblk), dim3(256), 0, stream, X, y, n, d, KP, V, w, w0, cls, hp[5],
                       hp[6], partial);
    FmdUpd u;
    u.nblk = nblk; u.d = d; u.KP = KP; u.k = k;
    u.inv_b = 1.f / (float)n; u.lr = hp[0]; u.eps = hp[1]; u.l0 = hp[2]; u.lw = hp[3]; u.lv = hp[4];
    const int NP = d * KP + d + 2;
    hipLaunchKernelGGL(fmd_update_kernel, dim3((NP + 3) / 4), dim3(256), 0, stream, partial, u, V, w, w0, GV,
                       Gw, Gw0, loss_sum);
    HM_LAUNCH_RET();
}
