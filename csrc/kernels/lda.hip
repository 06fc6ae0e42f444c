// Online-VB LDA E-step (upstream hivemall/topicmodel/OnlineLDAModel.eStep,
// Hoffman et al. NIPS'10): for every document d of a mini-batch, iterate
//     Et[k]      = exp(digamma(gamma[k]) - digamma(sum_k gamma[k]))
//     phinorm[n] = sum_k Et[k] * Eb[w_n][k]
//     gamma'[k]  = alpha + Et[k] * sum_n c_n * Eb[w_n][k] / phinorm[n]
// until mean_k |gamma' - gamma| < delta (per document, as upstream) or max_iter, then emit the
// sufficient statistics contrib[n][k] = Et[k] * Eb[w_n][k] * c_n / phinorm[n].
//
// One 256-thread workgroup per document; lanes span topics (K <= 64 * KC) so a word's topic row
// Eb[w] (expElogbeta transposed to [V][K]: contiguous per word) is one coalesced load, phinorm is
// a DPP wave sum, and each of the 4 waves accumulates its quarter of the words into per-lane
// registers; the 4 partial sums meet in LDS once per iteration.  The document's Eb rows are
// staged in LDS when they fit (the loop re-reads them every iteration).  The whole fixed-point
// loop runs inside the kernel: the torch formulation paid ~10 launches and a host sync per
// inner iteration.
#include "common.h"

namespace {

constexpr int LDA_LDS_FLOATS = 12 * 1024;      // 48 KB of staged Eb rows per workgroup

__device__ __forceinline__ float digammaf(float x) {
    float r = 0.f;
    while (x < 6.f) {
        r -= 1.f / x;
        x += 1.f;
    }
    const float f = 1.f / (x * x);
    const float t = f * (1.f / 12 - f * (1.f / 120 - f * (1.f / 252 - f * (1.f / 240 - f * (1.f / 132)))));
    return r + logf(x) - 0.5f / x - t;
}

template <int KC>
__global__ __launch_bounds__(256) void lda_estep_kernel(const int32_t* __restrict__ doc_off,
                                                        const int32_t* __restrict__ wid,
                                                        const float* __restrict__ cnt,
                                                        const float* __restrict__ EbT, int K, float alpha,
                                                        float delta, int max_iter, float* __restrict__ gamma,
                                                        float* __restrict__ contrib,
                                                        int32_t* __restrict__ iters_out) {
    __shared__ float s_acc[4][64 * KC];
    __shared__ float s_gamma[64 * KC];
    __shared__ float s_et[64 * KC];
    __shared__ float s_red[4];
    __shared__ int s_done;
    extern __shared__ float s_eb[];
    const int d = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n0 = doc_off[d], n1 = doc_off[d + 1], nd = n1 - n0;
    const bool staged = (int64_t)nd * K <= LDA_LDS_FLOATS;
    if (staged) {
        for (int i = tid; i < nd * K; i += 256) {
            const int n = i / K, k = i - n * K;
            s_eb[i] = EbT[(size_t)wid[n0 + n] * K + k];
        }
    }
    for (int k = tid; k < 64 * KC; k += 256) s_gamma[k] = k < K ? gamma[(size_t)d * K + k] : 0.f;
    __syncthreads();
    auto eb = [&](int n, int k) -> float {
        return staged ? s_eb[n * K + k] : EbT[(size_t)wid[n0 + n] * K + k];
    };
    int it = 0;
    for (;;) {
        // Et from the current gamma (wave 0; K <= 256 topics)
        if (wave == 0) {
            float gs = 0.f;
#pragma unroll
            for (int j = 0; j < KC; ++j) gs += s_gamma[lane + 64 * j];
            gs = hm::wave_sum(gs);
            const float dg = digammaf(gs);
#pragma unroll
            for (int j = 0; j < KC; ++j) {
                const int k = lane + 64 * j;
                s_et[k] = k < K ? __expf(digammaf(s_gamma[k]) - dg) : 0.f;
            }
        }
        __syncthreads();
        if (it == max_iter) break;           // final Et computed: emit the statistics below
        float et[KC], acc[KC];
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            et[j] = s_et[lane + 64 * j];
            acc[j] = 0.f;
        }
        for (int n = wave; n < nd; n += 4) {
            float e[KC], p = 0.f;
#pragma unroll
            for (int j = 0; j < KC; ++j) {
                const int k = lane + 64 * j;
                e[j] = k < K ? eb(n, k) : 0.f;
                p += et[j] * e[j];
            }
            p = hm::wave_sum(p) + 1e-30f;
            const float s = cnt[n0 + n] / p;
#pragma unroll
            for (int j = 0; j < KC; ++j) acc[j] += s * e[j];
        }
#pragma unroll
        for (int j = 0; j < KC; ++j) s_acc[wave][lane + 64 * j] = acc[j];
        __syncthreads();
        if (wave == 0) {
            float ch = 0.f;
#pragma unroll
            for (int j = 0; j < KC; ++j) {
                const int k = lane + 64 * j;
                if (k < K) {
                    const float g = alpha + et[j] * (s_acc[0][k] + s_acc[1][k] + s_acc[2][k] + s_acc[3][k]);
                    ch += fabsf(g - s_gamma[k]);
                    s_gamma[k] = g;
                }
            }
            ch = hm::wave_sum(ch);
            if (lane == 0) s_done = (ch / (float)K < delta) ? 1 : 0;
        }
        __syncthreads();
        ++it;
        if (s_done) {
            max_iter = it;                   // uniform: recompute Et once more, then emit
        }
    }
    // sufficient statistics with the final Et
    float et[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) et[j] = s_et[lane + 64 * j];
    for (int n = wave; n < nd; n += 4) {
        float e[KC], p = 0.f;
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            const int k = lane + 64 * j;
            e[j] = k < K ? eb(n, k) : 0.f;
            p += et[j] * e[j];
        }
        p = hm::wave_sum(p) + 1e-30f;
        const float s = cnt[n0 + n] / p;
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            const int k = lane + 64 * j;
            if (k < K) contrib[(size_t)(n0 + n) * K + k] = et[j] * e[j] * s;
        }
    }
    for (int k = tid; k < K; k += 256) gamma[(size_t)d * K + k] = s_gamma[k];
    if (tid == 0 && iters_out) iters_out[d] = it;
}

}  // namespace

// doc_off int32 [B+1] (CSR over the mini-batch non-zeros), wid int32 [N] word ids, cnt f32 [N],
// EbT f32 [V][K] = exp(E[log beta]) transposed, gamma f32 [B][K] (in: initial, out: final),
// contrib f32 [N][K] (out), iters_out int32 [B] (optional: inner iterations per document).
HM_API int hm_lda_estep(const int32_t* doc_off, const int32_t* wid, const float* cnt, const float* EbT, int B,
                        int K, float alpha, float delta, int max_iter, float* gamma, float* contrib,
                        int32_t* iters_out, hipStream_t stream) {
    if (B <= 0) return 0;
    if (K <= 0 || K > 256 || max_iter < 0) return (int)hipErrorInvalidValue;
    const size_t sh = LDA_LDS_FLOATS * sizeof(float);
#define HM_LDA(KC)                                                                                       \
    hipLaunchKernelGGL(lda_estep_kernel<KC>, dim3(B), dim3(256), sh, stream, doc_off, wid, cnt, EbT, K, alpha, \
                       delta, max_iter, gamma, contrib, iters_out)
    if (K <= 64) HM_LDA(1);
    else if (K <= 128) HM_LDA(2);
    else HM_LDA(4);
#undef HM_LDA
    HM_LAUNCH_RET();
}
