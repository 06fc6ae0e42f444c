// Fused join-predict (upstream's documented prediction queries, e.g.
//   SELECT t.rowid, sigmoid(sum(m.weight * t.value)) FROM test_exploded t
//   LEFT OUTER JOIN model m ON (t.feature = m.feature) GROUP BY t.rowid
// and the fm_predict(m.Wi, m.Vif, t.Xi) UDAF variant).  The SQL executor resolves the join to a
// model-row index per exploded test row (tm, -1 = no match) and the GROUP BY to a group code per
// row (g); these kernels then do the gather + multiply + per-group reduction in one pass over
// the exploded rows, with no joined table ever materialised:
//   dot: sum[g] += W[tm] * v,  cnt[g] += 1            (NULL products skipped, like SUM)
//   fm : lin[g] += W[tm] * x,  S[g][f] += V[tm][f] x,  Q[g][f] += (V[tm][f] x)^2
//        (fm_predict = lin + 1/2 sum_f (S^2 - Q), finished on the host)
// One thread per exploded row (fm: one thread per (row, factor)); fp64 accumulation with
// memory-side float atomics: the rows of one group are adjacent (~40 per test row), so a wave
// touches a handful of addresses and atomics are far cheaper than a sort + segmented reduce.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void join_dot_kernel(const int32_t* __restrict__ tm, const float* __restrict__ v,
                                                       const int32_t* __restrict__ g, const float* __restrict__ W,
                                                       int64_t n, double* __restrict__ sum,
                                                       int32_t* __restrict__ cnt) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int r = tm[i];
        if (r < 0) continue;
        const float w = W[r];
        const float x = v[i];
        if (isnan(w) || isnan(x)) continue;
        const int gi = g[i];
        atomicAdd(sum + gi, (double)w * (double)x);
        atomicAdd(cnt + gi, 1);
    }
}

// t = row * k + f; lanes of a row are adjacent so the V row is read as one contiguous span
__global__ __launch_bounds__(256) void join_fm_kernel(const int32_t* __restrict__ tm, const float* __restrict__ x,
                                                      const int32_t* __restrict__ g, const float* __restrict__ W,
                                                      const float* __restrict__ V, const uint8_t* __restrict__ vmask,
                                                      int64_t n, int k, double* __restrict__ lin,
                                                      double* __restrict__ S, double* __restrict__ Q) {
    const int64_t total = n * (int64_t)k;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
        const int64_t i = t / k;
        const int f = (int)(t - i * k);
        const int r = tm[i];
        if (r < 0) continue;
        const double xi = (double)x[i];
        const int gi = g[i];
        if (f == 0) {
            const float w = W[r];
            if (!isnan(w)) atomicAdd(lin + gi, (double)w * xi);
        }
        if (!vmask[r]) continue;
        const double vv = (double)V[(size_t)r * k + f] * xi;
        atomicAdd(S + (size_t)gi * k + f, vv);
        atomicAdd(Q + (size_t)gi * k + f, vv * vv);
    }
}

// FFM scoring query (two model joins: t.i = m1.i, t.j = m2.i; ffm_predict(m1.Wi, m1.Vi, m2.Vi,
// t.Xi, t.Xj)): per exploded row, <V1[ti], V2[tj]> xi xj when both V rows exist, else W1[ti] xi
// (linear and bias rows), the generic UDAF's rule.  One thread per row, the k-loop over the two
// contiguous V rows in registers; the rows of one test row are adjacent (~n_fields^2 / 2 of
// them), so a wave almost always shares one group: then it reduces through DPP shuffles and
// issues ONE fp64 atomic, else each lane adds its own value.
__global__ __launch_bounds__(256) void join_ffm_kernel(const int32_t* __restrict__ ti, const int32_t* __restrict__ tj,
                                                       const float* __restrict__ xi, const float* __restrict__ xj,
                                                       const int32_t* __restrict__ g, const float* __restrict__ W1,
                                                       const float* __restrict__ V1, const uint8_t* __restrict__ m1,
                                                       const float* __restrict__ V2, const uint8_t* __restrict__ m2,
                                                       int64_t n, int k, double* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    // every lane runs the same trip count so the wave-wide shuffles below see all 64 lanes
    for (int64_t base = (int64_t)blockIdx.x * 256; base < n; base += stride) {
        const int64_t i = base + threadIdx.x;
        double v = 0.0;
        int gi = -1;
        if (i < n) {
            const int a = ti[i];
            gi = g[i];
            if (a >= 0) {
                const int b = tj[i];
                const float x = xi[i];
                if (b >= 0 && m1[a] && m2[b]) {
                    const float* p = V1 + (size_t)a * k;
                    const float* q = V2 + (size_t)b * k;
                    double d = 0.0;
                    for (int f = 0; f < k; ++f) d += (double)p[f] * (double)q[f];
                    v = d * (double)x * (double)xj[i];
                } else {
                    const float w = W1[a];
                    if (!isnan(w)) v = (double)w * (double)x;
                }
            }
        }
        const int g0 = __shfl(gi, 0);
        const bool uniform = __all(gi == g0 || gi < 0);
        if (uniform) {
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
            if ((threadIdx.x & 63) == 0 && g0 >= 0) atomicAdd(out + g0, v);
        } else if (gi >= 0 && v != 0.0) {
            atomicAdd(out + gi, v);
        }
    }
}

int grid_for(int64_t n) {
    int64_t b = (n + 255) / 256;
    return (int)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

}  // namespace

// sum f64 [G] and cnt i32 [G] must be zeroed by the caller.
HM_API int hm_join_dot(const int32_t* tm, const float* v, const int32_t* g, const float* W, int64_t n,
                       double* sum, int32_t* cnt, hipStream_t stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(join_dot_kernel, dim3(grid_for(n)), dim3(256), 0, stream, tm, v, g, W, n, sum, cnt);
    HM_LAUNCH_RET();
}

// lin f64 [G], S/Q f64 [G][k] zeroed by the caller; V f32 [R][k], vmask u8 [R] (0 = NULL V row).
HM_API int hm_join_fm(const int32_t* tm, const float* x, const int32_t* g, const float* W, const float* V,
                      const uint8_t* vmask, int64_t n, int k, double* lin, double* S, double* Q,
                      hipStream_t stream) {
    if (n <= 0) return 0;
    if (k <= 0) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(join_fm_kernel, dim3(grid_for(n * (int64_t)k)), dim3(256), 0, stream, tm, x, g, W, V, vmask,
                       n, k, lin, S, Q);
    HM_LAUNCH_RET();
}

// ti/tj i32 [n] (-1 = no model row), xi/xj f32 [n], g i32 [n]; W1 f32 [R1] (NaN = NULL),
// V1 f32 [R1][k] + m1 u8 [R1], V2 f32 [R2][k] + m2 u8 [R2]; out f64 [G] zeroed by the caller.
HM_API int hm_join_ffm(const int32_t* ti, const int32_t* tj, const float* xi, const float* xj, const int32_t* g,
                       const float* W1, const float* V1, const uint8_t* m1, const float* V2, const uint8_t* m2,
                       int64_t n, int k, double* out, hipStream_t stream) {
    if (n <= 0) return 0;
    if (k <= 0) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(join_ffm_kernel, dim3(grid_for(n)), dim3(256), 0, stream, ti, tj, xi, xj, g, W1, V1, m1, V2,
                       m2, n, k, out);
    HM_LAUNCH_RET();
}
