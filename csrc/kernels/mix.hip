// Model-mixing device kernels (parallel/mix.py): the fp32-accumulating shard mean of an
// all-to-all and the in-place merge of an overlapped (stale-by-one) mix.
//
// Hivemall's MixServer averaged replicas in Java doubles (reference hivemall/mix/store/
// PartialAverage.java).  Here the replicas live in HBM, possibly in bf16:
//   * the wire carries the storage dtype (bf16 halves the bytes over xGMI);
//   * the SUM is never formed in bf16: every rank receives the world's copies of its 1/world
//     shard (all-to-all), sums them in fp32 here and rounds once, then the shards are
//     all-gathered.  Same 2(N-1)/N wire bytes as a ring all-reduce, exact fp32 accumulation,
//     and the all-to-all drives all 7 xGMI links of a GPU at once (point-to-point mesh);
//   * merge: x <- x + (mean - snapshot) in fp32 with one rounding, over a strided view (the V
//     half of the packed FFM V|G table) in one pass instead of five torch temporaries.
#include "common.h"

namespace {

template <bool BF>
__device__ __forceinline__ float4 ld4(const void* p, int64_t e) {
    if constexpr (BF) {
        const uint2 q = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(p) + e);
        return make_float4(__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xFFFF0000u),
                           __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xFFFF0000u));
    } else {
        return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + e);
    }
}

template <bool BF>
__device__ __forceinline__ void st4(void* p, int64_t e, float4 v) {
    if constexpr (BF) {
        const uint32_t lo = (uint32_t)hm::f32_to_bf16(v.x) | ((uint32_t)hm::f32_to_bf16(v.y) << 16);
        const uint32_t hi = (uint32_t)hm::f32_to_bf16(v.z) | ((uint32_t)hm::f32_to_bf16(v.w) << 16);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p) + e) = make_uint2(lo, hi);
    } else {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(p) + e) = v;
    }
}

// out[q] = (1/world) * sum_r recv[r * n + q], 4 elements per thread (n % 4 == 0).
template <bool BF>
__global__ __launch_bounds__(256) void shard_mean_kernel(const void* __restrict__ recv, int world,
                                                         int64_t n, float inv, void* __restrict__ out) {
    const int64_t nq = n >> 2;
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += (int64_t)gridDim.x * 256) {
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int r = 0; r < world; ++r) {
            const float4 v = ld4<BF>(recv, (int64_t)r * n + 4 * q);
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        s.x *= inv; s.y *= inv; s.z *= inv; s.w *= inv;
        st4<BF>(out, 4 * q, s);
    }
}

// x[r * row_stride + c] += mean[r * inner + c] - snap[r * inner + c]  (c < inner, inner % 4 == 0)
template <bool BF>
__global__ __launch_bounds__(256) void merge_kernel(void* __restrict__ x, const void* __restrict__ mean,
                                                    const void* __restrict__ snap, int64_t rows,
                                                    int inner, int64_t row_stride) {
    const int qpr = inner >> 2;
    const int64_t nq = rows * qpr;
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += (int64_t)gridDim.x * 256) {
        const int64_t r = q / qpr;
        const int c = (int)(q - r * qpr) * 4;
        const int64_t xe = r * row_stride + c, me = 4 * q;
        const float4 a = ld4<BF>(x, xe), m = ld4<BF>(mean, me), s = ld4<BF>(snap, me);
        st4<BF>(x, xe, make_float4(a.x + (m.x - s.x), a.y + (m.y - s.y), a.z + (m.z - s.z),
                                   a.w + (m.w - s.w)));
    }
}

int grid_for(int64_t quads) {
    const int64_t b = (quads + 255) / 256;
    return (int)(b < 256 * 16 ? (b > 0 ? b : 1) : 256 * 16);
}

}  // namespace

// dtype: 0 = fp32, 1 = bf16.  recv is [world][n] contiguous, n % 4 == 0.
HM_API int hm_mix_shard_mean(const void* recv, int world, int64_t n, int dtype, void* out,
                             hipStream_t stream) {
    if (world <= 0 || n < 0 || (n & 3)) return (int)hipErrorInvalidValue;
    if (n == 0) return 0;
    const float inv = 1.f / (float)world;
    if (dtype == 1)
        hipLaunchKernelGGL(shard_mean_kernel<true>, dim3(grid_for(n >> 2)), dim3(256), 0, stream, recv, world, n, inv, out);
    else if (dtype == 0)
        hipLaunchKernelGGL(shard_mean_kernel<false>, dim3(grid_for(n >> 2)), dim3(256), 0, stream, recv, world, n, inv, out);
    else
        return (int)hipErrorInvalidValue;
    HM_LAUNCH_RET();
}

// x: rows x inner view with row stride row_stride (elements); mean/snap: contiguous rows x inner.
HM_API int hm_mix_merge(void* x, const void* mean, const void* snap, int64_t rows, int inner,
                        int64_t row_stride, int dtype, hipStream_t stream) {
    if (rows < 0 || inner <= 0 || (inner & 3) || (row_stride & 3) || row_stride < inner)
        return (int)hipErrorInvalidValue;
    if (rows == 0) return 0;
    const int64_t nq = rows * (inner >> 2);
    if (dtype == 1)
        hipLaunchKernelGGL(merge_kernel<true>, dim3(grid_for(nq)), dim3(256), 0, stream, x, mean, snap, rows, inner, row_stride);
    else if (dtype == 0)
        hipLaunchKernelGGL(merge_kernel<false>, dim3(grid_for(nq)), dim3(256), 0, stream, x, mean, snap, rows, inner, row_stride);
    else
        return (int)hipErrorInvalidValue;
    HM_LAUNCH_RET();
}
