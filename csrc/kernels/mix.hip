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

// 3-level views: element (i0, i1, c) of x at i0 * s0 + i1 * s1 + c, c < inner (inner % 4 == 0):
// the V part of the per-slot FFM feature blocks (fp32: [NF][40][4] in 896-B blocks; bf16:
// [NF][40][4] in 12-B slots of 512-B blocks, so a slot is only 4-B aligned).  ALN: every quad
// of x is 16-B (fp32) / 8-B (bf16) aligned, so it moves as one vector; else as 32-bit words.
template <bool BF, bool ALN>
__device__ __forceinline__ float4 ldx(const void* p, int64_t e) {
    if constexpr (ALN || !BF) {
        if constexpr (ALN) return ld4<BF>(p, e);
        const float* f = reinterpret_cast<const float*>(p) + e;
        return make_float4(f[0], f[1], f[2], f[3]);
    } else {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint16_t*>(p) + e);
        const uint32_t a = w[0], b = w[1];
        return make_float4(__uint_as_float(a << 16), __uint_as_float(a & 0xFFFF0000u),
                           __uint_as_float(b << 16), __uint_as_float(b & 0xFFFF0000u));
    }
}

template <bool BF, bool ALN>
__device__ __forceinline__ void stx(void* p, int64_t e, float4 v) {
    if constexpr (ALN) {
        st4<BF>(p, e, v);
    } else if constexpr (!BF) {
        float* f = reinterpret_cast<float*>(p) + e;
        f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
    } else {
        uint32_t* w = reinterpret_cast<uint32_t*>(reinterpret_cast<uint16_t*>(p) + e);
        w[0] = (uint32_t)hm::f32_to_bf16(v.x) | ((uint32_t)hm::f32_to_bf16(v.y) << 16);
        w[1] = (uint32_t)hm::f32_to_bf16(v.z) | ((uint32_t)hm::f32_to_bf16(v.w) << 16);
    }
}

// Quad q of a [n0][d1][inner] view -> its element offset in x.  The divisions are 32-bit while
// the view has fewer than 2^31 quads (every FFM table below 2^23 features): 64-bit integer division
// is a ~40-instruction software sequence per quad.
__device__ __forceinline__ int64_t view3_elem(int64_t q, int64_t per0, int qps, int64_t s0, int64_t s1, bool small) {
    if (small) {
        const uint32_t uq = (uint32_t)q, up = (uint32_t)per0;
        const uint32_t i0 = uq / up, rem = uq - i0 * up;
        const uint32_t i1 = rem / (uint32_t)qps, c = (rem - i1 * (uint32_t)qps) * 4u;
        return (int64_t)i0 * s0 + (int64_t)i1 * s1 + c;
    }
    const int64_t i0 = q / per0;
    const int64_t rem = q - i0 * per0;
    const int64_t i1 = rem / qps;
    const int c = (int)(rem - i1 * qps) * 4;
    return i0 * s0 + i1 * s1 + c;
}

// MODE 0 (pack):   out[q] = x[view(q)]
// MODE 1 (merge):  x[view(q)] += mean[q] - snap[q]; when out != nullptr also out[q] = the new x
//                  (merge of the finished mix fused with the snapshot of the next one; out may
//                  alias snap: each quad is read before it is written by the same thread)
// MODE 2 (unpack): x[view(q)] = mean[q] (the inverse of pack: bit-exact)
template <int MODE, bool BF, bool ALN>
__global__ __launch_bounds__(256) void view3_kernel(void* __restrict__ x, const void* __restrict__ mean,
                                                    const void* snap, void* out, int64_t n0, int d1,
                                                    int inner, int64_t s0, int64_t s1) {
    const int qps = inner >> 2;
    const int64_t per0 = (int64_t)d1 * qps;
    const int64_t nq = n0 * per0;
    const bool small = nq < ((int64_t)1 << 31);
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += (int64_t)gridDim.x * 256) {
        const int64_t xe = view3_elem(q, per0, qps, s0, s1, small), qe = 4 * q;
        if constexpr (MODE == 2) {
            stx<BF, ALN>(x, xe, ld4<BF>(mean, qe));
            continue;
        }
        float4 a = ldx<BF, ALN>(x, xe);
        if constexpr (MODE == 1) {
            const float4 m = ld4<BF>(mean, qe), sn = ld4<BF>(snap, qe);
            a = make_float4(a.x + (m.x - sn.x), a.y + (m.y - sn.y), a.z + (m.z - sn.z), a.w + (m.w - sn.w));
            if constexpr (BF) {
                // round once here, so x and the next snapshot hold the same bits
                a = make_float4(__uint_as_float((uint32_t)hm::f32_to_bf16(a.x) << 16),
                                __uint_as_float((uint32_t)hm::f32_to_bf16(a.y) << 16),
                                __uint_as_float((uint32_t)hm::f32_to_bf16(a.z) << 16),
                                __uint_as_float((uint32_t)hm::f32_to_bf16(a.w) << 16));
            }
            stx<BF, ALN>(x, xe, a);
            if (out != nullptr) st4<BF>(out, qe, a);
        } else {
            st4<BF>(out, qe, a);
        }
    }
}

// Delta mixing of fp32 (or bf16) replicas over a [n0][d1][inner] view, base = the fp32 consensus
// of the last mix (contiguous, like the wire buffers).  One pass each, no payload-sized
// temporaries (the torch formulation ran 3-5 elementwise passes with fp32 temporaries):
// MODE 2 (pack):          wire[q] <- x[view(q)] - base[q]            (fp32 math, RNE to the wire)
// MODE 3 (merge, sync):   base[q] += m[q];  x[view(q)] <- base[q]    (average_delta)
// MODE 4 (merge, overlap): base[q] += m[q] (rounded to x's dtype);  x += m[q] - sent[q]
//                          (OverlappedMixer delta-sum modes: x keeps its progress since the snapshot)
// XBF: x in bf16; WBF: wire (m, sent) in bf16.  Rounding as torch's copy_ (RNE), so the
// results are bit-identical to the torch formulation.
__device__ __forceinline__ float rne_bf16(float v) {
    return __uint_as_float((uint32_t)hm::f32_to_bf16(v) << 16);
}

template <int MODE, bool XBF, bool WBF, bool ALN>
__global__ __launch_bounds__(256) void delta3_kernel(void* __restrict__ x, float* __restrict__ base,
                                                     void* __restrict__ wire, const void* __restrict__ sent,
                                                     int64_t n0, int d1, int inner, int64_t s0, int64_t s1) {
    const int qps = inner >> 2;
    const int64_t per0 = (int64_t)d1 * qps;
    const int64_t nq = n0 * per0;
    const bool small = nq < ((int64_t)1 << 31);
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += (int64_t)gridDim.x * 256) {
        const int64_t xe = view3_elem(q, per0, qps, s0, s1, small), qe = 4 * q;
        float4 b = *reinterpret_cast<const float4*>(base + qe);
        if constexpr (MODE == 2) {
            const float4 a = ldx<XBF, ALN>(x, xe);
            st4<WBF>(wire, qe, make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w));
        } else {
            const float4 m = ld4<WBF>(wire, qe);
            b = make_float4(b.x + m.x, b.y + m.y, b.z + m.z, b.w + m.w);
            if constexpr (MODE == 3) {
                *reinterpret_cast<float4*>(base + qe) = b;
                stx<XBF, ALN>(x, xe, b);
            } else {
                if constexpr (XBF) b = make_float4(rne_bf16(b.x), rne_bf16(b.y), rne_bf16(b.z), rne_bf16(b.w));
                *reinterpret_cast<float4*>(base + qe) = b;
                const float4 sn = ld4<WBF>(sent, qe);
                const float4 a = ldx<XBF, ALN>(x, xe);
                stx<XBF, ALN>(x, xe, make_float4(a.x + (m.x - sn.x), a.y + (m.y - sn.y), a.z + (m.z - sn.z),
                                                 a.w + (m.w - sn.w)));
            }
        }
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

namespace {
template <int MODE>
int launch_view3(void* x, const void* mean, const void* snap, void* out, int64_t n0, int d1, int inner,
                 int64_t s0, int64_t s1, int dtype, hipStream_t stream) {
    if (n0 < 0 || d1 <= 0 || inner <= 0 || (inner & 3) || s1 < inner || s0 < (int64_t)(d1 - 1) * s1 + inner)
        return (int)hipErrorInvalidValue;
    if (n0 == 0) return 0;
    const int64_t nq = n0 * d1 * (inner >> 2);
    const bool aln = (s0 % 4 == 0) && (s1 % 4 == 0) &&
                     ((uintptr_t)x % (dtype == 1 ? 8 : 16) == 0);
#define HM_V3(BF, ALN) hipLaunchKernelGGL((view3_kernel<MODE, BF, ALN>), dim3(grid_for(nq)), dim3(256), 0, stream, \
                                           x, mean, snap, out, n0, d1, inner, s0, s1)
    if (dtype == 1) {
        if (aln) HM_V3(true, true); else HM_V3(true, false);
    } else if (dtype == 0) {
        if (aln) HM_V3(false, true); else HM_V3(false, false);
    } else {
        return (int)hipErrorInvalidValue;
    }
#undef HM_V3
    HM_LAUNCH_RET();
}
}  // namespace

// x: [n0][d1][inner] view with strides (s0, s1, 1) elements; out: contiguous n0*d1*inner.
HM_API int hm_mix_pack3(const void* x, void* out, int64_t n0, int d1, int inner, int64_t s0, int64_t s1,
                        int dtype, hipStream_t stream) {
    return launch_view3<0>(const_cast<void*>(x), nullptr, nullptr, out, n0, d1, inner, s0, s1, dtype, stream);
}

// x <- mean over the view (mean contiguous n0*d1*inner; bit-exact inverse of hm_mix_pack3).
HM_API int hm_mix_unpack3(void* x, const void* mean, int64_t n0, int d1, int inner, int64_t s0, int64_t s1,
                          int dtype, hipStream_t stream) {
    return launch_view3<2>(x, mean, nullptr, nullptr, n0, d1, inner, s0, s1, dtype, stream);
}

// x += mean - snap over the view; out (nullable, may alias snap) <- the merged x.
HM_API int hm_mix_merge3(void* x, const void* mean, const void* snap, void* out, int64_t n0, int d1, int inner,
                         int64_t s0, int64_t s1, int dtype, hipStream_t stream) {
    return launch_view3<1>(x, mean, snap, out, n0, d1, inner, s0, s1, dtype, stream);
}

// Delta mixing over a view (see delta3_kernel).  mode 2 = pack, 3 = sync merge, 4 = overlapped
// merge; xdtype / wdtype: 0 = fp32, 1 = bf16; base: fp32, contiguous; sent: mode 4 only.
HM_API int hm_mix_delta3(void* x, float* base, void* wire, const void* sent, int64_t n0, int d1, int inner,
                         int64_t s0, int64_t s1, int mode, int xdtype, int wdtype, hipStream_t stream) {
    if (n0 < 0 || d1 <= 0 || inner <= 0 || (inner & 3) || s1 < inner || s0 < (int64_t)(d1 - 1) * s1 + inner ||
        mode < 2 || mode > 4 || (xdtype | wdtype) & ~1 || (mode == 4 && sent == nullptr) ||
        (uintptr_t)base % 16 != 0)
        return (int)hipErrorInvalidValue;
    if (n0 == 0) return 0;
    const int64_t nq = n0 * d1 * (inner >> 2);
    const bool aln = (s0 % 4 == 0) && (s1 % 4 == 0) && ((uintptr_t)x % (xdtype == 1 ? 8 : 16) == 0);
    const int key = mode * 8 + xdtype * 4 + wdtype * 2 + (aln ? 1 : 0);
    const dim3 g(grid_for(nq)), b(256);
#define HM_D3(M, XB, WB, AL) case M * 8 + XB * 4 + WB * 2 + AL: \
        hipLaunchKernelGGL((delta3_kernel<M, (bool)XB, (bool)WB, (bool)AL>), g, b, 0, stream, x, base, wire, sent, \
                           n0, d1, inner, s0, s1); break;
#define HM_D3M(M) HM_D3(M, 0, 0, 0) HM_D3(M, 0, 0, 1) HM_D3(M, 0, 1, 0) HM_D3(M, 0, 1, 1) \
                  HM_D3(M, 1, 0, 0) HM_D3(M, 1, 0, 1) HM_D3(M, 1, 1, 0) HM_D3(M, 1, 1, 1)
    switch (key) {
        HM_D3M(2) HM_D3M(3) HM_D3M(4)
        default: return (int)hipErrorInvalidValue;
    }
#undef HM_D3M
#undef HM_D3
    HM_LAUNCH_RET();
}
