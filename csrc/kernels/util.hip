// Small data-plane kernels shared by the learners (gfx950).
//
// hm_int_strlen / hm_int_format: decimal text of int64 ids as an Arrow string column (the
// model table's "feature" column of an integer-named string feature, e.g. a feature_hashing
// result).  2.9 M names cost 126 ms through pyarrow's host cast; on the device the lengths, a
// scan and the digits are three small passes plus one D2H of the bytes.
//
// hm_mark_touched: flags[i] = 1 for every valid feature id of a batch (the model table's
// "seen" mask of train_fm / train_ffm).  Replaces a torch pass that widened the ids to int64
// (8 B x nnz), built a mask, compacted it (nonzero) and scattered — ~10 ms per epoch on 2 M
// Criteo rows (profiles/configs_r3/kernel_stats_fm.csv).  Reading the byte first keeps the hot
// features (present in almost every row) from being stored again and again.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void mark_touched_kernel(const int32_t* __restrict__ idx, int64_t n,
                                                            int32_t dims, uint8_t* __restrict__ flags) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
    for (int64_t b = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; b < n; b += stride) {
        int32_t v[4];
        if (b + 3 < n && ((reinterpret_cast<uintptr_t>(idx + b) & 15) == 0)) {
            const int4 q = *reinterpret_cast<const int4*>(idx + b);
            v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = b + u < n ? idx[b + u] : -1;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = (uint32_t)v[u];
            if (i < (uint32_t)dims && flags[i] == 0) flags[i] = 1;
        }
    }
}

__device__ __forceinline__ int dec_len(int64_t v) {
    uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1u : (uint64_t)v;
    int n = 1;
    while (u >= 10u) { u /= 10u; ++n; }
    return n + (v < 0 ? 1 : 0);
}

__global__ __launch_bounds__(256) void int_strlen_kernel(const int64_t* __restrict__ v, int64_t n,
                                                          int32_t* __restrict__ len) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        len[i] = dec_len(v[i]);
}

// off: int32 [n + 1] exclusive offsets (off[0] = 0)
__global__ __launch_bounds__(256) void int_format_kernel(const int64_t* __restrict__ v, int64_t n,
                                                          const int32_t* __restrict__ off, uint8_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = v[i];
        uint64_t u = x < 0 ? (uint64_t)(-(x + 1)) + 1u : (uint64_t)x;
        int e = off[i + 1];
        const int b = off[i];
        do { out[--e] = (uint8_t)('0' + u % 10u); u /= 10u; } while (u);
        if (x < 0 && e > b) out[--e] = (uint8_t)'-';
    }
}

int grid_of(int64_t n) {
    int64_t b = (n + 255) / 256;
    return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

}  // namespace

HM_API int hm_int_strlen(const int64_t* v, int64_t n, int32_t* len, hipStream_t stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(int_strlen_kernel, dim3(grid_of(n)), dim3(256), 0, stream, v, n, len);
    HM_LAUNCH_RET();
}

HM_API int hm_int_format(const int64_t* v, int64_t n, const int32_t* off, uint8_t* out, hipStream_t stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(int_format_kernel, dim3(grid_of(n)), dim3(256), 0, stream, v, n, off, out);
    HM_LAUNCH_RET();
}

HM_API int hm_mark_touched(const int32_t* idx, int64_t n, int32_t dims, uint8_t* flags, hipStream_t stream) {
    if (n <= 0) return 0;
    int64_t blocks = ((n + 3) / 4 + 255) / 256;     // >= 1 for any n > 0
    if (blocks > 2048) blocks = 2048;      // 8 per CU: every CU busy, grid-stride over the rest
    hipLaunchKernelGGL(mark_touched_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, idx, n, dims, flags);
    HM_LAUNCH_RET();
}

