// Small data-plane kernels shared by the learners (gfx950).
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

}  // namespace

HM_API int hm_mark_touched(const int32_t* idx, int64_t n, int32_t dims, uint8_t* flags, hipStream_t stream) {
    if (n <= 0) return 0;
    int64_t blocks = ((n + 3) / 4 + 255) / 256;     // >= 1 for any n > 0
    if (blocks > 2048) blocks = 2048;      // 8 per CU: every CU busy, grid-stride over the rest
    hipLaunchKernelGGL(mark_touched_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, idx, n, dims, flags);
    HM_LAUNCH_RET();
}
