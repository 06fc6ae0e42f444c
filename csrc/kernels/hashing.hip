// MurmurHash3_x86_32 / mhash over packed UTF-8 strings on gfx950 (SURVEY.md §2.3.10, K1;
// upstream core/src/main/java/hivemall/utils/hashing/MurmurHash3.java,
// ftvec/hashing/{MurmurHash3UDF,FeatureHashingUDF}.java).
//
// Input: one byte buffer + int64 offsets (string s = buf[off[s] .. off[s+1])).  A 256-thread
// block owns 256 consecutive strings: their bytes are one contiguous span, which the block
// first copies into LDS with coalesced 16-B loads (the span is usually < 8 KB for feature
// names), then every lane hashes its own string from LDS (strings longer than the staged
// window are hashed straight from global memory).  Output = raw hash (uint32) or mhash
// ((int)h % num_features, negatives fixed up, +1) — bit-exact with the Java/C++ versions.
#include "common.h"
#include "murmur3.h"

namespace {

constexpr int HASH_LDS = 16 * 1024;

__global__ __launch_bounds__(256) void mhash_kernel(const uint8_t* __restrict__ buf,
                                                    const int64_t* __restrict__ off, int64_t n,
                                                    uint32_t seed, int32_t num_features,
                                                    int32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t s_buf[HASH_LDS];
    for (int64_t base = (int64_t)blockIdx.x * 256; base < n; base += (int64_t)gridDim.x * 256) {
        const int64_t last = min(n, base + 256);
        const int64_t span0 = off[base], span1 = off[last];
        const int64_t span = span1 - span0;
        const int64_t staged = span < HASH_LDS ? span : HASH_LDS;
        // coalesced staging: 16-B chunks when aligned, bytes at the edges
        const int64_t a0 = (span0 + 15) & ~(int64_t)15;
        const int64_t head = min(a0 - span0, staged);
        for (int64_t i = threadIdx.x; i < head; i += 256) s_buf[i] = buf[span0 + i];
        const int64_t nvec = (staged - head) / 16;
        for (int64_t v = threadIdx.x; v < nvec; v += 256) {
            const uint4 q = *reinterpret_cast<const uint4*>(buf + a0 + 16 * v);
            const int64_t dst = head + 16 * v;
            #pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t w = j == 0 ? q.x : j == 1 ? q.y : j == 2 ? q.z : q.w;
                s_buf[dst + 4 * j] = (uint8_t)w;
                s_buf[dst + 4 * j + 1] = (uint8_t)(w >> 8);
                s_buf[dst + 4 * j + 2] = (uint8_t)(w >> 16);
                s_buf[dst + 4 * j + 3] = (uint8_t)(w >> 24);
            }
        }
        for (int64_t i = head + 16 * nvec + threadIdx.x; i < staged; i += 256) s_buf[i] = buf[span0 + i];
        __syncthreads();
        const int64_t s = base + threadIdx.x;
        if (s < last) {
            const int64_t b = off[s] - span0, e = off[s + 1] - span0;
            const int len = (int)(e - b);
            uint32_t h;
            if (e <= staged) {
                h = hm::murmur3([&](int i) { return s_buf[b + i]; }, len, seed);
            } else {
                const uint8_t* g = buf + span0 + b;
                h = hm::murmur3([&](int i) { return g[i]; }, len, seed);
            }
            if (num_features > 0) {
                int32_t r = (int32_t)h % num_features;
                if (r < 0) r += num_features;
                out[s] = r + 1;
            } else {
                out[s] = (int32_t)h;
            }
        }
        __syncthreads();
    }
}

}  // namespace

// num_features <= 0: raw 32-bit hash; else mhash in [1, num_features].
HM_API int hm_mhash(const uint8_t* buf, const int64_t* off, int64_t n, uint32_t seed,
                    int32_t num_features, int32_t* out, hipStream_t stream) {
    if (n <= 0) return 0;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(mhash_kernel, dim3((int)blocks), dim3(256), 0, stream, buf, off, n, seed,
                       num_features, out);
    HM_LAUNCH_RET();
}
