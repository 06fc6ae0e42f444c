// Where does global_load_lds_dwordx3 (12 B per lane) put each lane's bytes in LDS, and does a
// 16-B LDS-DMA from a 4-B-aligned (not 16-B-aligned) global address return the right bytes?
//   out[0 .. 256)   : the LDS image (dwords) after lane l DMA'd 12 B from src + 12 l
//   out[256 .. 512) : the LDS image after lane l DMA'd 16 B from src + 12 l (4-B aligned)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* glb_ptr_t;

__global__ __launch_bounds__(64) void probe(const uint32_t* __restrict__ src, uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t s[256];
    const int l = threadIdx.x;
    for (int k = l; k < 256; k += 64) s[k] = 0xDEADBEEFu;
    __syncthreads();
    __builtin_amdgcn_global_load_lds((glb_ptr_t)(reinterpret_cast<const char*>(src) + 12 * l), (lds_ptr_t)s, 12, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    for (int k = l; k < 256; k += 64) out[k] = s[k];
    __syncthreads();
    for (int k = l; k < 256; k += 64) s[k] = 0xDEADBEEFu;
    __syncthreads();
    __builtin_amdgcn_global_load_lds((glb_ptr_t)(reinterpret_cast<const char*>(src) + 12 * l), (lds_ptr_t)s, 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    for (int k = l; k < 256; k += 64) out[256 + k] = s[k];
}

extern "C" int hm_probe_lds_dma12(const uint32_t* src, uint32_t* out, hipStream_t st) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, st, src, out);
    return (int)hipGetLastError();
}
