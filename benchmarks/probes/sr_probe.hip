// Probe: does gfx950's v_cvt_sr_bf16_f32 (hardware stochastic rounding f32 -> bf16) equal the
// software rounding used by the FFM/FM kernels ((bits + (rnd & 0xFFFF)) >> 16)?  Prints the
// number of mismatches over random finite inputs for a few ways of feeding the random operand.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

__global__ void probe(const float* x, const uint32_t* r, uint32_t* hw_lo, uint32_t* hw_hi, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    bf16x2 v = {};
    v = __builtin_amdgcn_cvt_sr_bf16_f32(v, x[i], r[i], false);
    uint32_t a;
    __builtin_memcpy(&a, &v, 4);
    hw_lo[i] = a & 0xFFFFu;
    bf16x2 w = {};
    w = __builtin_amdgcn_cvt_sr_bf16_f32(w, x[i], r[i], true);
    uint32_t b;
    __builtin_memcpy(&b, &w, 4);
    hw_hi[i] = b >> 16;
}

int main() {
    const int n = 1 << 20;
    std::mt19937 g(7);
    std::vector<float> x(n);
    std::vector<uint32_t> r(n);
    std::normal_distribution<float> nd(0.f, 1.f);
    for (int i = 0; i < n; ++i) { x[i] = nd(g) * (i % 7 == 0 ? 1e-3f : 1.f); r[i] = g(); }
    float* dx; uint32_t *dr, *dlo, *dhi;
    hipMalloc(&dx, n * 4); hipMalloc(&dr, n * 4); hipMalloc(&dlo, n * 4); hipMalloc(&dhi, n * 4);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dr, r.data(), n * 4, hipMemcpyHostToDevice);
    probe<<<n / 256, 256>>>(dx, dr, dlo, dhi, n);
    std::vector<uint32_t> lo(n), hi(n);
    hipMemcpy(lo.data(), dlo, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hi.data(), dhi, n * 4, hipMemcpyDeviceToHost);
    long m_low16 = 0, m_high16 = 0, m_lohi = 0, up = 0;
    for (int i = 0; i < n; ++i) {
        uint32_t u; __builtin_memcpy(&u, &x[i], 4);
        const uint32_t sw_low = (u + (r[i] & 0xFFFFu)) >> 16;
        const uint32_t sw_high = (u + (r[i] >> 16)) >> 16;
        m_low16 += lo[i] != sw_low;
        m_high16 += lo[i] != sw_high;
        m_lohi += lo[i] != hi[i];
        up += lo[i] != (u >> 16);
    }
    printf("{\"n\": %d, \"mismatch_vs_low16\": %ld, \"mismatch_vs_high16\": %ld, \"lo_vs_hi_dst\": %ld, \"rounded_up\": %ld}\n",
           n, m_low16, m_high16, m_lohi, up);
    return 0;
}
