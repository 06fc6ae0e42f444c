// Shared device helpers for the hivemall_amd HIP kernel library (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in csrc/kernels:
//   * wave64: lane = threadIdx.x & 63, all warp-level idioms assume 64 lanes.
//   * Every launcher is an `extern "C" int hm_*(..., hipStream_t)` that returns the
//     hipError_t of the launch (0 = ok); Python checks it and raises.
//   * Launchers never allocate or synchronise (they are hipGraph-capturable).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define HM_WAVE 64

#define HM_API extern "C" __attribute__((visibility("default")))

#define HM_LAUNCH_RET() return (int)hipGetLastError()
#define HM_LAUNCH_RET_IF_ERR() do { const hipError_t e_ = hipGetLastError(); if (e_ != hipSuccess) return (int)e_; } while (0)

namespace hm {

__device__ __forceinline__ int lane_id() { return threadIdx.x & (HM_WAVE - 1); }
__device__ __forceinline__ int wave_id() { return threadIdx.x / HM_WAVE; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, HM_WAVE);
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, HM_WAVE);
    return v;
}
// Full-wave sum on DPP lane permutes (quad_perm x2, row half-mirror, row mirror, row_bcast15,
// row_bcast31), total read from lane 63 -> a wave-uniform value.  ~8 instructions against ~36 for
// the ds_bpermute butterfly of __shfl_xor.  EXEC must be full.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp_take(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xF, false));
}
__device__ __forceinline__ float wave_sum_uniform(float v) {
    v += dpp_take<0xB1>(v);          // quad_perm [1,0,3,2]
    v += dpp_take<0x4E>(v);          // quad_perm [2,3,0,1]
    v += dpp_take<0x141>(v);         // row_half_mirror
    v += dpp_take<0x140>(v);         // row_mirror
    v += dpp_take<0x142, 0xA>(v);    // row_bcast:15 into rows 1, 3
    v += dpp_take<0x143, 0xC>(v);    // row_bcast:31 into rows 2, 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, HM_WAVE));
    return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024). `scratch` needs 16 floats.
// Every thread receives the total.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
    v = wave_sum(v);
    const int nw = blockDim.x / HM_WAVE;
    if (lane_id() == 0) scratch[wave_id()] = v;
    __syncthreads();
    float t = 0.f;
    for (int i = 0; i < nw; ++i) t += scratch[i];
    __syncthreads();
    return t;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

// Numerically safe log(1 + exp(x)) on the hardware exp/log (v_exp_f32 / v_log_f32): per-row
// loss reporting only.  libm's log1pf cost ~40 VALU and enough registers to push the FFM row
// loop into scratch spills; the absolute error here is < 1e-7 (1 + e^x rounds to 1 below
// x ~ -16.6, where the true value is < 6e-8).
__device__ __forceinline__ float log1pexp(float x) {
    const float t = __logf(1.f + __expf(-fabsf(x)));
    return x > 0.f ? x + t : t;
}

__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
    return __uint_as_float(((uint32_t)h) << 16);
}
// Round-to-nearest-even f32 -> bf16 (NaN-preserving path is not needed for weights).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    uint32_t u = __float_as_uint(f);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

// Two floats -> packed bf16x2 with stochastic rounding on gfx950's v_cvt_sr_bf16_f32.
// Bit-identical to the software rule (bits + (r & 0xFFFF)) >> 16 per value: the instruction
// adds the HIGH 16 bits of its random operand (benchmarks/probes/sr_probe.hip: 0 mismatches in
// 2^20 random inputs against that rule), hence the << 16.  One instruction per value instead of
// the and/add/shift/pack sequence (and no Inf/NaN special case to carry by hand).
__device__ __forceinline__ uint32_t pack_bf16x2_sr(float lo, uint32_t r_lo, float hi, uint32_t r_hi) {
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
    bf16x2_t v = {};
    v = __builtin_amdgcn_cvt_sr_bf16_f32(v, lo, r_lo << 16, false);
    v = __builtin_amdgcn_cvt_sr_bf16_f32(v, hi, r_hi << 16, true);
    uint32_t u;
    __builtin_memcpy(&u, &v, 4);
    return u;
}

// Load that bypasses the CU's L1 (agent-scope relaxed atomic load -> `sc1` global load on
// gfx950).  The vector L1 is not coherent with other CUs' stores: a Hogwild kernel whose rows
// are small enough to stay L1-resident would otherwise keep reading its own stale copy of a
// row that other CUs keep updating in L2 for the whole launch.
template <typename T>
__device__ __forceinline__ T ld_coherent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// XCD-aware bijective remap of a flat block id (cdna_hip_programming.md §5, "XCD swizzle
// must be bijective"): consecutive logical tiles land on the same XCD / L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int nx = 8;
    const int xcd = bid % nx;
    const int q = nwg / nx, r = nwg % nx;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + bid / nx;
}

// Counter-based RNG (splitmix64 finaliser) — deterministic per (seed, stream, counter).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ float u01(uint64_t h) {  // [0,1)
    return (float)(h >> 40) * (1.0f / 16777216.0f);
}

}  // namespace hm
