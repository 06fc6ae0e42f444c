// LDS atomic throughput probe (gfx950): lane-ops per CU-cycle for the histogram update forms
// the tree kernel could use.  Each block: 256 threads, 48 KB LDS image, ITERS updates/thread.
//   hipcc --offload-arch=gfx950 -O3 benchmarks/probes/lds_atomic_probe.hip -o benchmarks/probes/lds_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 4096;
constexpr int NB = 12288;  // 48 KB of 4-byte counters

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x;
}

template <int MODE>
__global__ __launch_bounds__(256) void probe(float* out, int spread) {
    __shared__ float sf[NB];
    uint32_t* su = reinterpret_cast<uint32_t*>(sf);
    for (int i = threadIdx.x; i < NB; i += 256) sf[i] = 0.f;
    __syncthreads();
    uint32_t s = hsh(blockIdx.x * 256 + threadIdx.x);
    const float v = 1.0f + threadIdx.x * 1e-3f;
    for (int it = 0; it < ITERS; ++it) {
        s = s * 1664525u + 1013904223u;
        int a;
        if (spread == 0) a = threadIdx.x;                              // distinct, lane-linear
        else a = ((s >> 8) % spread) + (it % 48) * 256;              // random bin of one feature row
        if (MODE == 0) atomicAdd(&sf[a], v);                          // ds_add_f32
        else if (MODE == 1) atomicAdd(&su[a], (uint32_t)(s & 0xff));  // ds_add_u32
        else if (MODE == 2) sf[a] += v;                               // plain RMW (racy: throughput bound only)
        else if (MODE == 3) {                                          // ds_add_u64: two packed sums per op
            const int a2 = spread == 0 ? threadIdx.x : ((s >> 8) % spread) + (it % 24) * 256;
            atomicAdd(reinterpret_cast<unsigned long long*>(su) + a2, (unsigned long long)(s & 0xff) << 32 | 3ull);
        }
    }
    __syncthreads();
    float acc = 0.f;
    for (int i = threadIdx.x; i < NB; i += 256) acc += sf[i];
    if (acc == 12345.f) out[0] = acc;
}

int main() {
    float* out;
    hipMalloc(&out, 4);
    int cus = 256;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    cus = p.multiProcessorCount;
    const double clk = p.clockRate * 1e3;
    const int blocks = cus * 3 * 8;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[] = {"ds_add_f32", "ds_add_u32", "ld/st RMW", "ds_add_u64"};
    for (int mode = 0; mode < 4; ++mode) {
        for (int spread : {0, 256, 64}) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(a);
                if (mode == 0) hipLaunchKernelGGL(probe<0>, blocks, 256, 0, 0, out, spread);
                if (mode == 1) hipLaunchKernelGGL(probe<1>, blocks, 256, 0, 0, out, spread);
                if (mode == 2) hipLaunchKernelGGL(probe<2>, blocks, 256, 0, 0, out, spread);
                if (mode == 3) hipLaunchKernelGGL(probe<3>, blocks, 256, 0, 0, out, spread);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                const double ops = (double)blocks * 256 * ITERS;
                if (rep) printf("{\"op\": \"%s\", \"spread\": %d, \"ms\": %.3f, \"Glane_ops_per_s\": %.1f, \"per_CU_clk\": %.2f}\n",
                                names[mode], spread, ms, ops / ms / 1e6, ops / (ms * 1e-3) / cus / clk);
            }
        }
    }
    return 0;
}
