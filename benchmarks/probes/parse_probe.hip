// Probe of the device decimal parser (csrc/kernels/parse.h) on gfx950: parses each string of a
// packed buffer with hm::dev_parse_float and reports (ok, value), so a device/host mismatch can
// be pinned to one string.  Built by benchmarks/parse_probe.py.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../csrc/kernels/parse.h"

__global__ void parse_probe_kernel(const uint8_t* buf, const int64_t* off, int n, float* val, int* ok) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = -12345.f;
    ok[i] = hm::dev_parse_float(buf + off[i], (int)(off[i + 1] - off[i]), &v) ? 1 : 0;
    val[i] = v;
}

extern "C" int parse_probe(const uint8_t* buf, const int64_t* off, int n, float* val, int* ok) {
    hipLaunchKernelGGL(parse_probe_kernel, dim3((n + 63) / 64), dim3(64), 0, 0, buf, off, n, val, ok);
    return (int)hipDeviceSynchronize();
}
