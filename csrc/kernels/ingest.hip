// Device-side ingest of Hivemall feature strings (SURVEY.md §2.5 K1, §3.2 "string -> hash ->
// CSR"; upstream parses per row inside the mapper: hivemall/fm/FFMStringFeatureMapModel,
// ftvec/hashing/FeatureHashingUDF, utils/hashing/MurmurHash3).
//
// The strings arrive as one UTF-8 byte buffer + offsets (an Arrow list<string> column's own
// buffers, uploaded as they are) and are parsed where the model lives:
//   ffm_parse : "field:index[:value]"  -> padded-ELL [B][F] (fld, idx, val) for hm_ffm_step
//   feat_parse: "name[:value]"         -> CSR-ordered (idx, val); names hashed with mhash
//               (mode 2, 1-based) or taken as integers (mode 0)
// One thread per string (per ELL cell for ffm_parse); consecutive threads read adjacent bytes,
// so the byte loads of a wave hit the same few cache lines.  Semantics are those of the host
// parser (csrc/host/hashing.cpp): integer fields / indices, non-integer ones mhash'd, values
// strtod -> float.  A string the device cannot parse (malformed, or a value outside the exact
// decimal fast path below) lowers *err to its index; the caller then re-parses that batch on
// the host, so error messages and corner cases stay the host's.
#include "common.h"
#include "murmur3.h"
#include "parse.h"

namespace {

using hm::dev_parse_float;
using hm::dev_parse_int;
using hm::find_colon;

__global__ __launch_bounds__(256) void ffm_parse_kernel(
    const uint8_t* __restrict__ data, const int64_t* __restrict__ soff,
    const int64_t* __restrict__ loff, int64_t B, int F, int32_t num_features, int32_t num_fields,
    int hash_ints, uint32_t seed, int32_t* __restrict__ fld_out, int32_t* __restrict__ idx_out,
    float* __restrict__ val_out, unsigned long long* __restrict__ err) {
    const int64_t cells = B * (int64_t)F;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < cells; t += (int64_t)gridDim.x * 256) {
        const int64_t row = t / F;
        const int slot = (int)(t - row * F);
        const int64_t s = loff[row] + slot;
        int32_t fo = 0, io = -1;
        float vo = 0.f;
        if (s < loff[row + 1]) {
            const uint8_t* p = data + soff[s];
            const int len = (int)(soff[s + 1] - soff[s]);
            bool ok = true;
            const int c1 = find_colon(p, len, 0);
            if (c1 <= 0 || c1 + 1 >= len) ok = false;
            int64_t f = 0, id = 0;
            float v = 1.f;
            if (ok) {
                const int c2 = find_colon(p, len, c1 + 1);
                const int ilen = (c2 < 0 ? len : c2) - c1 - 1;
                if (c2 >= 0 && !dev_parse_float(p + c2 + 1, len - c2 - 1, &v)) ok = false;
                if (!dev_parse_int(p, c1, &f))
                    f = hm::mhash_reduce(hm::murmur3([&](int i) { return p[i]; }, c1, seed), num_fields) - 1;
                if (f < 0 || f >= num_fields || ilen <= 0) ok = false;
                const uint8_t* q = p + c1 + 1;
                if (ok && dev_parse_int(q, ilen, &id)) {
                    if (hash_ints) {
                        id %= num_features;
                        if (id < 0) id += num_features;
                    } else if (id < 0 || id >= num_features) {
                        ok = false;
                    }
                } else if (ok) {
                    id = hm::mhash_reduce(hm::murmur3([&](int i) { return q[i]; }, ilen, seed), num_features) - 1;
                }
            }
            if (ok) {
                fo = (int32_t)f;
                io = (int32_t)id;
                vo = v;
            } else {
                atomicMin(err, (unsigned long long)s);
            }
        }
        fld_out[t] = fo;
        idx_out[t] = io;
        val_out[t] = vo;
    }
}

// mode 0: integer names; mode 2: mhash(name, num_features) (1-based).  OFF: the string
// offsets' type (Arrow string: int32, large_string / rebased chunks: int64)
template <typename OFF>
__global__ __launch_bounds__(256) void feat_parse_kernel(
    const uint8_t* __restrict__ data, const OFF* __restrict__ soff, int64_t n, int mode,
    int32_t num_features, uint32_t seed, int64_t* __restrict__ idx_out, float* __restrict__ val_out,
    unsigned long long* __restrict__ err) {
    for (int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x; s < n; s += (int64_t)gridDim.x * 256) {
        const uint8_t* p = data + soff[s];
        const int len = (int)(soff[s + 1] - soff[s]);
        const int c = find_colon(p, len, 0);
        const int nlen = c < 0 ? len : c;
        float v = 1.f;
        bool ok = nlen > 0;
        if (c >= 0 && !dev_parse_float(p + c + 1, len - c - 1, &v)) ok = false;
        int64_t id = 0;
        if (ok) {
            if (mode == 2) id = hm::mhash_reduce(hm::murmur3([&](int i) { return p[i]; }, nlen, seed), num_features);
            else ok = dev_parse_int(p, nlen, &id);
        }
        if (!ok) {
            atomicMin(err, (unsigned long long)s);
            id = 0;
            v = 0.f;
        }
        idx_out[s] = id;
        val_out[s] = v;
    }
}

int blocks_for(int64_t n) {
    const int64_t b = (n + 255) / 256;
    return (int)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

}  // namespace

// Arrow-layout FFM rows -> padded ELL [B][F].  soff: int64 [n_strings + 1] byte offsets into
// data; loff: int64 [B + 1] string offsets per row.  *err (host-initialised to ~0ull) receives
// the smallest index of a string the device could not parse.
HM_API int hm_ffm_parse(const uint8_t* data, const int64_t* soff, const int64_t* loff, int64_t B, int F,
                        int32_t num_features, int32_t num_fields, int hash_ints, uint32_t seed,
                        int32_t* fld, int32_t* idx, float* val, unsigned long long* err, hipStream_t stream) {
    if (B <= 0) return 0;
    if (F <= 0 || num_features <= 0 || num_fields <= 0) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(ffm_parse_kernel, dim3(blocks_for(B * (int64_t)F)), dim3(256), 0, stream, data, soff, loff,
                       B, F, num_features, num_fields, hash_ints, seed, fld, idx, val, err);
    HM_LAUNCH_RET();
}

HM_API int hm_feat_parse(const uint8_t* data, const int64_t* soff, int64_t n, int mode, int32_t num_features,
                         uint32_t seed, int64_t* idx, float* val, unsigned long long* err, hipStream_t stream) {
    if (n <= 0) return 0;
    if ((mode != 0 && mode != 2) || (mode == 2 && num_features <= 0)) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(feat_parse_kernel<int64_t>, dim3(blocks_for(n)), dim3(256), 0, stream, data, soff, n, mode,
                       num_features, seed, idx, val, err);
    HM_LAUNCH_RET();
}

// hm_feat_parse with int32 string offsets (an Arrow string column's own offsets, no widening)
HM_API int hm_feat_parse32(const uint8_t* data, const int32_t* soff, int64_t n, int mode, int32_t num_features,
                           uint32_t seed, int64_t* idx, float* val, unsigned long long* err, hipStream_t stream) {
    if (n <= 0) return 0;
    if ((mode != 0 && mode != 2) || (mode == 2 && num_features <= 0)) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(feat_parse_kernel<int32_t>, dim3(blocks_for(n)), dim3(256), 0, stream, data, soff, n, mode,
                       num_features, seed, idx, val, err);
    HM_LAUNCH_RET();
}
