// MurmurHash3_x86_32 for device code (bit-exact with upstream hivemall.utils.hashing.MurmurHash3
// and csrc/host/hashing.cpp): used by the mhash kernel and the device-side feature parsers.
#pragma once
#include <stdint.h>

namespace hm {

__device__ __forceinline__ uint32_t mm_rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

template <typename LoadByte>
__device__ __forceinline__ uint32_t murmur3(LoadByte at, int len, uint32_t seed) {
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    uint32_t h1 = seed;
    const int nblocks = len >> 2;
    for (int i = 0; i < nblocks; ++i) {
        uint32_t k1 = (uint32_t)at(4 * i) | ((uint32_t)at(4 * i + 1) << 8) |
                      ((uint32_t)at(4 * i + 2) << 16) | ((uint32_t)at(4 * i + 3) << 24);
        k1 *= c1; k1 = mm_rotl32(k1, 15); k1 *= c2;
        h1 ^= k1; h1 = mm_rotl32(h1, 13); h1 = h1 * 5 + 0xe6546b64u;
    }
    uint32_t k1 = 0;
    const int t = nblocks * 4;
    switch (len & 3) {
        case 3: k1 ^= (uint32_t)at(t + 2) << 16; [[fallthrough]];
        case 2: k1 ^= (uint32_t)at(t + 1) << 8; [[fallthrough]];
        case 1: k1 ^= (uint32_t)at(t); k1 *= c1; k1 = mm_rotl32(k1, 15); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint32_t)len;
    h1 ^= h1 >> 16; h1 *= 0x85ebca6bu; h1 ^= h1 >> 13; h1 *= 0xc2b2ae35u; h1 ^= h1 >> 16;
    return h1;
}

// Java int % semantics, 1-based (Hivemall mhash)
__device__ __forceinline__ int32_t mhash_reduce(uint32_t h, int32_t num_features) {
    int32_t r = (int32_t)h % num_features;
    if (r < 0) r += num_features;
    return r + 1;
}

}  // namespace hm
