// Host-side hashing + feature-string data plane (C ABI, loaded via ctypes).
//
// * MurmurHash3_x86_32 over UTF-8 bytes.  Hivemall's hivemall.utils.hashing.MurmurHash3
//   (core/src/main/java/hivemall/utils/hashing/MurmurHash3.java) hashes the
//   UTF-8 encoding of a CharSequence with seed 0x9747b28c; `mhash` reduces it modulo
//   num_features (default 2^24), fixes up negatives and returns a value starting from 1.
// * Feature strings "name:value" / "name" / "field:index:value" are parsed here so the
//   Python layer never loops over individual features.
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#define HM_API extern "C" __attribute__((visibility("default")))

namespace {

inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

uint32_t murmur3_x86_32(const uint8_t* data, int len, uint32_t seed) {
    const int nblocks = len / 4;
    uint32_t h1 = seed;
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    for (int i = 0; i < nblocks; ++i) {
        uint32_t k1;
        std::memcpy(&k1, data + 4 * i, 4);  // little-endian host
        k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2;
        h1 ^= k1; h1 = rotl32(h1, 13); h1 = h1 * 5 + 0xe6546b64u;
    }
    const uint8_t* tail = data + nblocks * 4;
    uint32_t k1 = 0;
    switch (len & 3) {
        case 3: k1 ^= (uint32_t)tail[2] << 16; [[fallthrough]];
        case 2: k1 ^= (uint32_t)tail[1] << 8; [[fallthrough]];
        case 1: k1 ^= tail[0]; k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint32_t)len;
    h1 ^= h1 >> 16; h1 *= 0x85ebca6bu; h1 ^= h1 >> 13; h1 *= 0xc2b2ae35u; h1 ^= h1 >> 16;
    return h1;
}

inline int32_t mhash_reduce(uint32_t h, int32_t num_features) {
    int32_t r = (int32_t)h % num_features;  // Java int % semantics
    if (r < 0) r += num_features;
    return r + 1;
}

// Strict integer parse of [p, p+n) ; returns false if not an integer literal.
bool parse_int(const char* p, int n, int64_t* out) {
    if (n <= 0 || n > 19) return false;
    int i = 0;
    bool neg = false;
    if (p[0] == '-' || p[0] == '+') { neg = p[0] == '-'; i = 1; if (n == 1) return false; }
    int64_t v = 0;
    for (; i < n; ++i) {
        const char c = p[i];
        if (c < '0' || c > '9') return false;
        v = v * 10 + (c - '0');
    }
    *out = neg ? -v : v;
    return true;
}

bool parse_float(const char* p, int n, float* out) {
    if (n <= 0 || n > 63) return false;
    {
        // exact fast path: [+-]digits[.digits] with <= 15 significant digits is m / 10^f with
        // m < 2^53 and f <= 15, both exact in double, so the one IEEE division is the correctly
        // rounded value strtod returns; anything else (exponents, inf/nan, spaces) -> strtod
        static const double P10[16] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10,
                                       1e11, 1e12, 1e13, 1e14, 1e15};
        int i = 0;
        bool neg = false;
        if (p[0] == '-' || p[0] == '+') { neg = p[0] == '-'; i = 1; }
        uint64_t m = 0;
        int nd = 0, fd = -1;
        bool ok = i < n;
        for (; i < n && ok; ++i) {
            const char c = p[i];
            if (c >= '0' && c <= '9') {
                m = m * 10 + (uint64_t)(c - '0');
                ++nd;
                if (fd >= 0) ++fd;
            } else if (c == '.' && fd < 0) {
                fd = 0;
            } else {
                ok = false;
            }
        }
        if (ok && nd > 0 && nd <= 15) {
            const double d = fd > 0 ? (double)m / P10[fd] : (double)m;
            *out = (float)(neg ? -d : d);
            return true;
        }
    }
    char tmp[64];
    std::memcpy(tmp, p, n);
    tmp[n] = 0;
    char* end = nullptr;
    const double d = std::strtod(tmp, &end);
    if (end != tmp + n) return false;
    *out = (float)d;
    return true;
}

struct Dict {
    std::unordered_map<std::string, int64_t> map;
    std::vector<std::string> keys;
    int64_t encode(std::string_view s, bool add) {
        auto it = map.find(std::string(s));
        if (it != map.end()) return it->second;
        if (!add) return -1;
        const int64_t id = (int64_t)keys.size();
        keys.emplace_back(s);
        map.emplace(keys.back(), id);
        return id;
    }
};

}  // namespace

HM_API uint32_t hm_murmur3(const uint8_t* data, int len, uint32_t seed) {
    return murmur3_x86_32(data, len, seed);
}

HM_API void hm_murmur3_batch(const uint8_t* buf, const int64_t* off, int64_t n, uint32_t seed,
                             uint32_t* out) {
#pragma omp parallel for schedule(static) if (n > 65536)
    for (int64_t i = 0; i < n; ++i)
        out[i] = murmur3_x86_32(buf + off[i], (int)(off[i + 1] - off[i]), seed);
}

HM_API void hm_mhash_batch(const uint8_t* buf, const int64_t* off, int64_t n, uint32_t seed,
                           int32_t num_features, int32_t* out) {
#pragma omp parallel for schedule(static) if (n > 65536)
    for (int64_t i = 0; i < n; ++i)
        out[i] = mhash_reduce(murmur3_x86_32(buf + off[i], (int)(off[i + 1] - off[i]), seed),
                              num_features);
}

// ---------------------------------------------------------------- dictionary
// feature_hashing over packed feature strings (ftvec/functions.py feature_hashing, vectorised):
// "name" -> "h", "name:v" -> "h:v", "field:index:v" -> "h:v" with h = mhash(name) (the name is
// everything before the LAST of at most two ':' separators, as the per-row UDF's _split).  The
// value text is copied verbatim.  out needs off[n] + 11 * n bytes; out_off gets n + 1 offsets;
// returns the bytes written.  Two passes (lengths, then a parallel fill) keep it O(bytes).
// decimal text of a signed 32-bit int (no locale, no format parsing); returns the length
inline int fmt_i32(int32_t v, char* o) {
    char t[12];
    uint32_t u = v < 0 ? 0u - (uint32_t)v : (uint32_t)v;
    int n = 0;
    do { t[n++] = (char)('0' + u % 10); u /= 10; } while (u);
    int k = 0;
    if (v < 0) o[k++] = '-';
    while (n) o[k++] = t[--n];
    return k;
}

// name length of a feature string (before the last of at most two ':'), -1 in *has_val when
// there is no value part
inline int feature_name_len(const uint8_t* p, int L, bool* has_val) {
    const void* a = std::memchr(p, ':', (size_t)L);
    if (!a) { *has_val = false; return L; }
    *has_val = true;
    const int c1 = (int)((const uint8_t*)a - p);
    const void* b = std::memchr(p + c1 + 1, ':', (size_t)(L - c1 - 1));
    return b ? (int)((const uint8_t*)b - p) : c1;
}

inline int dec_digits(uint32_t u) {
    int d = 1;
    while (u >= 10) { u /= 10; ++d; }
    return d;
}

// Exclusive prefix sum in place over out[1..n] (out[0] = 0 on return), parallel in blocks.
void prefix_sum_inplace(int64_t* out, int64_t n) {
    out[0] = 0;
    if (n < (1 << 20)) {
        for (int64_t i = 0; i < n; ++i) out[i + 1] += out[i];
        return;
    }
    constexpr int NB = 64;
    int64_t part[NB + 1] = {0};
#pragma omp parallel for schedule(static)
    for (int b = 0; b < NB; ++b) {
        const int64_t s = n * b / NB + 1, e = n * (b + 1) / NB + 1;
        int64_t acc = 0;
        for (int64_t i = s; i < e; ++i) { acc += out[i]; out[i] = acc; }
        part[b + 1] = acc;
    }
    for (int b = 0; b < NB; ++b) part[b + 1] += part[b];
#pragma omp parallel for schedule(static)
    for (int b = 1; b < NB; ++b) {
        const int64_t s = n * b / NB + 1, e = n * (b + 1) / NB + 1;
        for (int64_t i = s; i < e; ++i) out[i] += part[b];
    }
}

HM_API int64_t hm_feature_hash_strs(const uint8_t* buf, const int64_t* off, int64_t n,
                                    int32_t num_features, uint32_t seed, uint8_t* out,
                                    int64_t* out_off) {
    // pass 1: output length of each string into out_off[i + 1]; pass 2 re-hashes and writes.
    // Hashing a ~10-B name twice is cheaper than first-touching three n-sized temporaries
    // (the page faults of those cost more than the whole parallel pass).
#pragma omp parallel for schedule(static) if (n > 65536)
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t* p = buf + off[i];
        const int L = (int)(off[i + 1] - off[i]);
        bool hv;
        const int nl = feature_name_len(p, L, &hv);
        const int32_t h = mhash_reduce(murmur3_x86_32(p, nl, seed), num_features);   // >= 1
        out_off[i + 1] = dec_digits((uint32_t)h) + (hv ? L - nl : 0);
    }
    prefix_sum_inplace(out_off, n);
#pragma omp parallel for schedule(static) if (n > 65536)
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t* p = buf + off[i];
        const int L = (int)(off[i + 1] - off[i]);
        bool hv;
        const int nl = feature_name_len(p, L, &hv);
        uint8_t* o = out + out_off[i];
        const int hd = fmt_i32(mhash_reduce(murmur3_x86_32(p, nl, seed), num_features),
                               reinterpret_cast<char*>(o));
        if (hv) {
            o[hd] = ':';
            std::memcpy(o + hd + 1, p + nl + 1, L - nl - 1);
        }
    }
    return out_off[n];
}

// list<string> rows with one constant string appended to every valid row (add_bias): new string
// buffer + string offsets + row offsets in one pass.  valid may be null (every row valid);
// out needs off[row_off[n]] + n * clen bytes, out_off row_off[n] + n + 1, out_row n + 1.
HM_API int64_t hm_list_append_str(const uint8_t* buf, const int64_t* off, const int64_t* row_off,
                                  const uint8_t* valid, int64_t n, const uint8_t* cstr, int32_t clen,
                                  uint8_t* out, int64_t* out_off, int64_t* out_row) {
    int64_t s = 0, b = 0;
    out_off[0] = 0;
    for (int64_t r = 0; r < n; ++r) {
        out_row[r] = s;
        const int64_t a0 = row_off[r], a1 = row_off[r + 1];
        const int64_t nb = off[a1] - off[a0];
        std::memcpy(out + b, buf + off[a0], (size_t)nb);
        for (int64_t k = a0; k < a1; ++k) out_off[s + (k - a0) + 1] = b + (off[k + 1] - off[a0]);
        s += a1 - a0;
        b += nb;
        if (!valid || valid[r]) {
            std::memcpy(out + b, cstr, (size_t)clen);
            b += clen;
            out_off[++s] = b;
        }
    }
    out_row[n] = s;
    return b;
}

HM_API void* hm_dict_new() { return new Dict(); }
HM_API void hm_dict_free(void* d) { delete static_cast<Dict*>(d); }
HM_API int64_t hm_dict_size(void* d) { return (int64_t)static_cast<Dict*>(d)->keys.size(); }
HM_API void hm_dict_encode(void* d, const uint8_t* buf, const int64_t* off, int64_t n, int add,
                           int64_t* out) {
    Dict* D = static_cast<Dict*>(d);
    for (int64_t i = 0; i < n; ++i)
        out[i] = D->encode(std::string_view((const char*)buf + off[i], (size_t)(off[i + 1] - off[i])), add != 0);
}
// Two-phase dump: call with buf=null to get total bytes; then with buffers.
HM_API int64_t hm_dict_dump(void* d, uint8_t* buf, int64_t* off) {
    Dict* D = static_cast<Dict*>(d);
    int64_t tot = 0;
    for (auto& k : D->keys) tot += (int64_t)k.size();
    if (!buf) return tot;
    int64_t p = 0;
    for (size_t i = 0; i < D->keys.size(); ++i) {
        off[i] = p;
        std::memcpy(buf + p, D->keys[i].data(), D->keys[i].size());
        p += (int64_t)D->keys[i].size();
    }
    off[D->keys.size()] = p;
    return tot;
}

// ---------------------------------------------------------------- feature parsing
// mode 0: names must be integers (returned as-is)
// mode 1: names dictionary-encoded through `dict` (new names added when add_new)
// mode 2: names hashed with mhash(name, num_features) (1-based)
// mode 3: integer names kept, non-integer names dictionary-encoded and offset by int_base
// Returns -1 on success, else the index of the first malformed feature.
HM_API int64_t hm_parse_features(const uint8_t* buf, const int64_t* off, int64_t n, int mode,
                                 void* dict, int add_new, int32_t num_features, uint32_t seed,
                                 int64_t int_base, int64_t* idx_out, float* val_out) {
    Dict* D = static_cast<Dict*>(dict);
    if (mode == 0 || mode == 2) {
        // no dictionary: every feature parses on its own -> parallel; the first malformed
        // feature (lowest index) is reported as in the sequential loop
        int64_t bad = n;
#pragma omp parallel for schedule(static) reduction(min : bad) if (n > 65536)
        for (int64_t i = 0; i < n; ++i) {
            const char* s = (const char*)buf + off[i];
            const int len = (int)(off[i + 1] - off[i]);
            const char* colon = (const char*)std::memchr(s, ':', (size_t)len);
            int nlen = len;
            float v = 1.f;
            if (colon) {
                nlen = (int)(colon - s);
                if (!parse_float(colon + 1, len - nlen - 1, &v)) { bad = i < bad ? i : bad; continue; }
            }
            if (nlen <= 0) { bad = i < bad ? i : bad; continue; }
            int64_t id;
            if (mode == 0) {
                if (!parse_int(s, nlen, &id)) { bad = i < bad ? i : bad; continue; }
            } else {
                id = mhash_reduce(murmur3_x86_32((const uint8_t*)s, nlen, seed), num_features);
            }
            idx_out[i] = id;
            val_out[i] = v;
        }
        return bad < n ? bad : -1;
    }
    for (int64_t i = 0; i < n; ++i) {
        const char* s = (const char*)buf + off[i];
        const int len = (int)(off[i + 1] - off[i]);
        const char* colon = (const char*)std::memchr(s, ':', (size_t)len);
        int nlen = len;
        float v = 1.f;
        if (colon) {
            nlen = (int)(colon - s);
            if (!parse_float(colon + 1, len - nlen - 1, &v)) return i;
        }
        if (nlen <= 0) return i;
        int64_t id;
        switch (mode) {
            case 0:
                if (!parse_int(s, nlen, &id)) return i;
                break;
            case 1:
                id = D->encode(std::string_view(s, (size_t)nlen), add_new != 0);
                break;
            case 2:
                id = mhash_reduce(murmur3_x86_32((const uint8_t*)s, nlen, seed), num_features);
                break;
            default:
                if (!parse_int(s, nlen, &id)) {
                    id = D->encode(std::string_view(s, (size_t)nlen), add_new != 0);
                    if (id >= 0) id += int_base;
                }
        }
        idx_out[i] = id;
        val_out[i] = v;
    }
    return -1;
}

// FFM features "field:index[:value]".  field: integer (or mhash'd into num_fields when not
// an integer); index: integer (mod num_features when hash_ints) or mhash'd into num_features.
HM_API int64_t hm_parse_ffm_features(const uint8_t* buf, const int64_t* off, int64_t n,
                                     int32_t num_features, int32_t num_fields, int hash_ints,
                                     uint32_t seed, int32_t* fld_out, int32_t* idx_out,
                                     float* val_out) {
    for (int64_t i = 0; i < n; ++i) {
        const char* s = (const char*)buf + off[i];
        const int len = (int)(off[i + 1] - off[i]);
        const char* c1 = (const char*)std::memchr(s, ':', (size_t)len);
        if (!c1) return i;
        const int flen = (int)(c1 - s);
        const char* rest = c1 + 1;
        const int rlen = len - flen - 1;
        const char* c2 = (const char*)std::memchr(rest, ':', (size_t)rlen);
        const int ilen = c2 ? (int)(c2 - rest) : rlen;
        float v = 1.f;
        if (c2 && !parse_float(c2 + 1, rlen - ilen - 1, &v)) return i;
        int64_t f, id;
        if (!parse_int(s, flen, &f)) {
            if (flen <= 0) return i;
            f = mhash_reduce(murmur3_x86_32((const uint8_t*)s, flen, seed), num_fields) - 1;
        }
        if (f < 0 || f >= num_fields) return i;
        if (ilen <= 0) return i;
        if (parse_int(rest, ilen, &id)) {
            if (hash_ints) {
                id %= num_features;
                if (id < 0) id += num_features;
            } else if (id < 0 || id >= num_features) {
                return i;
            }
        } else {
            id = mhash_reduce(murmur3_x86_32((const uint8_t*)rest, ilen, seed), num_features) - 1;
        }
        fld_out[i] = (int32_t)f;
        idx_out[i] = (int32_t)id;
        val_out[i] = v;
    }
    return -1;
}

// ---------------------------------------------------------------- int64 open-addressing probe
// Bulk probe of utils/collections._OpenHashTable (power-of-two table of int64 keys, INT64_MIN =
// empty, splitmix64 slot, linear probing): out[i] = slot of keys[i] (-1 when absent and not
// inserting).  insert != 0: absent keys claim the first empty slot of their probe sequence, in
// input order (sequential; returns the number inserted); lookups run in parallel.
static inline uint64_t oht_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

HM_API int64_t hm_oht_probe(int64_t* table, int64_t cap, const int64_t* keys, int64_t n, int64_t* out,
                            int insert) {
    const int64_t empty = INT64_MIN;
    const uint64_t mask = (uint64_t)cap - 1;
    if (insert) {
        int64_t added = 0;
        for (int64_t i = 0; i < n; ++i) {
            const int64_t k = keys[i];
            uint64_t h = oht_mix64((uint64_t)k) & mask;
            while (table[h] != k && table[h] != empty) h = (h + 1) & mask;
            if (table[h] == empty) {
                table[h] = k;
                ++added;
            }
            out[i] = (int64_t)h;
        }
        return added;
    }
#pragma omp parallel for schedule(static) if (n > 65536)
    for (int64_t i = 0; i < n; ++i) {
        const int64_t k = keys[i];
        uint64_t h = oht_mix64((uint64_t)k) & mask;
        int64_t r = -1;
        for (;;) {
            const int64_t t = table[h];
            if (t == k) { r = (int64_t)h; break; }
            if (t == empty) break;
            h = (h + 1) & mask;
        }
        out[i] = r;
    }
    return 0;
}

// Lookup straight to values for int64-valued tables (Int2LongOpenHashTable.get_many): out[i] =
// vals[slot of keys[i]], or dflt when absent.
HM_API void hm_oht_get_i64(const int64_t* table, const int64_t* vals, int64_t cap, const int64_t* keys,
                           int64_t n, int64_t dflt, int64_t* out) {
    const int64_t empty = INT64_MIN;
    const uint64_t mask = (uint64_t)cap - 1;
#pragma omp parallel for schedule(static) if (n > 65536)
    for (int64_t i = 0; i < n; ++i) {
        const int64_t k = keys[i];
        uint64_t h = oht_mix64((uint64_t)k) & mask;
        int64_t r = dflt;
        for (;;) {
            const int64_t t = table[h];
            if (t == k) { r = vals[h]; break; }
            if (t == empty) break;
            h = (h + 1) & mask;
        }
        out[i] = r;
    }
}

// ---------------------------------------------------------------- add_feature_index
// Text of a feature value as ftvec/functions.py _fmt writes it: integral |v| <= 1e15 as "%.1f",
// anything else as Python's repr(float) — the shortest round-trip digits (std::to_chars, as
// Python's dtoa), in fixed notation when the decimal exponent is in [-4, 16), else "d.ddde+XX".
// Returns the length written to o (o needs 32 bytes); v must be finite.
int fmt_py_float(double v, char* o) {
    if (v == std::trunc(v) && std::fabs(v) <= 1e15) {
        char t[40];                                       // snprintf's NUL must not land in o
        const int n = std::snprintf(t, sizeof(t), "%.1f", v);
        std::memcpy(o, t, (size_t)n);
        return n;
    }
    char sci[32];
    auto r = std::to_chars(sci, sci + sizeof(sci), v, std::chars_format::scientific);
    const int sl = (int)(r.ptr - sci);
    const char* e = (const char*)std::memchr(sci, 'e', (size_t)sl);
    int ex = 0;                                           // value = d.ddd x 10^ex
    for (const char* q = e + 2; q < sci + sl; ++q) ex = ex * 10 + (*q - '0');
    if (e[1] == '-') ex = -ex;
    if (ex < -4 || ex >= 16) {
        std::memcpy(o, sci, (size_t)sl);
        return sl;
    }
    auto f = std::to_chars(o, o + 32, v, std::chars_format::fixed);
    int n = (int)(f.ptr - o);
    if (!std::memchr(o, '.', (size_t)n)) { o[n++] = '.'; o[n++] = '0'; }
    return n;
}

// add_feature_index over a list<double> column: row r's values vals[row_off[r] .. row_off[r+1])
// -> strings "<position + 1>:<value>", null values (valid[k] == 0) skipped with their position
// kept.  Two calls: out == nullptr returns the total bytes and fills out_off's lengths; then the
// bytes.  out_off has row_off[n] + 1 entries (strings of skipped values are empty and dropped by
// the caller through keep); returns -2 - k when value k is not finite (the per-row path raises).
HM_API int64_t hm_format_feature_index(const double* vals, const uint8_t* valid,
                                       const int64_t* row_off, int64_t n_rows, uint8_t* out,
                                       int64_t* out_off) {
    const int64_t nv = row_off[n_rows] - row_off[0];
    int64_t bad = nv;
    if (!out) {
#pragma omp parallel for schedule(static) reduction(min : bad) if (n_rows > 4096)
        for (int64_t r = 0; r < n_rows; ++r) {
            char tmp[48];
            for (int64_t k = row_off[r]; k < row_off[r + 1]; ++k) {
                const int64_t q = k - row_off[0];
                if (valid && !valid[q]) { out_off[q + 1] = 0; continue; }
                if (!std::isfinite(vals[q])) { bad = q < bad ? q : bad; out_off[q + 1] = 0; continue; }
                const int pos = (int)(k - row_off[r]) + 1;
                out_off[q + 1] = dec_digits((uint32_t)pos) + 1 + fmt_py_float(vals[q], tmp);
            }
        }
        if (bad < nv) return -2 - bad;
        prefix_sum_inplace(out_off, nv);
        return out_off[nv];
    }
#pragma omp parallel for schedule(static) if (n_rows > 4096)
    for (int64_t r = 0; r < n_rows; ++r) {
        for (int64_t k = row_off[r]; k < row_off[r + 1]; ++k) {
            const int64_t q = k - row_off[0];
            if (out_off[q + 1] == out_off[q]) continue;
            char* o = reinterpret_cast<char*>(out + out_off[q]);
            const int hd = fmt_i32((int32_t)(k - row_off[r]) + 1, o);
            o[hd] = ':';
            fmt_py_float(vals[q], o + hd + 1);
        }
    }
    return out_off[nv];
}

// ---------------------------------------------------------------- l1 / l2_normalize
// Python float() of a value text, for the plain forms only ([+-]digits[.digits][e[+-]digits]):
// strtod of those is the correctly rounded double, as float() is; anything else (spaces,
// underscores, inf / nan words, hex) returns false and the caller takes the per-row path.
bool parse_plain_double(const char* p, int n, double* out) {
    if (n <= 0 || n > 63) return false;
    for (int i = 0; i < n; ++i) {
        const char c = p[i];
        if (!((c >= '0' && c <= '9') || c == '.' || c == '-' || c == '+' || c == 'e' || c == 'E')) return false;
    }
    char tmp[64];
    std::memcpy(tmp, p, (size_t)n);
    tmp[n] = 0;
    char* end = nullptr;
    *out = std::strtod(tmp, &end);
    return end == tmp + n;
}

// ftvec/functions.py _normalize over a list<string> column: per row, every "name:value" is
// split as _split does, the values' L1 (p = 1) or L2 (p = 2) norm is summed left to right in
// double, and each feature becomes "name:" + repr(value / norm); a row whose norm is 0 is
// copied verbatim.  Two calls as hm_format_feature_index (out == nullptr: lengths + total).
// Returns -2 - k when string k needs the per-row path (unparsable / non-finite).
HM_API int64_t hm_normalize_features(const uint8_t* buf, const int64_t* off, const int64_t* row_off,
                                     int64_t n_rows, int p, uint8_t* out, int64_t* out_off,
                                     double* norm) {
    const int64_t ns = row_off[n_rows] - row_off[0];
    auto split = [&](int64_t q, int* nl, double* v) -> bool {
        const char* s = (const char*)buf + off[q];
        const int L = (int)(off[q + 1] - off[q]);
        bool hv;
        *nl = feature_name_len((const uint8_t*)s, L, &hv);
        if (!hv) { *v = 1.0; return true; }
        return parse_plain_double(s + *nl + 1, L - *nl - 1, v);
    };
    if (!out) {
        int64_t bad = ns;
#pragma omp parallel for schedule(static) reduction(min : bad) if (n_rows > 4096)
        for (int64_t r = 0; r < n_rows; ++r) {
            double acc = 0.0;
            bool ok = true;
            for (int64_t k = row_off[r]; k < row_off[r + 1]; ++k) {
                const int64_t q = k - row_off[0];
                int nl;
                double v;
                if (!split(q, &nl, &v) || !std::isfinite(v)) { bad = q < bad ? q : bad; ok = false; break; }
                acc += p == 1 ? std::fabs(v) : v * v;
            }
            const double nr = p == 1 ? acc : std::sqrt(acc);
            norm[r] = nr;
            char tmp[48];
            for (int64_t k = row_off[r]; k < row_off[r + 1]; ++k) {
                const int64_t q = k - row_off[0];
                const int L = (int)(off[q + 1] - off[q]);
                if (!ok || nr == 0.0) { out_off[q + 1] = L; continue; }
                int nl;
                double v;
                split(q, &nl, &v);
                const double x = v / nr;
                if (!std::isfinite(x)) { bad = q < bad ? q : bad; out_off[q + 1] = L; continue; }
                out_off[q + 1] = nl + 1 + fmt_py_float(x, tmp);
            }
        }
        if (bad < ns) return -2 - bad;
        prefix_sum_inplace(out_off, ns);
        return out_off[ns];
    }
#pragma omp parallel for schedule(static) if (n_rows > 4096)
    for (int64_t r = 0; r < n_rows; ++r) {
        const double nr = norm[r];
        for (int64_t k = row_off[r]; k < row_off[r + 1]; ++k) {
            const int64_t q = k - row_off[0];
            char* o = reinterpret_cast<char*>(out + out_off[q]);
            const char* s = (const char*)buf + off[q];
            if (nr == 0.0) { std::memcpy(o, s, (size_t)(off[q + 1] - off[q])); continue; }
            int nl;
            double v;
            split(q, &nl, &v);
            std::memcpy(o, s, (size_t)nl);
            o[nl] = ':';
            fmt_py_float(v / nr, o + nl + 1);
        }
    }
    return out_off[ns];
}
