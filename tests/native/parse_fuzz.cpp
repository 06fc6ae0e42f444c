// Host build of csrc/kernels/parse.h (the device feature-string parsers) fuzzed against strtod /
// the host parser's rules: every string the device parser accepts must give the host's
// (float)strtod bit for bit; refusals are allowed (the ingest falls back to the host).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#define __device__
#define __forceinline__ inline
#include "../../csrc/kernels/parse.h"

int main() {
    const char* fixed[] = {"2.5e+1", "1E3", "3.0e-2", "1e-2", "0.5", ".5", "5.", "-.5", "1e", "e5", "1.2.3", "+",
                           "-", "1e+", "0", "00.000", "1e22", "1e23", "9007199254740993", ".", "1e0001",
                           "0.1", "12345.678", "-7", "+3.25E-02", "1e-22", "4.9e-324", "3.4e39"};
    int bad = 0, acc = 0;
    for (const char* s : fixed) {
        float v;
        const int n = (int)strlen(s);
        const bool ok = hm::dev_parse_float((const uint8_t*)s, n, &v);
        char* end;
        const double d = strtod(s, &end);
        const bool hok = end == s + n;
        if (ok && (!hok || (float)d != v)) { printf("MISMATCH %s\n", s); ++bad; }
    }
    const char* must[] = {"2.5e+1", "1E3", "3.0e-2", "1e-2", "0.5", ".5", "-7", "12345.678", "1e22"};
    for (const char* s : must) {
        float v;
        if (!hm::dev_parse_float((const uint8_t*)s, (int)strlen(s), &v)) { printf("REFUSED %s\n", s); ++bad; }
    }
    char buf[64];
    srand(1);
    for (int it = 0; it < 1000000; ++it) {
        int n;
        if (rand() % 3 == 0)
            n = snprintf(buf, 64, "%d.%de%d", rand() % 1000, rand() % 1000, rand() % 40 - 20);
        else
            n = snprintf(buf, 64, "%.*g", rand() % 10 + 1, (rand() / (double)RAND_MAX - 0.5) * pow(10, rand() % 30 - 15));
        float v;
        if (hm::dev_parse_float((const uint8_t*)buf, n, &v)) {
            ++acc;
            if ((float)strtod(buf, nullptr) != v) { if (++bad < 10) printf("MISMATCH %s\n", buf); }
        }
        int64_t a;
        char ib[32];
        const int m = snprintf(ib, 32, "%lld", (long long)(rand() - RAND_MAX / 2) * (rand() % 1000));
        if (!hm::dev_parse_int((const uint8_t*)ib, m, &a) || a != strtoll(ib, nullptr, 10)) {
            if (++bad < 10) printf("INT %s\n", ib);
        }
    }
    printf("accepted %d bad %d\n", acc, bad);
    return bad != 0 || acc < 900000;
}
