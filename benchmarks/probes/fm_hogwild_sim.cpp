// Host model of train_fm's Hogwild kernel with W rows in flight (round 6 probe, CPU only): the rule
// of csrc/host/fm_cpu.cpp, where row r reads the state W rows stale and its write lands W rows later
// as a plain store (a concurrent row's step to the same address is lost) or an added delta,
// per feature: mode bit 1 = V adds its delta, 4 = w adds.  w0 always adds (the GPU's atomic shards).
//   g++ -O3 -march=native -shared -fPIC -o /tmp/fm_hogwild_sim.so fm_hogwild_sim.cpp
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {
struct VW { int32_t i; uint8_t mode; float w, dw; float v[16], dv[16]; };
}

// ip: dims, k, KP, eta_kind, use_w0, W, F (features per row); hp: eta0, power_t, total, l0, lw, lv
extern "C" int fm_hogwild_sim(const int32_t* ip, const float* hp, int64_t n_rows, int64_t t0,
                              const int32_t* idx, const float* y, const uint8_t* mode, float* w,
                              float* V, float* w0) {
    const int dims = ip[0], k = ip[1], KP = ip[2], eta_kind = ip[3], use_w0 = ip[4], W = ip[5], F = ip[6];
    const float eta0 = hp[0], power_t = hp[1], total = hp[2], l0 = hp[3], lw = hp[4], lv = hp[5];
    if (KP > 16) return 22;
    std::vector<std::vector<VW>> ring(W);
    std::vector<float> dw0(W, 0.f);
    std::vector<float> S(KP);
    auto apply = [&](int slot) {
        for (const VW& e : ring[slot]) {
            float* v = V + (size_t)e.i * KP;
            if (e.mode & 4) w[e.i] += e.dw; else w[e.i] = e.w;
            if (e.mode & 1) for (int f = 0; f < KP; ++f) v[f] += e.dv[f];
            else for (int f = 0; f < KP; ++f) v[f] = e.v[f];
        }
        ring[slot].clear();
        if (use_w0) *w0 += dw0[slot];
        dw0[slot] = 0.f;
    };
    for (int64_t row = 0; row < n_rows; ++row) {
        const int slot = (int)(row % W);
        apply(slot);
        const int32_t* ri = idx + row * F;
        std::fill(S.begin(), S.end(), 0.f);
        float lin = 0.f, sq = 0.f;
        for (int a = 0; a < F; ++a) {
            const int i = ri[a];
            if (i < 0 || i >= dims) continue;
            lin += w[i];
            const float* v = V + (size_t)i * KP;
            for (int f = 0; f < KP; ++f) { S[f] += v[f]; sq += v[f] * v[f]; }
        }
        float pair = 0.f;
        for (int f = 0; f < KP; ++f) pair += S[f] * S[f];
        float p = lin + 0.5f * (pair - sq);
        if (use_w0) p += *w0;
        const float yy = y[row];
        const float d = -yy / (1.f + std::exp(yy * p));
        const float t = (float)(t0 + row + 1);
        float eta = eta0;
        if (eta_kind == 1) eta = total > 0.f ? eta0 / (1.f + t / total) : eta0;
        else if (eta_kind == 2) eta = eta0 / std::pow(t > 1.f ? t : 1.f, power_t);
        for (int a = 0; a < F; ++a) {
            const int i = ri[a];
            if (i < 0 || i >= dims) continue;
            VW e;
            e.i = i;
            e.mode = mode ? mode[i] : 0;
            e.dw = -eta * (d + 2.f * lw * w[i]);
            e.w = w[i] + e.dw;
            const float* v = V + (size_t)i * KP;
            for (int f = 0; f < KP; ++f) {
                const float g = f < k ? d * (S[f] - v[f]) + 2.f * lv * v[f] : 0.f;
                e.dv[f] = f < k ? -eta * g : 0.f;
                e.v[f] = v[f] + e.dv[f];
            }
            ring[slot].push_back(e);
        }
        if (use_w0) dw0[slot] = -eta * (d + 2.f * l0 * *w0);
    }
    for (int64_t r = n_rows; r < n_rows + W; ++r) apply((int)(r % W));
    return 0;
}
