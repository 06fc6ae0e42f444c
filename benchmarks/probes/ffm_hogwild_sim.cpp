// Host model of Hogwild FFM training with W rows in flight (round-6 parity probe, CPU only).
//
// Row r reads the state as it stood after the writes of rows <= r - W and its write lands W rows
// later (a staggered window: the same one-row read-modify-write race the GPU's ~1,000 resident
// rows run).  Per feature class and per state part, a write either OVERWRITES (a plain store of
// the value the row computed: updates of rows r' in (r - W, r) to the same address are lost, as
// on the GPU) or ADDS the row's delta (an atomic: nothing lost, only the read is stale).  With
// W = 1 this is ffm_step_cpu (csrc/host/ffm_cpu.cpp) on rows without repeated features, per-slot
// AdaGrad (Hivemall's AdaGradEntry), fields = positions.
//
//   g++ -O3 -march=native -shared -fPIC -o /tmp/ffm_hogwild_sim.so ffm_hogwild_sim.cpp
//
// mode[i] bits for feature i: 1 = V of its slots add deltas, 2 = G adds, 4 = its linear (z, n) add.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

inline float ftrl_weight(float z, float n, float alpha, float beta, float l1, float l2) {
    if (std::fabs(z) <= l1) return 0.f;
    const float s = z > 0.f ? 1.f : -1.f;
    return -(z - s * l1) / ((beta + std::sqrt(n)) / alpha + l2);
}

struct SlotW { int32_t addr; uint8_t mode; float v[4]; float g; float dv[4]; float dg; };
struct LinW { int32_t i; uint8_t mode; float w, z, n, dz, dn; };

struct Pending {
    std::vector<SlotW> s;
    std::vector<LinW> l;
    float dz0 = 0.f, dn0 = 0.f;
};

}  // namespace

// ip: {rows, F, NF, W, use_lin, use_bias, norm, D}: D > 0 delays the ADDED linear steps by D rows
// instead of W (a block that sums its rows' linear steps in LDS and flushes them every R rows
// publishes them ~R x resident-blocks rows late); hp: {eta0, eps, lambda_v, alpha, beta, l1, l2}
// V [NF][F][4], G [NF][F], w / z / n [NF], bias {w0, z0, n0}; pending writes carried in `ring`
// across calls when `keep` (one call per batch; the GPU drains its grid at the end of a launch,
// so pass keep = 0 to flush at a batch boundary).
extern "C" int ffm_hogwild_sim(const int32_t* ip, const float* hp, const int32_t* idx,
                               const float* val, const float* y, const uint8_t* mode, float* V,
                               float* G, float* w, float* z, float* n, float* bias,
                               float* loss_out) {
    const int B = ip[0], F = ip[1], W = ip[3], use_lin = ip[4], use_bias = ip[5], norm = ip[6];
    const int D = ip[7];
    std::vector<std::vector<LinW>> lring(D > 0 ? D : 1);
    const float eta0 = hp[0], eps = hp[1], lv = hp[2], alpha = hp[3], beta = hp[4], l1 = hp[5], l2 = hp[6];
    std::vector<Pending> ring(W);
    std::vector<int> ri(F);
    std::vector<float> rx(F), snap((size_t)F * F * 4), gsnap((size_t)F * F);
    auto apply = [&](Pending& p) {
        for (const SlotW& e : p.s) {
            float* pv = V + (size_t)e.addr * 4;
            if (e.mode & 1) for (int k = 0; k < 4; ++k) pv[k] += e.dv[k];
            else for (int k = 0; k < 4; ++k) pv[k] = e.v[k];
            if (e.mode & 2) G[e.addr] += e.dg; else G[e.addr] = e.g;
        }
        for (const LinW& e : p.l) {
            if (e.mode & 4) {
                z[e.i] += e.dz;
                n[e.i] += e.dn;
                w[e.i] = ftrl_weight(z[e.i], n[e.i], alpha, beta, l1, l2);
            } else {
                w[e.i] = e.w; z[e.i] = e.z; n[e.i] = e.n;
            }
        }
        if (use_bias) {
            bias[1] += p.dz0;
            bias[2] += p.dn0;
            bias[0] = ftrl_weight(bias[1], bias[2], alpha, beta, 0.f, 0.f);
        }
        p.s.clear(); p.l.clear(); p.dz0 = p.dn0 = 0.f;
    };
    for (int r = 0; r < B; ++r) {
        Pending& slot = ring[r % W];
        apply(slot);                       // row r - W's writes land before row r reads
        if (D > 0) {
            Pending tmp;
            tmp.l.swap(lring[r % D]);
            apply(tmp);
        }
        float sq = 0.f;
        for (int a = 0; a < F; ++a) {
            ri[a] = idx[(size_t)r * F + a];
            rx[a] = val ? val[(size_t)r * F + a] : 1.f;
            sq += rx[a] * rx[a];
        }
        const float scale = (norm && sq > 0.f) ? 1.f / std::sqrt(sq) : 1.f;
        for (int a = 0; a < F; ++a)
            for (int b = 0; b < F; ++b) {
                const size_t s = (size_t)a * F + b;
                const size_t addr = (size_t)ri[a] * F + b;
                std::memcpy(&snap[s * 4], V + addr * 4, 16);
                gsnap[s] = G[addr];
            }
        double p = 0.0;
        for (int a = 0; a < F; ++a)
            for (int b = a + 1; b < F; ++b) {
                const float* u = &snap[((size_t)a * F + b) * 4];
                const float* v = &snap[((size_t)b * F + a) * 4];
                float d = 0.f;
                for (int k = 0; k < 4; ++k) d += u[k] * v[k];
                p += (double)d * rx[a] * rx[b] * scale * scale;
            }
        if (use_lin) for (int a = 0; a < F; ++a) p += (double)w[ri[a]] * rx[a] * scale;
        if (use_bias) p += bias[0];
        const float yy = y[r];
        const float e = yy * (float)p;
        const float kappa = -yy / (1.f + std::exp(e));
        if (loss_out) loss_out[r] = e > 0.f ? std::log1p(std::exp(-e)) : -e + std::log1p(std::exp(e));
        const float ks = kappa * scale * scale;
        for (int a = 0; a < F; ++a)
            for (int b = 0; b < F; ++b) {
                if (a == b) continue;
                const size_t s = (size_t)a * F + b;
                const float* own = &snap[s * 4];
                const float* par = &snap[((size_t)b * F + a) * 4];
                const float coef = ks * rx[a] * rx[b];
                float gk[4], gs = gsnap[s];
                for (int k = 0; k < 4; ++k) { gk[k] = coef * par[k] + lv * own[k]; gs += gk[k] * gk[k]; }
                const float rr = 1.f / std::sqrt(gs + eps);
                SlotW o;
                o.addr = (int32_t)((size_t)ri[a] * F + b);
                o.mode = mode ? mode[ri[a]] : 0;
                for (int k = 0; k < 4; ++k) { o.dv[k] = -eta0 * gk[k] * rr; o.v[k] = own[k] + o.dv[k]; }
                o.g = gs;
                o.dg = gs - gsnap[s];
                slot.s.push_back(o);
            }
        if (use_lin)
            for (int a = 0; a < F; ++a) {
                const int i = ri[a];
                const float g = kappa * rx[a] * scale;
                const float n0 = n[i], n1 = n0 + g * g;
                const float z1 = z[i] + g - (std::sqrt(n1) - std::sqrt(n0)) / alpha * w[i];
                LinW o;
                o.i = i;
                o.mode = mode ? mode[i] : 0;
                o.z = z1; o.n = n1; o.w = ftrl_weight(z1, n1, alpha, beta, l1, l2);
                o.dz = z1 - z[i]; o.dn = g * g;
                if (D > 0 && (o.mode & 4)) lring[r % D].push_back(o); else slot.l.push_back(o);
            }
        if (use_bias) {
            const float n0 = bias[2], n1 = n0 + kappa * kappa;
            slot.dz0 = kappa - (std::sqrt(n1) - std::sqrt(n0)) / alpha * bias[0];
            slot.dn0 = kappa * kappa;
        }
    }
    for (int r = B; r < B + W; ++r) apply(ring[r % W]);   // drain
    for (int r = 0; r < D; ++r) { Pending tmp; tmp.l.swap(lring[r]); apply(tmp); }
    return 0;
}
