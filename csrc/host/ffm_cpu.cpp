// CPU engine for FFM: same update rule and layout as csrc/kernels/ffm.hip, processed
// strictly row by row (Hivemall's per-mapper online semantics, no Hogwild).  Used for CPU
// runs (world_size=1 plumbing) and as the numerical oracle for the GPU kernel.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#define HM_API extern "C" __attribute__((visibility("default")))

namespace {

inline float ftrl_weight(float z, float n, float alpha, float beta, float l1, float l2) {
    if (std::fabs(z) <= l1) return 0.f;
    const float s = z > 0.f ? 1.f : -1.f;
    return -(z - s * l1) / ((beta + std::sqrt(n)) / alpha + l2);
}

inline float ftrl_update(float* z, float* n, float w, float g, float alpha, float beta, float l1,
                         float l2) {
    const float n0 = *n, n1 = n0 + g * g;
    const float sigma = (std::sqrt(n1) - std::sqrt(n0)) / alpha;
    *z += g - sigma * w;
    *n = n1;
    return ftrl_weight(*z, n1, alpha, beta, l1, l2);
}

inline float log1pexp(float x) { return x > 0.f ? x + std::log1p(std::exp(-x)) : std::log1p(std::exp(x)); }

template <int KP>
int ffm_step_cpu(const int32_t* ip, const float* hp, const int32_t* idx,
                 const int32_t* fld, const float* val, const float* y, float* V,
                 float* G, float* w, float* wz, float* wn, float* bias, float* pred,
                 float* loss) {
    // KP > 0: the factor count as a compile-time constant (k = 4 / 8: the slot copies and the
    // k-loops unroll, no memcpy call per slot); KP = 0: any Kp.  Same operations in the same
    // order either way, so the results are identical.
    const int B = ip[0], F = ip[1], NF = ip[2], NFLD = ip[3], Kp = KP > 0 ? KP : ip[4];
    const int cls = ip[5], train = ip[6], use_lin = ip[7], use_bias = ip[8], norm = ip[9];
    const float eta0 = hp[0], eps = hp[1], lv = hp[2], alpha = hp[3], beta = hp[4];
    const float l1 = hp[5], l2 = hp[6], tmin = hp[7], tmax = hp[8];
    // slot stride: Kp (separate V / G tables) or 2*Kp (packed [NF][NFLD][2][Kp], G = V + Kp)
    const size_t ss = ip[14] ? (size_t)2 * Kp : (size_t)Kp;
    // slots between consecutive features (>= NFLD: the GPU's packed table pads each feature
    // block to whole 128-B lines)
    const size_t FS = ip[16] > 0 ? (size_t)ip[16] : (size_t)NFLD;
    // AdaGrad accumulator: 1 = ONE per (feature, field) slot, G[i * GS + f] (Hivemall's
    // AdaGradEntry: a single sum of squared gradients per entry, shared by the k factors);
    // 0 = one per element, laid out like V
    const int slot_g = ip[17];
    const size_t GS = ip[18] > 0 ? (size_t)ip[18] : FS;   // slot-G: floats between features
    const size_t GF = ip[21] > 0 ? (size_t)ip[21] : 1;    // slot-G: floats between fields
    if (slot_g && Kp > 64) return 22;
    std::vector<int> ri(F), rf(F);
    std::vector<float> rx(F);
    std::vector<float> snap((size_t)F * F * Kp);
    // multi-hot rows: a row updates each (feature, field) address once with its summed gradient
    // (docs/compat.md).  ni / nf: next position with the same feature / field (-1: none);
    // first: bit 0 = first position of its feature, bit 1 = first of its field
    std::vector<int> ni(F), nf(F), first(F);
    std::vector<float> gsum(Kp);
    for (int r = 0; r < B; ++r) {
        float sq = 0.f;
        for (int a = 0; a < F; ++a) {
            const size_t o = (size_t)r * F + a;
            int i = idx[o];
            int f = fld ? fld[o] : a;
            float x = val ? val[o] : 1.f;
            if (i < 0 || i >= NF || f < 0 || f >= NFLD) { i = -1; x = 0.f; }
            ri[a] = i;
            rf[a] = f < 0 ? 0 : (f >= NFLD ? NFLD - 1 : f);
            rx[a] = x;
            sq += x * x;
        }
        const float scale = (norm && sq > 0.f) ? 1.f / std::sqrt(sq) : 1.f;
        bool multi = false;
        for (int a = 0; a < F; ++a) {
            ni[a] = nf[a] = -1;
            first[a] = 3;
            if (ri[a] < 0) continue;
            for (int b = 0; b < F; ++b) {
                if (b == a || ri[b] < 0) continue;
                if (ri[b] == ri[a]) { if (b < a) first[a] &= ~1; else if (ni[a] < 0) ni[a] = b; multi = true; }
                if (rf[b] == rf[a]) { if (b < a) first[a] &= ~2; else if (nf[a] < 0) nf[a] = b; multi = true; }
            }
        }
        // snapshot of the row's slot vectors (matches the LDS staging of the GPU kernel; the
        // diagonal (a, a) is staged for multi-hot rows, where it can own an address)
        for (int a = 0; a < F; ++a)
            for (int b = 0; b < F; ++b) {
                float* dst = &snap[((size_t)a * F + b) * Kp];
                if ((a != b || multi) && ri[a] >= 0 && ri[b] >= 0) {
                    const float* src = V + ((size_t)ri[a] * FS + rf[b]) * ss;
                    for (int k = 0; k < Kp; ++k) dst[k] = src[k];
                } else {
                    for (int k = 0; k < Kp; ++k) dst[k] = 0.f;
                }
            }
        double p = 0.0;
        for (int a = 0; a < F; ++a)
            for (int b = a + 1; b < F; ++b) {
                if (ri[a] < 0 || ri[b] < 0) continue;
                const float* u = &snap[((size_t)a * F + b) * Kp];
                const float* v = &snap[((size_t)b * F + a) * Kp];
                float d = 0.f;
                for (int k = 0; k < Kp; ++k) d += u[k] * v[k];
                p += (double)d * rx[a] * rx[b] * scale * scale;
            }
        if (use_lin)
            for (int a = 0; a < F; ++a)
                if (ri[a] >= 0) p += (double)w[ri[a]] * rx[a] * scale;
        if (use_bias) p += bias[0];
        const float yy = y ? y[r] : 0.f;
        float kappa;
        if (cls) {
            const float e = yy * (float)p;
            kappa = -yy / (1.f + std::exp(e));
            if (loss) loss[r] = log1pexp(-e);
            if (pred) pred[r] = (float)p;
        } else {
            const float pc = std::fmin(std::fmax((float)p, tmin), tmax);
            kappa = pc - yy;
            if (loss) loss[r] = 0.5f * kappa * kappa;
            if (pred) pred[r] = pc;
        }
        if (!train) continue;
        const float ks = kappa * scale * scale;
        for (int a = 0; a < F; ++a)
            for (int b = 0; b < F; ++b) {
                if (ri[a] < 0 || ri[b] < 0) continue;
                float* pv = V + ((size_t)ri[a] * FS + rf[b]) * ss;
                const float* own = &snap[((size_t)a * F + b) * Kp];
                float* gk = gsum.data();
                if (!multi) {
                    if (a == b) continue;
                    const float coef = ks * rx[a] * rx[b];
                    const float* par = &snap[((size_t)b * F + a) * Kp];
                    for (int k = 0; k < Kp; ++k) gk[k] = coef * par[k] + lv * own[k];
                } else {
                    // the address (i_a, f_b) is updated by its owner slot (first position of the
                    // feature, first of the field) with the sum over every pair that maps to it
                    if (!(first[a] & 1) || !(first[b] & 2)) continue;
                    bool any = false;
                    for (int k = 0; k < Kp; ++k) gk[k] = 0.f;
                    for (int a2 = a; a2 >= 0; a2 = ni[a2])
                        for (int b2 = b; b2 >= 0; b2 = nf[b2]) {
                            if (a2 == b2) continue;
                            any = true;
                            const float coef = ks * rx[a2] * rx[b2];
                            const float* par = &snap[((size_t)b2 * F + a2) * Kp];
                            for (int k = 0; k < Kp; ++k) gk[k] += coef * par[k];
                        }
                    if (!any) continue;
                    for (int k = 0; k < Kp; ++k) gk[k] += lv * own[k];
                }
                if (slot_g) {
                    // G += sum_f g_f^2 (fp32, factor order), then every factor steps with it
                    float* pg = G + (size_t)ri[a] * GS + (size_t)rf[b] * GF;
                    float gs = *pg;
                    for (int k = 0; k < Kp; ++k) gs += gk[k] * gk[k];
                    *pg = gs;
                    const float r = 1.f / std::sqrt(gs + eps);
                    for (int k = 0; k < Kp; ++k) pv[k] = own[k] - eta0 * gk[k] * r;
                    continue;
                }
                float* pg = G + ((size_t)ri[a] * FS + rf[b]) * ss;
                for (int k = 0; k < Kp; ++k) {
                    const float g = gk[k];
                    pg[k] += g * g;
                    pv[k] = own[k] - eta0 * g / std::sqrt(pg[k] + eps);
                }
            }
        if (use_lin)
            for (int a = 0; a < F; ++a) {
                const int i = ri[a];
                if (i < 0 || !(first[a] & 1)) continue;
                // a feature repeated in the row: one FTRL step with the summed gradient
                float xs = rx[a];
                for (int a2 = ni[a]; a2 >= 0; a2 = ni[a2]) xs += rx[a2];
                w[i] = ftrl_update(wz + i, wn + i, w[i], kappa * xs * scale, alpha, beta, l1, l2);
            }
        if (use_bias) bias[0] = ftrl_update(bias + 1, bias + 2, bias[0], kappa, alpha, beta, 0.f, 0.f);
    }
    return 0;
}

}  // namespace

HM_API int hm_ffm_step_cpu(const int32_t* ip, const float* hp, const int32_t* idx,
                           const int32_t* fld, const float* val, const float* y, float* V,
                           float* G, float* w, float* wz, float* wn, float* bias, float* pred,
                           float* loss) {
    switch (ip[4]) {
        case 4: return ffm_step_cpu<4>(ip, hp, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss);
        case 8: return ffm_step_cpu<8>(ip, hp, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss);
        default: return ffm_step_cpu<0>(ip, hp, idx, fld, val, y, V, G, w, wz, wn, bias, pred, loss);
    }
}
