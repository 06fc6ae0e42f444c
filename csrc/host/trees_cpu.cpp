// CPU twins of csrc/kernels/trees.hip (same layouts and semantics), OpenMP-parallel.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#define HM_API extern "C" __attribute__((visibility("default")))
#define HM_TREE_CAT 0x40000000    // nominal split flag (csrc/kernels/trees.hip)
#define HM_TREE_DLEFT 0x20000000  // missing values go left (learned default direction)

HM_API int hm_hist_build_cpu(const uint8_t* bins, int d, int dpad, int B, const int32_t* rows,
                             const int64_t* seg, int n_seg, const float* stats, const float* smax,
                             int NS, int FG, float* hist) {
    (void)FG; (void)smax;  // exact fp32 sums on the host
#pragma omp parallel for schedule(dynamic, 1) collapse(2)
    for (int node = 0; node < n_seg; ++node) {
        for (int f = 0; f < d; ++f) {
            float* h = hist + (((size_t)node * d + f) * B) * NS;
            for (int64_t q = seg[node]; q < seg[node + 1]; ++q) {
                const int64_t r = rows[q];
                const int b = bins[r * dpad + f];
                const float* st = stats + r * NS;
                for (int s = 0; s < NS; ++s) h[b * NS + s] += st[s];
            }
        }
    }
    return 0;
}

HM_API int hm_tree_predict_cpu(const float* X, int64_t n, int d, const int32_t* feature,
                               const float* threshold, const int32_t* left, const int32_t* right,
                               const int32_t* voff, const float* values, const int32_t* roots,
                               int n_trees, int n_out, float* out, int sum_trees,
                               const float* tree_w) {
#pragma omp parallel for schedule(static)
    for (int64_t row = 0; row < n; ++row) {
        const float* x = X + row * d;
        for (int t = 0; t < n_trees; ++t) {
            int k = roots[t];
            for (int depth = 0; depth < 64; ++depth) {
                int f = feature[k];
                if (f < 0) break;
                const bool cat = f & HM_TREE_CAT;
                const bool dl = f & HM_TREE_DLEFT;
                f &= ~(HM_TREE_CAT | HM_TREE_DLEFT);
                const float v = x[f];
                // NaN goes right unless the split learned a default direction
                k = std::isnan(v) ? (dl ? left[k] : right[k])
                                  : ((cat ? v == threshold[k] : v <= threshold[k]) ? left[k] : right[k]);
            }
            const float* val = values + voff[k];
            if (sum_trees) {
                const float w = tree_w ? tree_w[t] : 1.f;
                for (int o = 0; o < n_out; ++o) out[row * n_out + o] += w * val[o];
            } else {
                float* dst = out + (row * n_trees + t) * n_out;
                for (int o = 0; o < n_out; ++o) dst[o] = val[o];
            }
        }
    }
    return 0;
}

HM_API int hm_quantize_cpu(const float* X, int64_t n, int d, int dpad, const float* edges,
                           int n_edges, uint8_t* bins) {
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < n; ++r) {
        for (int f = 0; f < d; ++f) {
            const float v = X[r * d + f];
            const float* e = edges + (size_t)f * n_edges;
            int lo = 0, hi = n_edges;
            if (std::isnan(v)) lo = n_edges;
            else
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (e[mid] < v) lo = mid + 1; else hi = mid;
                }
            bins[r * dpad + f] = (uint8_t)lo;
        }
    }
    return 0;
}

HM_API int hm_route_rows_cpu(const uint8_t* bins, int64_t n, int dpad, int32_t* node_of_row,
                             const int32_t* split_feat, const int32_t* split_bin,
                             const int32_t* left_child, const int32_t* right_child, int miss_bin) {
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < n; ++r) {
        const int nd = node_of_row[r];
        if (nd < 0) continue;
        int f = split_feat[nd];
        if (f < 0) continue;
        const bool cat = f & HM_TREE_CAT;
        const bool dl = f & HM_TREE_DLEFT;
        f &= ~(HM_TREE_CAT | HM_TREE_DLEFT);
        const int b = bins[r * dpad + f];
        const bool go_left = b == miss_bin ? dl : (cat ? b == split_bin[nd] : b <= split_bin[nd]);
        node_of_row[r] = go_left ? left_child[nd] : right_child[nd];
    }
    return 0;
}

// ---------------------------------------------------------------------------------------------
// Host twin of split_find_kernel (csrc/kernels/trees.hip): same criteria, candidate-feature
// draw (feat_key ranking) and tie-break (larger gain, then smaller feature*B + bin).
namespace {

inline uint32_t feat_key(uint32_t seed, uint32_t node, uint32_t f) {
    uint32_t h = seed * 0x9E3779B1u ^ (node + 0x7F4A7C15u) * 0x85EBCA77u ^ (f + 1u) * 0xC2B2AE3Du;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    return h;
}

inline float split_weight(const float* S, int NS, int crit) {
    if (crit <= 1) { float w = 0.f; for (int s = 0; s < NS; ++s) w += S[s]; return w; }
    if (crit == 3) return NS > 2 ? S[2] : 0.f;
    return NS > 1 ? S[1] : 0.f;
}

inline float split_score(const float* S, int NS, int crit, float lam, float alpha) {
    if (crit == 0) {
        float w = 0.f, q = 0.f;
        for (int s = 0; s < NS; ++s) { w += S[s]; q += S[s] * S[s]; }
        return w > 0.f ? q / std::fmax(w, 1e-30f) : 0.f;
    }
    if (crit == 1) {
        float w = 0.f;
        for (int s = 0; s < NS; ++s) w += S[s];
        const float iw = 1.f / std::fmax(w, 1e-30f);
        float e = 0.f;
        for (int s = 0; s < NS; ++s) e += S[s] * std::log(std::fmax(S[s] * iw, 1e-30f));
        return e;
    }
    const float s0 = S[0];
    if (crit == 2) { const float s1 = S[NS > 1 ? 1 : 0]; return s1 > 0.f ? s0 * s0 / std::fmax(s1, 1e-30f) : 0.f; }
    if (crit == 3) { const float s2 = S[NS > 2 ? 2 : 0]; return s2 > 0.f ? s0 * s0 / (s2 + lam) : 0.f; }
    const float s1 = S[NS > 1 ? 1 : 0];
    float g = s0;
    if (alpha > 0.f) { const float m = std::fabs(g) - alpha; g = m > 0.f ? std::copysign(m, g) : 0.f; }
    return s1 > 0.f ? g * g / (s1 + lam) : 0.f;
}

inline float wide_term(float S, float W, int crit) {
    return crit == 0 ? S * S : S * std::log(std::fmax(S / std::fmax(W, 1e-30f), 1e-30f));
}
inline float wide_score(float W, float T, int crit) {
    if (W <= 0.f) return 0.f;
    return crit == 0 ? T / std::fmax(W, 1e-30f) : T;
}

// NS > 8 (many classes, gini / entropy): the class-decomposed scores of split_find_wide_kernel,
// same accumulation order (classes 0..NS-1 per candidate bin).
void split_find_wide(const float* hist, int L, int d, int B, int NS, int n_edges, int crit, int mtry,
                     int node_base, uint32_t seed, float min_leaf, const uint8_t* cat, const uint8_t* fmask,
                     float* gain, int32_t* feat, int32_t* bin, float* left, float* tot) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int node = 0; node < L; ++node) {
        const float* hn = hist + (size_t)node * d * B * NS;
        std::vector<float> T(NS, 0.f);
        for (int c = 0; c < NS; ++c)
            for (int b = 0; b < B; ++b) T[c] += hn[(size_t)b * NS + c];
        float pw = 0.f, pt = 0.f;
        for (int c = 0; c < NS; ++c) pw += T[c];
        for (int c = 0; c < NS; ++c) pt += wide_term(T[c], pw, crit);
        const float parent = wide_score(pw, pt, crit);
        std::vector<float> wl(B), tl(B), wr(B), tr(B);
        float best = -INFINITY;
        int best_i = 0x7FFFFFFF;
        for (int f = 0; f < d; ++f) {
            if (fmask && !fmask[f]) continue;
            if (mtry > 0 && mtry < d) {
                const uint32_t kf = feat_key(seed, (uint32_t)(node_base + node), (uint32_t)f);
                int before = 0;
                for (int g = 0; g < d; ++g) {
                    const uint32_t kg = feat_key(seed, (uint32_t)(node_base + node), (uint32_t)g);
                    before += (kg < kf || (kg == kf && g < f)) ? 1 : 0;
                }
                if (before >= mtry) continue;
            }
            const bool is_cat = cat && cat[f];
            const float* hf = hn + (size_t)f * B * NS;
            std::fill(wl.begin(), wl.end(), 0.f); std::fill(tl.begin(), tl.end(), 0.f);
            std::fill(wr.begin(), wr.end(), 0.f); std::fill(tr.begin(), tr.end(), 0.f);
            for (int pass = crit == 1 ? 0 : 1; pass < 2; ++pass) {
                for (int c = 0; c < NS; ++c) {
                    float tc = 0.f;
                    for (int b = 0; b < B; ++b) tc += hf[(size_t)b * NS + c];
                    float run = 0.f;
                    for (int b = 0; b < B; ++b) {
                        const float h = hf[(size_t)b * NS + c];
                        run += h;
                        const float l = is_cat ? h : run;
                        const float r = tc - l;
                        if (pass == 0 || crit == 0) { wl[b] += l; wr[b] += r; }
                        if (pass == 1) { tl[b] += wide_term(l, wl[b], crit); tr[b] += wide_term(r, wr[b], crit); }
                    }
                }
            }
            for (int b = 0; b < B; ++b) {
                if (wl[b] < min_leaf || wr[b] < min_leaf) continue;
                if (is_cat && b >= n_edges) continue;
                const float g = wide_score(wl[b], tl[b], crit) + wide_score(wr[b], tr[b], crit) - parent;
                const int i = f * B + b;
                if (g > best || (g == best && i < best_i)) { best = g; best_i = i; }
            }
        }
        const bool found = best_i != 0x7FFFFFFF;
        gain[node] = found ? best : -INFINITY;
        feat[node] = found ? best_i / B : 0;
        bin[node] = found ? best_i % B : 0;
        const int bf = found ? best_i / B : 0, bb = found ? best_i % B : -1;
        const bool bcat = found && cat && cat[bf];
        for (int c = 0; c < NS; ++c) {
            float t = 0.f, l = 0.f;
            for (int b = 0; b < B; ++b) {
                t += hn[(size_t)b * NS + c];
                const float hv = hn[((size_t)bf * B + b) * NS + c];
                if (bcat ? b == bb : b <= bb) l += hv;
            }
            tot[(size_t)node * NS + c] = t;
            left[(size_t)node * NS + c] = found ? l : 0.f;
        }
    }
}

}  // namespace

HM_API int hm_split_find_cpu(const float* hist, const int32_t* ip, const float* fp, const uint8_t* cat,
                             const uint8_t* fmask, float* gain, int32_t* feat, int32_t* bin, float* left,
                             float* tot) {
    const int L = ip[0], d = ip[1], B = ip[2], NS = ip[3], n_edges = ip[4], crit = ip[5];
    const int mtry = ip[6], node_base = ip[7];
    const uint32_t seed = (uint32_t)ip[8];
    const int miss = ip[9];
    const float lam = fp[0], alpha = fp[1], min_leaf = fp[2];
    if (B <= 0 || B > 256 || NS <= 0 || crit < 0 || crit > 4) return 1;
    if (NS > 8) {
        if (crit > 1 || miss) return 1;
        split_find_wide(hist, L, d, B, NS, n_edges, crit, mtry, node_base, seed, min_leaf, cat, fmask, gain,
                        feat, bin, left, tot);
        return 0;
    }
#pragma omp parallel for schedule(dynamic, 1)
    for (int node = 0; node < L; ++node) {
        const float* hn = hist + (size_t)node * d * B * NS;
        float T[8] = {0}, Lb[8] = {0}, run[8], lf[8], rt[8];
        for (int b = 0; b < B; ++b)
            for (int s = 0; s < NS; ++s) T[s] += hn[(size_t)b * NS + s];
        const float parent = split_score(T, NS, crit, lam, alpha);
        float best = -INFINITY;
        int best_i = 0x7FFFFFFF;
        for (int f = 0; f < d; ++f) {
            if (fmask && !fmask[f]) continue;
            if (mtry > 0 && mtry < d) {
                const uint32_t kf = feat_key(seed, (uint32_t)(node_base + node), (uint32_t)f);
                int before = 0;
                for (int g = 0; g < d; ++g) {
                    const uint32_t kg = feat_key(seed, (uint32_t)(node_base + node), (uint32_t)g);
                    before += (kg < kf || (kg == kf && g < f)) ? 1 : 0;
                }
                if (before >= mtry) continue;
            }
            const bool is_cat = cat && cat[f];
            const float* hf = hn + (size_t)f * B * NS;
            const bool fmiss = miss && !is_cat;
            float M[8] = {0};
            if (fmiss)
                for (int s = 0; s < NS; ++s) M[s] = hf[(size_t)(B - 1) * NS + s];
            for (int s = 0; s < NS; ++s) run[s] = 0.f;
            for (int b = 0; b < B; ++b) {
                for (int s = 0; s < NS; ++s) {
                    run[s] += hf[(size_t)b * NS + s];
                    lf[s] = is_cat ? hf[(size_t)b * NS + s] : run[s];
                    rt[s] = T[s] - lf[s];
                }
                if (fmiss && b == B - 1) break;
                for (int v = 0; v < (fmiss ? 2 : 1); ++v) {
                    if (v == 1)
                        for (int s = 0; s < NS; ++s) { lf[s] += M[s]; rt[s] -= M[s]; }
                    if (split_weight(lf, NS, crit) < min_leaf || split_weight(rt, NS, crit) < min_leaf) continue;
                    if (is_cat && b >= n_edges) continue;
                    const float g = split_score(lf, NS, crit, lam, alpha) + split_score(rt, NS, crit, lam, alpha) - parent;
                    const int i = (f * B + b) * 2 + v;
                    if (g > best || (g == best && i < best_i)) {
                        best = g;
                        best_i = i;
                        for (int s = 0; s < NS; ++s) Lb[s] = lf[s];
                    }
                }
            }
        }
        const bool found = best_i != 0x7FFFFFFF;
        const int fb = best_i >> 1;
        gain[node] = found ? best : -INFINITY;
        feat[node] = found ? fb / B : 0;
        bin[node] = found ? (fb % B) | ((best_i & 1) << 16) : 0;
        for (int s = 0; s < NS; ++s) {
            left[node * NS + s] = Lb[s];
            tot[node * NS + s] = T[s];
        }
    }
    return 0;
}
