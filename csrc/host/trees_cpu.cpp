// CPU twins of csrc/kernels/trees.hip (same layouts and semantics), OpenMP-parallel.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#define HM_API extern "C" __attribute__((visibility("default")))
#define HM_TREE_CAT 0x40000000  // nominal split flag (csrc/kernels/trees.hip)

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
                f &= ~HM_TREE_CAT;
                const float v = x[f];
                k = (cat ? v == threshold[k] : v <= threshold[k]) ? left[k] : right[k];  // NaN goes right
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
                             const int32_t* left_child, const int32_t* right_child) {
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < n; ++r) {
        const int nd = node_of_row[r];
        if (nd < 0) continue;
        int f = split_feat[nd];
        if (f < 0) continue;
        const bool cat = f & HM_TREE_CAT;
        f &= ~HM_TREE_CAT;
        const int b = bins[r * dpad + f];
        node_of_row[r] = (cat ? b == split_bin[nd] : b <= split_bin[nd]) ? left_child[nd] : right_child[nd];
    }
    return 0;
}
