// Histogram tree learning + batched tree inference for gfx950 (RandomForest / GBT).
//
// Upstream (core/src/main/java/hivemall/smile/classification/
// {DecisionTree,RandomForestClassifierUDTF,GradientTreeBoostingClassifierUDTF}.java,
// smile/regression/RegressionTree.java, smile/tools/TreePredictUDF.java) grows trees with
// exact splits over pre-sorted columns.  This engine uses LightGBM/XGBoost-hist style
// quantised splits instead (documented in docs/compat.md): features are quantised to <= 256
// bins (uint8), rows are kept grouped by tree node, and every level builds per-(node,
// feature, bin) sums of NS statistics (GBT: residual, hessian, count; RF: per-class
// bootstrap-weighted counts; regression: w·y, w).
//
// hist_build: block (tile t, node n, feature group g) walks TILE rows of node n's segment,
//   privatises the group's histogram [FG][B][NS] in LDS (ds_add_f32 float atomics; rows of
//   one node contend only on equal bins), then adds it to the global histogram with one
//   pass of global float atomics (skipping zero bins).  Feature groups keep the LDS image
//   small (FG=8, B=256, NS=3 -> 24 KB) so several blocks share a CU.
// tree_predict: one lane per (row, tree); trees are flattened SoA arrays
//   (feature, threshold, left, right, value offset) so a traversal is a chain of coalesced-ish
//   16-B loads that stay in L2 for forests of a few MB.
#include "common.h"

namespace {

constexpr int TILE = 4096;

template <int NS>
__global__ __launch_bounds__(256) void hist_kernel(const uint8_t* __restrict__ bins, int64_t n,
                                                   int d, int dpad, int B,
                                                   const int32_t* __restrict__ rows,
                                                   const int64_t* __restrict__ seg,
                                                   const int32_t* __restrict__ node_ids,
                                                   const float* __restrict__ stats, int FG,
                                                   float* __restrict__ hist) {
    extern __shared__ __attribute__((aligned(16))) float s_hist[];
    const int node = blockIdx.y;
    const int g = blockIdx.z;
    const int f0 = g * FG;
    const int nf = min(FG, d - f0);
    if (nf <= 0) return;
    const int64_t beg = seg[node], end = seg[node + 1];
    const int64_t t0 = beg + (int64_t)blockIdx.x * TILE;
    if (t0 >= end) return;
    const int64_t t1 = min(end, t0 + TILE);
    const int hsz = nf * B * NS;
    for (int i = threadIdx.x; i < hsz; i += blockDim.x) s_hist[i] = 0.f;
    __syncthreads();
    for (int64_t q = t0 + threadIdx.x; q < t1; q += blockDim.x) {
        const int64_t r = rows ? rows[q] : q;
        float st[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) st[s] = stats[r * NS + s];
        bool zero = true;
#pragma unroll
        for (int s = 0; s < NS; ++s) zero = zero && st[s] == 0.f;
        if (zero) continue;  // out-of-bag / zero-weight rows add nothing
        const uint8_t* br = bins + r * dpad + f0;
        for (int f = 0; f < nf; ++f) {
            const int b = br[f];
            float* h = s_hist + (f * B + b) * NS;
#pragma unroll
            for (int s = 0; s < NS; ++s) atomicAdd(h + s, st[s]);
        }
    }
    __syncthreads();
    const int out_node = node_ids ? node_ids[node] : node;
    float* gh = hist + ((size_t)out_node * d + f0) * B * NS;
    for (int i = threadIdx.x; i < hsz; i += blockDim.x) {
        const float v = s_hist[i];
        if (v != 0.f) atomicAdd(gh + i, v);
    }
}

// Flattened forest: node k of the forest has feature[k] (<0: leaf), threshold[k] (go left
// when x <= threshold), left[k]/right[k] (absolute node ids), value offset voff[k] into
// values (n_out floats per leaf).  roots[t] = root node of tree t.
__global__ __launch_bounds__(256) void tree_predict_kernel(
    const float* __restrict__ X, int64_t n, int d, const int32_t* __restrict__ feature,
    const float* __restrict__ threshold, const int32_t* __restrict__ left,
    const int32_t* __restrict__ right, const int32_t* __restrict__ voff,
    const float* __restrict__ values, const int32_t* __restrict__ roots, int n_trees, int n_out,
    float* __restrict__ out /* [n, n_trees, n_out] or summed [n, n_out] */, int sum_trees,
    const float* __restrict__ tree_w) {
    const int64_t total = n * (int64_t)n_trees;
    for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = g / n_trees;
        const int t = (int)(g - row * n_trees);
        int k = roots[t];
        const float* x = X + row * d;
        for (int depth = 0; depth < 64; ++depth) {
            const int f = feature[k];
            if (f < 0) break;
            const float v = x[f];
            k = (v <= threshold[k] || v != v) ? left[k] : right[k];
        }
        const float* val = values + voff[k];
        if (sum_trees) {
            const float w = tree_w ? tree_w[t] : 1.f;
            for (int o = 0; o < n_out; ++o) atomicAdd(out + row * n_out + o, w * val[o]);
        } else {
            float* dst = out + (row * n_trees + t) * n_out;
            for (int o = 0; o < n_out; ++o) dst[o] = val[o];
        }
    }
}

// Quantisation: bins[r, f] = #edges[f] < x  (edges sorted, n_edges per feature), NaN -> last bin.
__global__ __launch_bounds__(256) void quantize_kernel(const float* __restrict__ X, int64_t n,
                                                       int d, int dpad,
                                                       const float* __restrict__ edges,
                                                       int n_edges, uint8_t* __restrict__ bins) {
    const int64_t total = n * (int64_t)d;
    for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = g / d;
        const int f = (int)(g - r * d);
        const float v = X[g];
        const float* e = edges + (size_t)f * n_edges;
        int lo = 0, hi = n_edges;
        if (v != v) {
            lo = n_edges;
        } else {
            while (lo < hi) {  // first edge >= v
                const int mid = (lo + hi) >> 1;
                if (e[mid] < v) lo = mid + 1; else hi = mid;
            }
        }
        bins[r * dpad + f] = (uint8_t)lo;
    }
}

// Row routing after a level's splits: node_of_row[r] -> child id (or stays when the node
// became a leaf).  split_feat[node] < 0 means leaf.
__global__ __launch_bounds__(256) void route_kernel(const uint8_t* __restrict__ bins, int64_t n,
                                                    int dpad, int32_t* __restrict__ node_of_row,
                                                    const int32_t* __restrict__ split_feat,
                                                    const int32_t* __restrict__ split_bin,
                                                    const int32_t* __restrict__ left_child,
                                                    const int32_t* __restrict__ right_child) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        const int nd = node_of_row[r];
        if (nd < 0) continue;
        const int f = split_feat[nd];
        if (f < 0) continue;
        const int b = bins[r * dpad + f];
        node_of_row[r] = b <= split_bin[nd] ? left_child[nd] : right_child[nd];
    }
}

}  // namespace

HM_API int hm_hist_build(const uint8_t* bins, int64_t n, int d, int dpad, int B,
                         const int32_t* rows, const int64_t* seg, const int32_t* node_ids,
                         int n_nodes, int64_t max_seg, const float* stats, int NS, int FG,
                         float* hist, hipStream_t stream) {
    if (n_nodes <= 0 || max_seg <= 0) return 0;
    if (B > 256 || NS <= 0 || NS > 8 || FG <= 0) return (int)hipErrorInvalidValue;
    const size_t lds = (size_t)FG * B * NS * sizeof(float);
    if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)((max_seg + TILE - 1) / TILE), (unsigned)n_nodes, (unsigned)((d + FG - 1) / FG));
#define HM_H(K)                                                                                     \
    case K:                                                                                         \
        hipLaunchKernelGGL((hist_kernel<K>), grid, dim3(256), lds, stream, bins, n, d, dpad, B, rows, \
                           seg, node_ids, stats, FG, hist);                                         \
        break;
    switch (NS) {
        HM_H(1) HM_H(2) HM_H(3) HM_H(4) HM_H(5) HM_H(6) HM_H(7) HM_H(8)
    }
#undef HM_H
    HM_LAUNCH_RET();
}

HM_API int hm_tree_predict(const float* X, int64_t n, int d, const int32_t* feature,
                           const float* threshold, const int32_t* left, const int32_t* right,
                           const int32_t* voff, const float* values, const int32_t* roots,
                           int n_trees, int n_out, float* out, int sum_trees, const float* tree_w,
                           hipStream_t stream) {
    const int64_t total = n * (int64_t)n_trees;
    if (total <= 0) return 0;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(tree_predict_kernel, dim3((int)blocks), dim3(256), 0, stream, X, n, d, feature,
                       threshold, left, right, voff, values, roots, n_trees, n_out, out, sum_trees,
                       tree_w);
    HM_LAUNCH_RET();
}

HM_API int hm_quantize(const float* X, int64_t n, int d, int dpad, const float* edges, int n_edges,
                       uint8_t* bins, hipStream_t stream) {
    const int64_t total = n * (int64_t)d;
    if (total <= 0) return 0;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(quantize_kernel, dim3((int)blocks), dim3(256), 0, stream, X, n, d, dpad, edges,
                       n_edges, bins);
    HM_LAUNCH_RET();
}

HM_API int hm_route_rows(const uint8_t* bins, int64_t n, int dpad, int32_t* node_of_row,
                         const int32_t* split_feat, const int32_t* split_bin,
                         const int32_t* left_child, const int32_t* right_child, hipStream_t stream) {
    if (n <= 0) return 0;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(route_kernel, dim3((int)blocks), dim3(256), 0, stream, bins, n, dpad,
                       node_of_row, split_feat, split_bin, left_child, right_child);
    HM_LAUNCH_RET();
}
