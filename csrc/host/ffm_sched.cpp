// Conflict-aware row scheduling for the Hogwild FFM kernels (a CYCLADES-
// style experiment).  The pipelined fp32 kernel (csrc/kernels/ffm.hip ffm_pipe_sg32_kernel) runs
// block b over rows b, b + G, b + 2G, ... with ~512 blocks resident, so the rows whose read-
// modify-writes overlap in time are (to first order) the 512 consecutive row indices of one
// "time slot" (generation g = b / 512, position p = r / G).  This pass assigns each row of a
// batch to one of S slots of equal capacity so that rows sharing a feature of the given band
// land in different (and non-adjacent) slots where possible: greedy, rows in stream order, each
// row to the open slot with the fewest band-feature co-occurrences within +-window slots.
// ops/ffm_sched.py turns the slot assignment into the row permutation the kernel sees.
#include <cstdint>
#include <cstring>
#include <vector>

#define HM_API extern "C" __attribute__((visibility("default")))

// idx [B, F] feature ids; band [NF] -> compact band id or -1; S slots of B / S rows each
// (B % S == 0); slot_out [B].  Returns the number of band co-occurrences the assignment kept
// inside +-window slots (the greedy's objective), or -1 on bad arguments.
HM_API long long hm_ffm_schedule_slots(const int32_t* idx, int B, int F, const int32_t* band,
                                       int NF, int nband, int S, int window, int32_t* slot_out) {
    if (B <= 0 || F <= 0 || S <= 0 || B % S || nband < 0 || window < 0) return -1;
    const int cap = B / S;
    std::vector<uint16_t> cnt((size_t)nband * S, 0);
    std::vector<int> fill(S, 0);
    std::vector<int32_t> cost(S), wc(S);
    std::vector<int> fb;
    fb.reserve(F);
    long long kept = 0;
    int rot = 0;
    for (int r = 0; r < B; ++r) {
        fb.clear();
        const int32_t* row = idx + (size_t)r * F;
        for (int j = 0; j < F; ++j) {
            const int i = row[j];
            if (i >= 0 && i < NF && band[i] >= 0) fb.push_back(band[i]);
        }
        std::memset(cost.data(), 0, sizeof(int32_t) * S);
        for (int c : fb) {
            const uint16_t* cc = cnt.data() + (size_t)c * S;
            for (int t = 0; t < S; ++t) cost[t] += cc[t];
        }
        if (window > 0) {
            for (int t = 0; t < S; ++t) {
                int s = 0;
                for (int d = -window; d <= window; ++d) {
                    const int u = t + d;
                    if (u >= 0 && u < S) s += cost[u];
                }
                wc[t] = s;
            }
        } else {
            wc = cost;
        }
        int best = -1;
        int32_t bc = 0;
        for (int k = 0; k < S; ++k) {
            const int t = (rot + k) % S;   // rotating start: ties spread over the slots
            if (fill[t] >= cap) continue;
            if (best < 0 || wc[t] < bc) { best = t; bc = wc[t]; if (bc == 0) break; }
        }
        rot = (best + 1) % S;
        slot_out[r] = best;
        ++fill[best];
        kept += bc;
        for (int c : fb) {
            uint16_t& v = cnt[(size_t)c * S + best];
            if (v < 65535) ++v;
        }
    }
    return kept;
}
