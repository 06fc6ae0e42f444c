"""Expected LDS bank-conflict cycles of the tree histogram's 64-bit LDS adds (hist_kernel, packed
statistic pairs) when a wave's 64 lanes add at independent uniformly random bins.

gfx950 services an 8-byte LDS write-class access in 4 groups of 16 lanes, bank = (address / 4) mod
32 (MI355X_MICROARCH.md §LDS), so an 8-B histogram entry at bin b occupies bank pair b mod 16 of
its feature's sub-histogram (whose base is a multiple of 32 banks).  Each extra distinct address
on a busy bank pair adds one cycle.  This prints the expectation per wave-instruction of the
row-per-lane mapping (every lane of an instruction adds the same feature, so its bank is set by
its random bin): 7.7-8.3, against 6.7-7.7 measured.  A feature-per-lane mapping with a
[bin][feature] image takes the bin out of the bank; round 5 built it and measured 0.2-0.3
conflict cycles per instruction, but a slower kernel (docs/perf_notes.md, profiles/r5/hist_fl/).

    python benchmarks/lds_conflict_model.py
"""
import numpy as np


def main(trials=20000, seed=0):
    rng = np.random.default_rng(seed)
    tot_any, tot_distinct = 0.0, 0.0
    for _ in range(4):                                  # 4 lane groups of 16
        b = rng.integers(0, 256, size=(trials, 16))
        cnt = np.zeros((trials, 16), int)
        np.add.at(cnt, (np.arange(trials)[:, None], b % 16), 1)
        tot_any += (cnt.max(1) - 1).mean()
        e = [np.bincount(np.unique(r) % 16, minlength=16).max() - 1 for r in b]
        tot_distinct += float(np.mean(e))
    print({"extra_cycles_per_instr_all_lanes": round(tot_any, 2),
           "extra_cycles_per_instr_distinct_addresses": round(tot_distinct, 2)})


if __name__ == "__main__":
    main()
