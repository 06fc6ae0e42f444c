"""Expected LDS bank-conflict cycles of the tree histogram's 64-bit LDS adds (hist_kernel, packed
statistic pairs) when a wave's 64 lanes add at independent uniformly random bins.

gfx950 services an 8-byte LDS write-class access in 4 groups of 16 lanes, bank = (address / 4) mod
32 (MI355X_MICROARCH.md §LDS), so an 8-B histogram entry at bin b occupies bank pair b mod 16 of
its feature's sub-histogram (whose base is a multiple of 32 banks).  Each extra distinct address
on a busy bank pair adds one cycle.  This prints the expectation per wave-instruction, which any
row -> lane or feature -> bank mapping leaves unchanged while the bins are random: the bank of
every lane is set by its bin.

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
