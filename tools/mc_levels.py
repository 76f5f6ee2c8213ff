"""Per-level profile of the MCCompletePathV2 combine (PPR_MC_LEVEL_LOG=1): where the time goes by
level size and by the level's largest hub.

    PPR_MC_LEVEL_LOG=1 python bench.py --workload mc --steps 1 --warmup 0 --no-cpu-baseline 2> lv.txt
    python tools/mc_levels.py lv.txt
"""
import sys

import numpy as np

rows = [tuple(float(x) for x in ln.split()[1:]) for ln in open(sys.argv[1]) if ln.startswith("mc_level ")]
a = np.array(rows)  # level, size, hubs, max need, ms
nl = int(a[:, 0].max()) + 1
a = a[-nl:]  # the last combine
lv, size, hubs, need, ms = a.T
print(f"levels {nl}  total {ms.sum():.1f} ms  levels with hubs {(hubs > 0).sum()}")
for lo, hi in [(0, 1), (1, 16), (16, 256), (256, 4096), (4096, 1 << 30)]:
    m = (size >= lo) & (size < hi)
    print(f"  level size [{lo}, {hi}): {m.sum():5d} levels {ms[m].sum():8.1f} ms  mean {ms[m].mean() if m.any() else 0:.3f}")
for lo, hi in [(0, 1), (1, 1 << 14), (1 << 14, 1 << 17), (1 << 17, 1 << 20), (1 << 20, 1 << 40)]:
    m = (need >= lo) & (need < hi)
    print(f"  largest hub [{lo}, {hi}): {m.sum():5d} levels {ms[m].sum():8.1f} ms  mean {ms[m].mean() if m.any() else 0:.3f}")
top = np.argsort(-ms)[:10]
print("slowest levels (level, size, hubs, max need, ms):")
for i in top:
    print("  ", int(lv[i]), int(size[i]), int(hubs[i]), int(need[i]), round(ms[i], 3))
