#!/usr/bin/env python3
"""Kernel-by-kernel listing of chosen GRank iterations from a rocprofv3 kernel trace (start / end in
ms from the iteration's k_classify, hardware queue, workgroups): where the GPU idles between an
iteration's stages and which streams overlap.

    python tools/iter_kernels.py gpurun_out/<tag>/prof/.../run_kernel_trace.csv [iteration ...]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
its = [int(x) for x in sys.argv[2:]] or [10, 11]
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pprk::", "")[:40], int(r["Queue_Id"]),
             int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))) for r in rows)
cls = [i for i, k in enumerate(ks) if k[2] == "k_classify"]
starts = cls[-31:]  # init + 30 iterations of the last job
print("sum of the 30 iteration spans: %.1f ms" % sum((ks[starts[i + 1]][0] - ks[starts[i]][0]) / 1e6 for i in range(30)))
for it in its:
    a, b = starts[it], starts[it + 1]
    t0 = ks[a][0]
    print(f"iteration {it}: {(ks[b][0] - t0) / 1e6:.2f} ms")
    for s, e, n, q, nb in ks[a:b]:
        print(f"  {(s - t0) / 1e6:7.2f} {(e - t0) / 1e6:7.2f} q{q} {n} [{nb}]")
