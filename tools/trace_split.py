"""Median / min duration per (kernel, grid size) from a rocprofv3 kernel trace CSV (lab helper).
usage: python tools/trace_split.py gpurun_out/<dir>/run_kernel_trace.csv"""
import collections
import csv
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0]
    if "lk::" not in n:
        continue
    d[(n, r["Grid_Size_X"], r["LDS_Block_Size"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items()):
    v.sort()
    print(f"{k[0]:45s} grid={k[1]:>8s} lds={k[2]:>6s} n={len(v):4d} med {v[len(v) // 2] / 1e3:8.2f} us  min {v[0] / 1e3:8.2f}")
