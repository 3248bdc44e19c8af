#!/usr/bin/env python3
"""Per-launch durations of chosen kernels from a rocprofv3 kernel-trace csv, grouped by grid:
    python tools/tn_trace.py TRACE.csv [name_substring ...]"""
import collections
import csv
import sys


def main():
    subs = sys.argv[2:] or ["tn_glds"]
    groups = collections.OrderedDict()
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            if not any(s in name for s in subs):
                continue
            grid = (r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Grid_Size_Y", ""), r.get("Grid_Size_Z", ""),
                    r.get("Workgroup_Size_X", r.get("Workgroup_Size", "")))
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
            groups.setdefault((name[:40], grid), []).append(dur)
    tot = 0.0
    for (name, grid), ds in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        tot += sum(ds)
        print(f"{name:40s} grid {str(grid):34s} n {len(ds):4d} avg {sum(ds) / len(ds):8.2f} us  total {sum(ds) / 1000:7.3f} ms")
    print(f"total {tot / 1000:.3f} ms")


if __name__ == "__main__":
    main()
