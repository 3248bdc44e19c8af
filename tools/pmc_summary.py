#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per kernel over one or more counter_collection.csv files."""
import collections
import csv
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).replace("cfm::", "")[:70]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in acc.items():
    if "cfm" not in name and "kernel" not in name:
        continue
    print(name)
    for c, v in sorted(cs.items()):
        print(f"    {c:32s} {sum(v) / len(v):16.1f}   (n={len(v)})")
