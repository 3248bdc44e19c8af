#!/usr/bin/env python3
"""Per-stage HBM traffic per launch from two rocprofv3 --pmc passes over tools/traffic_driver.py.

    python tools/traffic_summary.py FETCH_counter_collection.csv WRITE_counter_collection.csv OUT.json

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced streaming read (16 B/lane global_load and buffer_load...lds alike) -> doubled here.
WRITE_SIZE is exact for 16-B-per-lane streaming stores.  rocprofv3 reports both in KiB.
The last forward's dispatches are mapped to stages with tools/stage_trace.py's rules.
"""
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from stage_trace import stage_of  # noqa: E402


def per_stage(path, counter):
    disp = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        e = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "value": 0.0})
        e["value"] += float(r["Counter_Value"])         # summed over instance dimensions
    rows = [disp[k] for k in sorted(disp) if "cfm" in disp[k]["name"] or "gemm_kernel" in disp[k]["name"]]
    start = max(i for i, r in enumerate(rows) if "calc_length" in r["name"])
    state, agg = {"resid": 0}, {}
    for r in rows[start:]:
        name = re.sub(r"\(anonymous namespace\)::", "", re.sub(r"^(void )?cfm::", "", r["name"]))
        st = stage_of(name, state)
        if st is not None:
            a = agg.setdefault(st, [0, 0.0])
            a[0] += 1
            a[1] += r["value"]
    return {k: v[1] / v[0] for k, v in agg.items()}


def main(fetch_csv, write_csv, out_path):
    fetch = per_stage(fetch_csv, "FETCH_SIZE")
    write = per_stage(write_csv, "WRITE_SIZE")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, kernel-trace only) over "
                     "tools/traffic_driver.py: Large-17 B=32 T=1000 bf16 single-stream forward; per-launch average "
                     "of each stage's kernels in the last forward; FETCH_SIZE x2 (gfx950 correction); KiB -> bytes",
           "stages": {}}
    for stage in fetch:
        fb, wb = 2 * fetch[stage] * 1024, write.get(stage, 0.0) * 1024
        out["stages"][stage] = {"fetch_bytes": round(fb), "write_bytes": round(wb), "hbm_bytes": round(fb + wb)}
        print(f"{stage:20s} fetch {fb / 1e6:9.2f} MB  write {wb / 1e6:9.2f} MB  per launch")
    json.dump(out, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:4])
