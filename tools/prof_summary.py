#!/usr/bin/env python3
"""Summarise a rocprofv3 `--kernel-trace --stats` CSV (kernel_stats.csv) into a short table."""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = name.replace("cfm::", "").replace("unsigned short", "bf16")
    m = re.match(r"(?:void )?([\w:]+)(<[^()]*>)?", name)
    base = m.group(1) if m else name[:60]
    targs = (m.group(2) or "") if m else ""
    return (base + targs)[:90]


def main(path, top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'kernel':90s} {'calls':>6s} {'total_ms':>9s} {'avg_us':>9s} {'pct':>6s}")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        t = float(r["TotalDurationNs"])
        print(f"{short(r['Name']):90s} {int(r['Calls']):6d} {t / 1e6:9.3f} {float(r['AverageNs']) / 1e3:9.2f} {100 * t / tot:6.2f}")
    print(f"{'TOTAL':90s} {'':6s} {tot / 1e6:9.3f}")


def main_trace(path, top=40):
    """Group a kernel_trace.csv by (kernel, grid): separates e.g. the B=32 single-stream launches of
    forward_timed from the micro-batched B=16 launches of the timed loop."""
    agg = {}
    for r in csv.DictReader(open(path)):
        key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]))
        a = agg.setdefault(key, [0, 0.0])
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(f"{'kernel':90s} {'grid':>9s} {'calls':>6s} {'total_ms':>9s} {'avg_us':>9s}")
    for (name, grid), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{name:90s} {grid:9d} {n:6d} {t / 1e6:9.3f} {t / n / 1e3:9.2f}")


if __name__ == "__main__":
    if sys.argv[1] == "--trace":
        main_trace(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 40)
    else:
        main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
