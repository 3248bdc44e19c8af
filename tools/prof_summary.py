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


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
