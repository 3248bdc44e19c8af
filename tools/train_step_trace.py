#!/usr/bin/env python3
"""Per-kernel totals of the LAST training step in a rocprofv3 kernel-trace csv (steps delimited by
the optimizer's multi-tensor kernels):  python tools/train_step_trace.py TRACE.csv [top]"""
import collections
import csv
import sys


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")))
    rows.sort()
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    opt = [i for i, r in enumerate(rows) if "multi_tensor_apply" in r[2] or "FusedOptimizer" in r[2]]
    if not opt:
        sys.exit("no optimizer kernels in the trace")
    # optimizer groups: runs of optimizer kernels with no other kernel between them
    ends = [opt[k] for k in range(len(opt)) if k + 1 == len(opt) or opt[k + 1] != opt[k] + 1]
    lo = ends[-2] + 1 if len(ends) > 1 else 0
    step = rows[lo:ends[-1] + 1]
    span = (step[-1][1] - step[0][0]) / 1000.0
    gaps = sorted(((step[i + 1][0] - step[i][1]) / 1000.0, i) for i in range(len(step) - 1))[::-1]
    tot = collections.OrderedDict()
    for s, e, n in step:
        k = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:90]
        c, t = tot.get(k, (0, 0.0))
        tot[k] = (c + 1, t + (e - s) / 1000.0)
    ksum = sum(t for _, t in tot.values())
    print(f"last step: {len(step)} kernels, span {span:.1f} us, kernel sum {ksum:.1f} us, steps seen {len(ends)}")
    print("largest gaps (us, after kernel -> before kernel):")
    for g, i in gaps[:25]:
        a = step[i][2].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        b = step[i + 1][2].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        print(f"  {g:8.1f}  #{i:5d} {a}  ->  {b}")
    nm = lambda i: step[i][2].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]  # noqa: E731
    for g, i in gaps[:4]:
        print(f"-- around the {g:.1f} us gap after #{i}:")
        for j in range(max(0, i - 10), min(len(step), i + 6)):
            gp = (step[j][0] - step[j - 1][1]) / 1000.0 if j else 0.0
            print(f"   #{j:5d} gap {gp:8.1f} dur {(step[j][1] - step[j][0]) / 1000.0:8.1f}  {nm(j)}")
    print(f"gaps > 20 us: {sum(g for g, _ in gaps if g > 20):.1f} us in {sum(1 for g, _ in gaps if g > 20)}; "
          f"all gaps {sum(g for g, _ in gaps if g > 0):.1f} us")
    print(f"{'kernel':90s} {'n':>5s} {'total_us':>10s} {'avg_us':>8s} {'pct':>6s}")
    for k, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{k:90s} {c:5d} {t:10.1f} {t / c:8.2f} {100 * t / ksum:6.2f}")


if __name__ == "__main__":
    main()
