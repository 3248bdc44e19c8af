#!/usr/bin/env python3
"""In-forward per-stage profile of the north-star forward from rocprofv3 runs (tools/forward_profile.sh).

    python tools/forward_profile.py TRACE_kernel_trace.csv MFMA_counter_collection.csv OUT.json [--forwards N]

TRACE: `rocprofv3 --kernel-trace` over bench.py --no-breakdown (every forward of the timed loop runs as
in production: one launch per kernel, no replay).  The last N bf16 forwards are used; per stage: launches
per forward, mean duration per launch, the stage's share of the forward, and the forward's own span
(first kernel start -> last kernel end) so that the per-stage sums can be checked against ms_per_step.

MFMA: `rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace` over
tools/traffic_driver.py (same forward).  MFMA utilisation of a dispatch (MI355X_MICROARCH.md, constants
table and DVFS item): SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) - the busy cycles are
summed over every SIMD, GRBM_GUI_ACTIVE over the 8 XCDs.  The FLOP-rate fraction (algorithmic FLOP /
(duration x 2.5 PF)) is printed beside it: it also charges the clock the chip holds under load.
"""
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stage_trace import stage_of  # noqa: E402

PEAK_TF = 2500.0


def clean(name):
    return re.sub(r"\(anonymous namespace\)::", "", re.sub(r"^(void )?cfm::", "", name))


def forwards_from_trace(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    rows = [r for r in rows if "cfm" in r["Kernel_Name"] or "gemm" in r["Kernel_Name"]]
    starts = [i for i, r in enumerate(rows) if "calc_length" in r["Kernel_Name"]]
    fws = []
    for j, s0 in enumerate(starts):
        seg = rows[s0:starts[j + 1] if j + 1 < len(starts) else len(rows)]
        if any("conv1_kernel<unsigned short>" in r["Kernel_Name"] or "conv12" in r["Kernel_Name"] for r in seg):
            fws.append(seg)
    return fws


def stage_table(fws, n):
    sel = fws[-n:]
    agg, spans, sums = {}, [], []
    for seg in sel:
        state = {"resid": 0}
        t0 = min(int(r["Start_Timestamp"]) for r in seg)
        t1 = max(int(r["End_Timestamp"]) for r in seg)
        spans.append((t1 - t0) / 1e3)
        s = 0.0
        for r in seg:
            st = stage_of(clean(r["Kernel_Name"]), state)
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            s += dur
            if st is None:
                st = "other"
            a = agg.setdefault(st, [0, 0.0])
            a[0] += 1
            a[1] += dur
        sums.append(s)
    return agg, spans, sums


def mfma_table(path):
    disp = {}
    for r in csv.DictReader(open(path)):
        e = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "busy": 0.0, "gui": 0.0})
        if r["Counter_Name"] == "SQ_VALU_MFMA_BUSY_CYCLES":
            e["busy"] += float(r["Counter_Value"])
        elif r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            e["gui"] += float(r["Counter_Value"])
    rows = [disp[k] for k in sorted(disp) if "cfm" in disp[k]["name"] or "gemm" in disp[k]["name"]]
    start = max(i for i, r in enumerate(rows) if "calc_length" in r["name"])
    state, agg = {"resid": 0}, {}
    for r in rows[start:]:
        st = stage_of(clean(r["name"]), state) or "other"
        a = agg.setdefault(st, [0.0, 0.0])
        a[0] += r["busy"]
        a[1] += r["gui"]
    return {k: (v[0] / (1024.0 * v[1] / 8.0) if v[1] > 0 else None) for k, v in agg.items()}


def main(argv):
    trace, mfma, out = argv[0], argv[1], argv[2]
    n = int(argv[argv.index("--forwards") + 1]) if "--forwards" in argv else 5
    import bench
    work = bench.stage_work(32, 1000, 512, 17, 8)
    fws = forwards_from_trace(trace)
    agg, spans, sums = stage_table(fws, n)
    util = mfma_table(mfma) if mfma and os.path.exists(mfma) else {}
    nf = min(n, len(fws))
    span = sum(spans) / len(spans)
    res = {"source": "rocprofv3 --kernel-trace over bench.py --no-breakdown (in-forward: every kernel launched once, "
                     f"as in production), mean of the last {nf} bf16 forwards; MFMA utilisation from "
                     "SQ_VALU_MFMA_BUSY_CYCLES / (1024 x GRBM_GUI_ACTIVE / 8) over tools/traffic_driver.py",
           "forward_span_us": round(span, 1), "kernel_sum_us": round(sum(sums) / len(sums), 1), "stages": {}}
    print(f"forward span (first kernel start -> last end): {span:.1f} us; sum of kernel durations "
          f"{sum(sums) / len(sums):.1f} us ({nf} forwards)")
    print(f"{'stage':18s} {'n':>3s} {'us/launch':>10s} {'us/forward':>10s} {'share':>6s} {'TF/s':>7s} "
          f"{'flop_frac':>9s} {'mfma_util':>9s}")
    for st, (cnt, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        per_fw = tot / nf
        per_launch = tot / cnt
        kind, amt = work.get(st, ("byte", 0))
        t_work = per_fw if st in bench.WORK_PER_FORWARD else per_launch
        rate = amt / (t_work * 1e-6) / (1e12 if kind == "flop" else 1e9) if amt else None
        frac = rate / PEAK_TF if (rate and kind == "flop") else None
        u = util.get(st)
        res["stages"][st] = {"launches_per_forward": cnt // nf, "us_per_launch": round(per_launch, 2),
                             "us_per_forward": round(per_fw, 1), "share_of_span": round(per_fw / span, 4),
                             ("TFLOP/s" if kind == "flop" else "GB/s"): None if rate is None else round(rate, 1),
                             "flop_frac_of_peak": None if frac is None else round(frac, 4),
                             "mfma_util": None if u is None else round(u, 4)}
        print(f"{st:18s} {cnt // nf:3d} {per_launch:10.2f} {per_fw:10.1f} {per_fw / span:6.3f} "
              f"{'' if rate is None else f'{rate:7.1f}'} {'' if frac is None else f'{frac:9.4f}'} "
              f"{'' if u is None else f'{u:9.4f}'}")
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
