#!/usr/bin/env python3
"""Print a bench.py JSON line compactly (value, ms/step, per-stage breakdown)."""
import json
import sys

for path in sys.argv[1:]:
    d = json.loads(open(path).read().strip().splitlines()[-1])
    print(f"== {path}: {d['value']:.0f} frames/s  {d['ms_per_step']:.3f} ms/step  "
          f"model {d['model_flops']['TFLOP/s_per_gpu']} TF/s  roof {d['roofline'] and (d['roofline']['kernel'], d['roofline']['frac'])}")
    for k, v in d.get("breakdown", {}).items():
        rate = v.get("TFLOP/s", v.get("GB/s"))
        unit = "TF/s" if "TFLOP/s" in v else "GB/s"
        print(f"   {k:18s} {v['ms_total']:8.3f} ms  x{v['launches']:<3d} {v['ms_per_launch'] * 1000:8.1f} us  {rate:8.1f} {unit}")
