#!/usr/bin/env python3
"""Per-stage kernel durations from a rocprofv3 kernel_trace.csv of `bench.py` (tools/profile_round.sh),
for checking bench.py's breakdown / roofline (burst-replay HIP events) against the profiler.

Only the single-stream forwards of the breakdown (the launches whose calc_length is followed by
the full-batch kernels, i.e. the LAST `--forwards` forwards of the trace) are used.  Kernels map to
stages by name; the RESID GEMMs of a layer run in the fixed order ffn_down, out_proj, pw2, ffn_down.
    python tools/stage_trace.py run_kernel_trace.csv [bench.json] [--forwards 3] [--burst 8]
The breakdown replays every launch `burst` times back-to-back; those replays are collapsed here
into one launch whose duration is the replays' average.
"""
import csv
import json
import re
import sys

RESID_ORDER = ["ffn_down_gemm", "out_proj_gemm", "pw2_gemm", "ffn_down_gemm"]
EPI_STAGE = {"0": "pos_gemm", "2": "ffn_up_gemm", "4": "subsample_linear", "5": "pw1_glu_gemm", "6": "qkv_gemm",
             "7": "pw1_glu_gemm"}   # 7: pointwise_conv1 + GLU + depthwise conv + BN + Swish in one launch


def stage_of(name, state):
    if name.startswith("calc_length"):
        state["resid"] = 0
        state["pos_done"] = False
        return "lengths"
    if name.startswith("conv1_kernel"):
        return "conv1"
    if name.startswith("layernorm_kernel"):
        return "layernorm"
    if "qkv_rel_attn" in name:         # fused QKV projection + attention
        return "qkv_attention"
    if "rel_attn" in name:
        return "rel_attention"
    if name.startswith("dwconv"):
        return "dwconv_bn_swish"
    if name.startswith("transpose_kernel"):
        return "output"
    if "gemm8_kernel" in name or name.startswith(("conv12_kernel", "cfm::(anonymous namespace)::conv12_kernel")):
        return "conv2_gemm"             # the 8-phase conv2 implicit GEMM (with conv.0 fused: conv12_kernel)
    if "conv12_patch_kernel" in name:   # the fused front end's per-pixel input patches (bench: conv2 stage)
        return "conv2_gemm"
    m = re.match(r"(?:void )?(?:cfm::)?(?:\(anonymous namespace\)::)?gemm_kernel<[^,]+, (\d+),", name)
    if m:
        if "ALoadConv" in name:
            return "conv2_gemm"
        if m.group(1) == "3":
            s = RESID_ORDER[state["resid"] % 4]
            state["resid"] += 1
            return s
        if m.group(1) == "0":
            # plain-store GEMMs: the first of a forward is the position projection, the others are
            # the layers' QKV projections (natural-layout attention, bf16)
            if not state.get("pos_done"):
                state["pos_done"] = True
                return "pos_gemm"
            return "qkv_gemm"
        return EPI_STAGE.get(m.group(1), "gemm_other")
    return None


def main(argv):
    path = argv[0]
    nfw, burst = 3, 8
    if "--forwards" in argv:
        nfw = int(argv[argv.index("--forwards") + 1])
    if "--burst" in argv:
        burst = int(argv[argv.index("--burst") + 1])
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    rows = [r for r in rows if "cfm" in r["Kernel_Name"] or "gemm_kernel" in r["Kernel_Name"]]
    # collapse the timed forward's bursts (identical consecutive dispatches) into launches
    launches = []
    for r in rows:
        key = (r["Kernel_Name"], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if launches and launches[-1][0] == key and launches[-1][1] < burst:
            launches[-1][1] += 1
            launches[-1][2] += dur
        else:
            launches.append([key, 1, dur])
    starts = [i for i, l in enumerate(launches) if "calc_length" in l[0][0]]
    # keep the bf16 forwards (bench.py also times an fp32 parity-mode forward at the end): a forward
    # is bf16 when its conv1 launch is conv1_kernel<unsigned short>
    bf16 = []
    for j, s0 in enumerate(starts):
        end = starts[j + 1] if j + 1 < len(starts) else len(launches)
        seg = launches[s0:end]
        if any("conv1_kernel<unsigned short>" in l[0][0] for l in seg):
            bf16.append(seg)
    sel = [l for seg in bf16[-nfw:] for l in seg]
    state = {"resid": 0}
    agg = {}
    for key, n, dur in sel:
        name = re.sub(r"^(void )?cfm::", "", key[0])
        name = re.sub(r"\(anonymous namespace\)::", "", name)
        st = stage_of(name, state)
        if st is None:
            continue
        a = agg.setdefault(st, [0, 0.0])
        a[0] += 1
        a[1] += dur / n
    bench = None
    if len(argv) > 1 and argv[1].endswith(".json"):
        bench = json.loads(open(argv[1]).read().strip().splitlines()[-1]).get("breakdown", {})
    print(f"{'stage':20s} {'launches':>8s} {'rocprof_avg_us':>15s} {'bench_avg_us':>13s}")
    for st, (n, t) in agg.items():
        b = bench.get(st, {}).get("ms_per_launch") if bench else None
        print(f"{st:20s} {n // nfw:8d} {t / n:15.2f} {'' if b is None else f'{1e3 * b:13.2f}'}")


if __name__ == "__main__":
    main(sys.argv[1:])
