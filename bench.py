#!/usr/bin/env python3
"""North-star benchmark: Conformer-Large (17 layers, d512, 8 heads) encoder forward,
B=32 x T=1000 x 80-mel per GPU, eval mode, through the drop-in
`nemo.collections.asr.modules.ConformerEncoder` (one C-ABI call per forward).

    python bench.py [--gpus N --steps K --warmup W] [--compute bf16|fp16|fp32]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

`--gpus N` is authoritative: started without a torch.distributed environment (no WORLD_SIZE) and
N > 1, bench.py starts the N ranks itself (torch.distributed.run children, 127.0.0.1) before any GPU
call; under a launcher whose WORLD_SIZE differs from N it exits non-zero; the ranks count themselves
over RCCL and the line reports that count (`ranks_joined`).

Multi-GPU: utterances shard across ranks with no data-path collective in the forward (weak scaling,
per-GPU B=32); the training leg (`train`, BASELINE config 3) all-reduces its gradients over RCCL.
Times are the MAX over ranks between barrier+synchronize brackets.  Rank 0 prints ONE JSON line.
See DESIGN.md §5 for every field.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "conformer-nemo_amd"))

import torch  # noqa: E402

METRIC = "encoder audio-frames/sec, Conformer-Large B=32 T=1000 @1/2/4/8 MI355X"
PEAK = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 157.3}          # dense MFMA TFLOP/s (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0
WORK_PER_FORWARD = {"conv2_gemm"}   # stage_work amounts given per forward, not per launch


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def stage_work(B, T, d, L, H, C=None, F=80, K=31, dff=None, es=2):
    """Algorithmic work per launch of every stage: (kind, amount) with kind 'flop' or 'byte'."""
    C = C or d
    dff = dff or 4 * d
    T1 = (T - 1) // 2 + 1
    Tp = (T1 - 1) // 2 + 1
    F1 = (F - 1) // 2 + 1
    F2 = (F1 - 1) // 2 + 1
    M = B * Tp
    return {
        "conv1": ("byte", B * F * T * 4 + B * T1 * F1 * C * es),
        "conv2_gemm": ("flop", 2 * B * Tp * F2 * C * C * 9),
        "subsample_linear": ("flop", 2 * M * C * F2 * d),
        "pos_gemm": ("flop", 2 * (2 * Tp - 1) * d * L * d),
        "layernorm": ("byte", M * d * (4 + es)),
        "ffn_up_gemm": ("flop", 2 * M * d * dff),
        "ffn_down_gemm": ("flop", 2 * M * dff * d),
        "qkv_gemm": ("flop", 2 * M * d * 3 * d),
        "rel_attention": ("flop", 2 * B * Tp * d * (4 * Tp - 1)),
        "qkv_attention": ("flop", 2 * M * d * 3 * d + 2 * B * Tp * d * (4 * Tp - 1)),   # fused: both above
        "out_proj_gemm": ("flop", 2 * M * d * d),
        "pw1_glu_gemm": ("flop", 2 * M * d * 2 * d),
        "dwconv_bn_swish": ("byte", 2 * M * d * es),
        "pw2_gemm": ("flop", 2 * M * d * d),
        "output": ("byte", 2 * M * d * 4),
    }


def pmc_traffic(stage, B, T, L, compute):
    """HBM bytes per launch of `stage` from the newest committed PMC summary (profiles/*_traffic.json,
    written by tools/profile_round.sh: FETCH_SIZE x2 + WRITE_SIZE, gfx950-corrected), or None.
    Only valid for the shape it was collected on (Large-17, B=32, T=1000, bf16)."""
    import glob
    if (B, T, L, compute) != (32, 1000, 17, "bf16"):
        return None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")))
    if not files:
        return None
    st = json.load(open(files[-1]))["stages"].get(stage)
    return None if st is None else {"bytes_per_launch": st["hbm_bytes"], "fetch": st["fetch_bytes"],
                                    "write": st["write_bytes"], "file": os.path.relpath(files[-1], ROOT)}


def cpu_baseline(enc, B, T, budget_s):
    """The reference encoder's arithmetic on the host cores: oracle/conformer_torch_cpu.py, a torch-CPU
    restatement of the reference forward (bitwise equal to the imported reference and within 10 % of
    its time in the survey container: profiles/r02_cpu_baseline_check.txt), fp32, eval,
    torch.no_grad, the timed encoder's weights, the full B x T batch; a small warm-up, then the min of 2.
    Threads: the CPU share the job is given (OMP_NUM_THREADS, 16 per GPU on the GPU boxes; the box's
    os.cpu_count() is the whole host, shared with other jobs), else every core of this machine.
    The batch is cut only if the full batch would exceed `budget_s` seconds."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import conformer_torch_cpu as TC  # CPU baseline leg only
    threads = int(os.environ.get("OMP_NUM_THREADS", 0)) or (os.cpu_count() or 1)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    sd = {k: v.detach().float().cpu() for k, v in enc.state_dict().items() if v.is_floating_point()}
    cfg = dict(d_model=512, n_heads=8, n_layers=17)
    g = torch.Generator().manual_seed(0)
    t_start = time.perf_counter()
    Bs = 2
    x = torch.randn(Bs, 80, T, generator=g)
    t0 = time.perf_counter()
    TC.encoder_forward(x, None, sd, cfg)                    # warm-up at a small batch: sizes the sample
    per_utt = (time.perf_counter() - t0) / Bs
    Bs = int(max(1, min(B, budget_s / 2.0 / max(per_utt, 1e-6))))
    x = torch.randn(Bs, 80, T, generator=g)
    ts = []
    for _ in range(2):
        t0 = time.perf_counter()
        TC.encoder_forward(x, None, sd, cfg)
        ts.append(time.perf_counter() - t0)
    total = time.perf_counter() - t_start
    torch.set_num_threads(prev)
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next(ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {"value": round(Bs * T / min(ts), 1), "unit": "audio-frames/s", "cores": int(threads), "kind": "port",
            "cpu_model": cpu_model, "host_cpus_visible": os.cpu_count(),
            "threads_note": "OMP_NUM_THREADS = the CPU share the GPU box grants this job (the host's other cores "
                            "belong to other jobs)" if os.environ.get("OMP_NUM_THREADS") else "all cores",
            "sample": f"oracle/conformer_torch_cpu.py (torch-CPU restatement of the reference, fp32 eval), "
                      f"Large-17, B={Bs} x T={T} per forward, min of 2 after a B=2 warm-up, {total:.1f} s in all"}


def stage_breakdown(args, enc, dev, x, lengths, B, T, d, L, H, es):
    """Per-stage kernel durations of the forward (cfm_encoder_forward_timed: a start and a stop event in
    every kernel's dispatch packet, the durations rocprofv3's kernel trace reports; mean of 3 forwards),
    and the dominant stage's roofline entry."""
    breakdown = {}
    roof = None
    native = enc._native_for(dev)
    agg = {}
    reps = 3
    with torch.inference_mode():
        for _ in range(reps):
            for k, (ms, n) in native.forward_timed(x, lengths.to(torch.int32)).items():
                a = agg.setdefault(k, [0.0, 0])
                a[0] += ms / reps
                a[1] = n
    work = stage_work(B, T, d, L, H, es=es)
    for k, (ms, n) in agg.items():
        if n == 0:
            continue
        kind, amt = work.get(k, ("byte", 0))
        per = ms / n
        # conv2's work is the whole conv.0 + conv.2 (one fused kernel plus its patch pre-pass)
        rate = amt / ((ms if k in WORK_PER_FORWARD else per) * 1e-3) / (1e12 if kind == "flop" else 1e9)
        breakdown[k] = {"ms_total": round(ms, 4), "launches": n, "ms_per_launch": round(per, 5),
                        ("TFLOP/s" if kind == "flop" else "GB/s"): round(rate, 1)}
    dom = max((k for k in agg if agg[k][1]), key=lambda k: agg[k][0])
    kind, amt = work[dom]
    per_ms = agg[dom][0] if dom in WORK_PER_FORWARD else agg[dom][0] / agg[dom][1]
    tr = pmc_traffic(dom, B, T, L, args.compute)
    traffic = None if tr is None else tr["bytes_per_launch"]
    if kind == "flop":
        ach = amt / (per_ms * 1e-3) / 1e12
        roof = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 1), "peak": PEAK[args.compute],
                "unit": "TFLOP/s", "frac": round(ach / PEAK[args.compute], 4), "traffic": traffic,
                "per_launch": f"{amt / 1e9:.2f} GFLOP in {per_ms:.4f} ms (start + stop event in each kernel's dispatch packet, {agg[dom][1]} launches per forward)"}
    else:
        ach = amt / (per_ms * 1e-3) / 1e9
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "per_launch": f"{amt / 1e6:.2f} MB in {per_ms:.4f} ms"}
    roof["traffic_unit"] = "bytes/launch (HBM, PMC)"
    if tr is not None:
        roof["traffic_source"] = tr["file"]
    # the clock's own cost per kernel (empty kernels timed the same way), reported beside the sum
    try:
        breakdown["_clock_overhead_us"] = round(native.stage_clock_overhead_us(200), 3)
    except Exception:  # noqa: BLE001 - an older library: no calibration entry
        pass
    return roof, breakdown


def parity_and_fp32(dev, B, T, steps=5):
    """What the bf16 headline hides (rank 0, after the timed loop):
    * the error of every compute mode at the timed shape against the REFERENCE encoder: the two
      reference utterances of tests/golden/enc_large17.npz (Large-17, outputs of the reference
      ConformerEncoder, fp32 CPU) embedded at positions 5 and 30 of a B x T batch, weights from the
      golden's seed recipe (tests/golden/recipe.py) -> relL2 per compute mode (north-star gate:
      relL2 <= 1e-3);
    * the throughput of the two modes that meet that gate, at the same shape: fp32
      (v_mfma_f32_32x32x2_f32 contractions) and fp16 (libcfm_f16.so: the bf16 kernels with fp16
      operands, same MFMA rate)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from recipe import make_state_dict  # fixture recipe (checker only)
    from nemo.collections.asr.modules import ConformerEncoder
    z = np.load(os.path.join(ROOT, "tests", "golden", "enc_large17.npz"))
    cfg = dict(d_model=512, n_heads=8, n_layers=17)
    sd = make_state_dict(cfg, int(z["seed"]))
    enc = ConformerEncoder(feat_in=80, n_layers=17, d_model=512, n_heads=8)
    ref_sd = enc.state_dict()
    enc.load_state_dict({k: torch.from_numpy(np.asarray(v)).reshape(ref_sd[k].shape) for k, v in sd.items()})
    enc = enc.to(dev).eval()
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(B, 80, T, device=dev, generator=g)
    ln = torch.full((B,), T, dtype=torch.int64, device=dev)
    slots = [5 % B, 30 % B]
    for i, s in enumerate(slots):
        x[s] = torch.from_numpy(z["x"][i]).to(dev)
        ln[s] = int(z["lengths"][i])
    out = {"reference": "tests/golden/enc_large17.npz: reference ConformerEncoder outputs (fp32, CPU) for 2 "
                        f"utterances embedded in the B={B} x T={T} batch", "gate_fp32_relL2": 1e-3}
    yref = torch.from_numpy(z["y"]).to(dev, torch.float64)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from conformer_oracle import encoder_flops
    lines = {}
    for compute in ("bf16", "fp16", "fp32"):
        enc.set_compute_mode(compute)
        with torch.inference_mode():
            y, yl = enc(audio_signal=x, length=ln)
            y = y[slots].to(torch.float64)
            out[f"{compute}_relL2"] = float((y - yref).norm() / yref.norm())
            out[f"{compute}_max_abs_err_over_max_ref"] = float((y - yref).abs().max() / yref.abs().max())
            if compute != "bf16":
                n = steps if compute == "fp32" else 4 * steps
                for _ in range(2):
                    enc(audio_signal=x, length=ln)
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(n):
                    enc(audio_signal=x, length=ln)
                torch.cuda.synchronize(dev)
                ms = 1000.0 * (time.perf_counter() - t0) / n
                tf = encoder_flops(B, T, 512, 17) / (ms * 1e-3) / 1e12
                lines[compute] = {"ms_per_step": round(ms, 3), "value": round(B * T / (ms * 1e-3), 1),
                                  "unit": "audio-frames/s", "TFLOP/s": round(tf, 1),
                                  f"frac_of_{compute}_mfma_peak": round(tf / PEAK[compute], 4), "steps": n,
                                  "relL2": round(out[f"{compute}_relL2"], 7)}
    enc.set_compute_mode("bf16")
    return out, lines["fp32"], lines["fp16"]


def max_over_ranks(elapsed, dev, dist):
    """Wall time of the job = MAX of the per-rank elapsed times (ranks run replicas)."""
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def job_throughput(t_max, world, B, T, steps):
    """Whole-job audio-frames/s: every rank processes its own B utterances of T frames per step."""
    return world * B * T * steps / t_max


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` started without a torch.distributed environment: start N ranks, one per GPU,
    as children of this process (torch.distributed.run, 127.0.0.1 rendezvous) BEFORE anything here touches
    the GPU, and return their exit status.  Rank 0 prints the one JSON line."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "16")
    return subprocess.call(cmd, env=env)


def check_world(gpus, world):
    """--gpus N and the launcher's WORLD_SIZE must agree (a mismatch would time the wrong job)."""
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: refusing to report a "
                         f"{world}-rank job as {gpus} GPUs")


def ranks_joined(dev, dist):
    """Number of ranks that joined the process group, counted by an all-reduce over it (RCCL on GPUs)."""
    if not dist:
        return 1
    t = torch.ones(1, dtype=torch.float64, device=dev)
    torch.distributed.all_reduce(t)
    return int(t.item())


def dry_run(args, world, rank):
    """--dry-run: the launcher and rendezvous only, on CPU (gloo): every rank joins, rank 0 prints the
    rank count.  Lets tests check `--gpus N` without a GPU."""
    dist = world > 1
    if dist:
        torch.distributed.init_process_group("gloo")
    n = ranks_joined(torch.device("cpu"), dist)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks_joined": n, "gpus_arg": args.gpus, "dry_run": True}), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node; without a torch.distributed environment bench.py starts N ranks itself")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/rendezvous check on CPU (gloo): no GPU, prints the ranks that joined")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--compute", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=1000)
    ap.add_argument("--layers", type=int, default=17)
    ap.add_argument("--cpu-budget", type=float, default=40.0,
                    help="seconds of CPU-baseline timing (torch-CPU restatement of the reference; 0 = skip)")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the bf16/fp32 relL2 against the reference golden and the fp32-mode throughput line")
    ap.add_argument("--no-breakdown", action="store_true")
    ap.add_argument("--no-train", action="store_true",
                    help="forward mode: skip the config-3 training-step leg reported under 'train'")
    ap.add_argument("--train-steps", type=int, default=10)
    ap.add_argument("--train-warmup", type=int, default=3)
    ap.add_argument("--mode", default="forward", choices=["forward", "train", "joint", "rnnt_train", "stream", "cache_stream", "mel", "decode"],
                    help="forward: the north-star encoder forward (default); train: the BASELINE config-3 "
                         "training step (encoder fwd+bwd + CTC head/loss + gradient all-reduce + AdamW); "
                         "joint: config 4 (Large-17 encoder B=16 T=1600 + RNN-T joint U=100 V=1024); "
                         "rnnt_train: the config-4 transducer training step (encoder + prediction net + joint "
                         "+ RNN-T loss, fwd+bwd, AdamW); "
                         "stream: config 5 (XL d1024/24 layers, B=64 streams, 400-frame buffers, 160-frame chunks); "
                         "cache_stream: the same 64 streams and 160-frame chunks through the cache-aware chunked "
                         "encoder (SURVEY f3, causal variant, 60 frames of attention history); "
                         "mel: the log-mel preprocessor in front of config 2 (SURVEY f1); "
                         "decode: config-4 transducer inference (encoder + greedy batch RNN-T decoding, SURVEY f2)")
    ap.add_argument("--vocab", type=int, default=256, help="train mode: CTC vocabulary (without blank)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # nothing has touched the GPU yet: the ranks are children, this process only waits for them
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    check_world(args.gpus, world)
    if args.dry_run:
        return dry_run(args, world, rank)
    dist = world > 1
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist:
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        tdist.init_process_group("nccl", device_id=dev)
        joined = ranks_joined(dev, dist)
        if joined != args.gpus:
            raise SystemExit(f"bench.py: {joined} ranks joined the RCCL group, --gpus {args.gpus}")

    def barrier():
        if dist:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)

    if args.mode == "train":
        return run_train(args, world, rank, dev, dist, barrier)
    if args.mode == "joint":
        return run_joint(args, world, rank, dev, dist, barrier)
    if args.mode == "rnnt_train":
        return run_rnnt_train(args, world, rank, dev, dist, barrier)
    if args.mode == "stream":
        return run_stream(args, world, rank, dev, dist, barrier)
    if args.mode == "cache_stream":
        return run_cache_stream(args, world, rank, dev, dist, barrier)
    if args.mode == "mel":
        return run_mel(args, world, rank, dev, dist, barrier)
    if args.mode == "decode":
        return run_decode(args, world, rank, dev, dist, barrier)
    from nemo.collections.asr.modules import ConformerEncoder
    torch.manual_seed(0)
    d, H, L, B, T = 512, 8, args.layers, args.batch, args.seq
    enc = ConformerEncoder(feat_in=80, n_layers=L, d_model=d, n_heads=H).to(dev).eval()
    enc.set_compute_mode(args.compute)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.randn(B, 80, T, device=dev, generator=g)          # synthetic 80-mel, resident in HBM
    lengths = torch.full((B,), T, dtype=torch.int64, device=dev)

    with torch.inference_mode():
        for _ in range(args.warmup):
            y, yl = enc(audio_signal=x, length=lengths)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            y, yl = enc(audio_signal=x, length=lengths)
        barrier()
        elapsed = time.perf_counter() - t0
    # CFM_GEMM_PROBE (kernel timing studies) drops work inside kernels on purpose: outputs are not meaningful
    assert os.environ.get("CFM_GEMM_PROBE") or torch.isfinite(y).all().item()
    t_max = max_over_ranks(elapsed, dev, dist)
    value = job_throughput(t_max, world, B, T, args.steps)
    ms_step = 1000.0 * t_max / args.steps
    es = 4 if args.compute == "fp32" else 2
    roof, breakdown = None, {}
    if rank == 0 and not args.no_breakdown:
        # per-kernel stage clock, right after the timed loop (same clock / thermal state as ms_per_step)
        roof, breakdown = stage_breakdown(args, enc, dev, x, lengths, B, T, d, L, H, es)
    # BASELINE config 3 (training step, DP over the same ranks, RCCL gradient buckets): every rank runs it
    train = None if args.no_train else train_leg(args, world, rank, dev, dist, barrier, args.train_steps,
                                                   args.train_warmup)

    if rank == 0:
        total_flop = None
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from conformer_oracle import encoder_flops
        total_flop = encoder_flops(B, T, d, L)
        # the CPU baseline is a rank-0, N=1 measurement (a multi-GPU job reports the GPU lines only)
        cpu = cpu_baseline(enc, B, T, args.cpu_budget) if (args.cpu_budget > 0 and world == 1) else None
        parity, fp32_line, fp16_line = (None, None, None)
        if not args.no_parity and L == 17 and d == 512:
            parity, fp32_line, fp16_line = parity_and_fp32(dev, B, T)
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "audio-frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.compute, "data": "synthetic",
            "config": {"workload": f"Conformer-CTC-Large encoder forward (d_model 512, 8 heads, {L} layers, eval), "
                                   f"B={B}/GPU, T={T} 80-mel frames, random-init weights",
                       "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world} (replicas, no collective)"},
            "roofline": roof,
            "model_flops": {"GFLOP_per_step_per_gpu": round(total_flop / 1e9, 1),
                            "TFLOP/s_per_gpu": round(total_flop / (ms_step * 1e-3) / 1e12, 1),
                            "frac_of_peak": round(total_flop / (ms_step * 1e-3) / 1e12 / PEAK[args.compute], 4)},
            "cpu_baseline": cpu,
            "ranks_joined": world,
            "train": train,
            "parity": parity,
            "fp32_parity_mode": fp32_line,
            "fp16_mode": fp16_line,
            "breakdown": breakdown,
        }
        if breakdown:
            # kernel durations only: the rest of ms_per_step is dispatch gaps between the kernels
            ovh = breakdown.pop("_clock_overhead_us", None)
            bsum = sum(v["ms_total"] for v in breakdown.values())
            out["breakdown_sum"] = {"ms": round(bsum, 4), "of_ms_per_step": round(bsum / ms_step, 4),
                                    "clock": os.environ.get("CFM_STAGE_CLOCK", "packet")}
            if ovh is not None:
                # minus the clock's own begin -> end of an empty kernel, once per launch
                nl = sum(v["launches"] for v in breakdown.values())
                net = bsum - nl * ovh * 1e-3
                out["breakdown_sum"].update({"clock_overhead_us_per_kernel": ovh, "launches": nl,
                                             "ms_net": round(net, 4), "net_of_ms_per_step": round(net / ms_step, 4)})
        print(json.dumps(out), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


TRAIN_METRIC = "training-step audio-frames/sec, Conformer-CTC-Large B=32/GPU T=1000 (BASELINE config 3)"


def train_leg(args, world, rank, dev, dist, barrier, steps, warmup):
    """BASELINE config 3: one step = encoder train-mode forward (dropout 0.1, batch-statistics BatchNorm,
    SyncBatchNorm across ranks) + ConvASRDecoder + CTCLoss(mean_batch) + backward with the per-layer
    gradient buckets all-reduced over RCCL while the backward runs (conformer_amd.dist.GradBuckets)
    + AdamW (conformer_ctc_bpe.yaml optim: betas 0.9/0.98, wd 1e-3).
    Synthetic targets U=60 uniform in [0, V).  Every rank runs it (the gradient exchange is
    collective); returns the max-over-ranks timing and, on rank 0, the FLOP accounting."""
    from conformer_amd import dist as cdist
    from nemo.collections.asr.losses import CTCLoss
    from nemo.collections.asr.modules import ConformerEncoder, ConvASRDecoder
    torch.manual_seed(0)
    d, H, L, B, T, V, U = 512, 8, args.layers, args.batch, args.seq, args.vocab, 60
    # conformer_ctc_bpe.yaml:130-132 regularisation, unchanged: dropout 0.1, dropout_emb 0.0, dropout_att 0.1
    enc = ConformerEncoder(feat_in=80, n_layers=L, d_model=d, n_heads=H, dropout=0.1, dropout_emb=0.0,
                           dropout_att=0.1).to(dev).train()
    dec = ConvASRDecoder(feat_in=d, num_classes=V).to(dev).train()
    for m in (enc, dec):
        m.set_compute_mode("bf16" if args.compute == "fp16" else args.compute)   # fp16 is inference-only
    if dist:
        cdist.convert_sync_batchnorm(enc)
    loss_fn = CTCLoss(num_classes=V, zero_infinity=True, reduction="mean_batch")
    params = [p for m in (enc, dec) for p in m.parameters()]
    try:
        opt = torch.optim.AdamW(params, lr=1e-4, betas=(0.9, 0.98), weight_decay=1e-3, fused=True)
    except (RuntimeError, TypeError):
        opt = torch.optim.AdamW(params, lr=1e-4, betas=(0.9, 0.98), weight_decay=1e-3, foreach=True)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.randn(B, 80, T, device=dev, generator=g)
    lengths = torch.full((B,), T, dtype=torch.int64, device=dev)
    targets = torch.randint(0, V, (B, U), device=dev, generator=g)
    tlen = torch.full((B,), U, dtype=torch.int64, device=dev)
    if dist:   # grads = views of one flat buffer, each layer all-reduced as soon as its backward is enqueued
        cdist.enable_gradient_buckets(torch.nn.ModuleList([enc, dec]))

    def step():
        opt.zero_grad(set_to_none=True)
        y, yl = enc(audio_signal=x, length=lengths)
        lp = dec(encoder_output=y)
        loss = loss_fn(log_probs=lp, targets=targets, input_lengths=yl, target_lengths=tlen)
        loss.backward()          # with dist: the bucket all-reduces finish inside the backward
        opt.step()
        return loss

    elapsed, loss = timed_loop(step, warmup, steps, barrier)
    finite = bool(torch.isfinite(loss).item())
    t_max = max_over_ranks(elapsed, dev, dist)
    ms_step = 1000.0 * t_max / steps
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from conformer_oracle import encoder_flops   # FLOP accounting only (after the timed loop)
    fwd = encoder_flops(B, T, d, L)
    res = {
        "ms_per_step": round(ms_step, 4), "value": round(job_throughput(t_max, world, B, T, steps), 1),
        "unit": "audio-frames/s", "steps": steps, "warmup": warmup,
        "TFLOP/s_per_gpu": round(3 * fwd / (ms_step * 1e-3) / 1e12, 1),
        "frac_of_peak": round(3 * fwd / (ms_step * 1e-3) / 1e12 / PEAK[args.compute], 4),
        "GFLOP_per_step_per_gpu_(3x_fwd)": round(3 * fwd / 1e9, 1),
        "loss": round(float(loss.detach()), 4), "loss_finite": finite, "params": sum(p.numel() for p in params),
        "workload": f"Conformer-CTC-Large training step (encoder d512/8 heads/{L} layers, dropout 0.1, dropout_att 0.1, "
                    f"BatchNorm train stats{' + SyncBN' if dist else ''}, CTC head V={V}+1, CTC loss U={U}, AdamW), "
                    f"B={B}/GPU, T={T}",
        "parallelism": f"dp{world}" + (f" (per-layer RCCL gradient buckets overlapped with the backward, "
                                       f"{L + 2} all-reduces per step)" if dist else ""),
    }
    del enc, dec, opt, params
    torch.cuda.empty_cache()
    if not finite:
        raise SystemExit("bench.py: training loss is not finite")
    return res


def run_train(args, world, rank, dev, dist, barrier):
    r = train_leg(args, world, rank, dev, dist, barrier, args.steps, args.warmup)
    emit(rank, dist, {
        "metric": TRAIN_METRIC, "value": r["value"], "unit": "audio-frames/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": r["ms_per_step"], "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.compute, "data": "synthetic",
        "config": {"workload": r["workload"], "global_batch": args.batch * world, "seq_len": args.seq,
                   "parallelism": r["parallelism"]},
        "model_flops": {"GFLOP_per_step_per_gpu_(3x_fwd)": r["GFLOP_per_step_per_gpu_(3x_fwd)"],
                        "TFLOP/s_per_gpu": r["TFLOP/s_per_gpu"], "frac_of_peak": r["frac_of_peak"]},
        "params": r["params"], "loss": r["loss"],
    })


def timed_loop(step, warmup, steps, barrier):
    for _ in range(warmup):
        r = step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        r = step()
    barrier()
    return time.perf_counter() - t0, r


def emit(rank, dist, out):
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


JOINT_METRIC = "encoder+joint audio-frames/sec, Conformer-Transducer-Large B=16 T=1600 U=100 V=1024 (BASELINE config 4)"


def run_joint(args, world, rank, dev, dist, barrier):
    """BASELINE config 4: Large-17 encoder forward (B=16, T=1600) + RNNTDecoder prediction network
    over U=100 random targets (+SOS) + RNNTJoint forward over the (B, T'=400, U+1=101) lattice with
    V=1024 (+blank), logits as on a GPU (rnnt.py:998-1002)."""
    from nemo.collections.asr.modules import ConformerEncoder, RNNTDecoder, RNNTJoint
    torch.manual_seed(0)
    d, H, L, B, T, U, V = 512, 8, args.layers, 16, 1600, 100, 1024
    enc = ConformerEncoder(feat_in=80, n_layers=L, d_model=d, n_heads=H).to(dev).eval()
    enc.set_compute_mode(args.compute)
    joint = RNNTJoint(jointnet=dict(encoder_hidden=d, pred_hidden=640, joint_hidden=640, activation="relu"),
                      num_classes=V).to(dev).eval()
    joint.set_compute_mode(args.compute)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.randn(B, 80, T, device=dev, generator=g)
    lengths = torch.full((B,), T, dtype=torch.int64, device=dev)
    dec = RNNTDecoder(prednet=dict(pred_hidden=640, pred_rnn_layers=1), vocab_size=V).to(dev).eval()
    targets = torch.randint(0, V, (B, U), device=dev, generator=g)
    tlen = torch.full((B,), U, dtype=torch.int64, device=dev)

    def step():
        y, yl = enc(audio_signal=x, length=lengths)
        pred, _, _ = dec(targets=targets, target_length=tlen)
        return joint(encoder_outputs=y, decoder_outputs=pred)

    with torch.inference_mode():
        elapsed, out = timed_loop(step, args.warmup, args.steps, barrier)
        assert torch.isfinite(out[:1]).all().item()
        # per-module device time (rank 0, after the timed loop): each module's call timed alone with
        # stream events over a few repetitions, on the outputs of the timed step's inputs
        parts = {}
        if rank == 0 and not args.no_breakdown:
            y, yl = enc(audio_signal=x, length=lengths)
            pred, _, _ = dec(targets=targets, target_length=tlen)
            calls = {"encoder": lambda: enc(audio_signal=x, length=lengths),
                     "prediction_net": lambda: dec(targets=targets, target_length=tlen),
                     "joint": lambda: joint(encoder_outputs=y, decoder_outputs=pred)}
            for name, fn in calls.items():
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                parts[name] = e0.elapsed_time(e1) / 5
    t_max = max_over_ranks(elapsed, dev, dist)
    ms_step = 1000.0 * t_max / args.steps
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from conformer_oracle import encoder_flops
    Tp = (((T - 1) // 2 + 1) - 1) // 2 + 1
    f_enc = encoder_flops(B, T, d, L)
    f_joint = 2 * B * Tp * d * 640 + 2 * B * (U + 1) * 640 * 640 + 2 * B * Tp * (U + 1) * 640 * (V + 1)
    f_pred = 2 * B * (U + 1) * (2 * 640) * (4 * 640)
    tot = f_enc + f_joint + f_pred
    breakdown = None
    roof = None
    if parts:
        logit_bytes = B * Tp * (U + 1) * (V + 1) * 4
        work = {"encoder": ("flop", f_enc), "prediction_net": ("flop", f_pred), "joint": ("flop", f_joint)}
        breakdown = {}
        for k, ms in parts.items():
            kind, amt = work[k]
            breakdown[k] = {"ms": round(ms, 4), "TFLOP/s": round(amt / (ms * 1e-3) / 1e12, 1)}
        breakdown["joint"]["logits_GB/s"] = round(logit_bytes / (parts["joint"] * 1e-3) / 1e9, 1)
        # the joint's bound: its GEMM FLOPs at the MFMA peak or its fp32 logits at the HBM peak
        t_mfma = f_joint / (PEAK[args.compute] * 1e12) * 1e3
        t_hbm = logit_bytes / (HBM_PEAK_GBS * 1e9) * 1e3
        fused = os.environ.get("CFM_JOINT_FUSED", "1") != "0" and args.compute == "bf16"
        roof = {"kernel": "joint (logits kernel, hidden formed in registers)" if fused else "joint (hidden + logits GEMM)", "bound": "hbm" if t_hbm >= t_mfma else "mfma",
                "floor_ms": round(max(t_mfma, t_hbm), 4), "achieved_ms": round(parts["joint"], 4),
                "frac": round(max(t_mfma, t_hbm) / parts["joint"], 4),
                "note": f"{f_joint / 1e9:.0f} GFLOP at {PEAK[args.compute]} TFLOP/s = {t_mfma:.3f} ms; "
                        f"{logit_bytes / 1e9:.2f} GB fp32 logits at {HBM_PEAK_GBS} GB/s = {t_hbm:.3f} ms"}
    emit(rank, dist, {
        "metric": JOINT_METRIC, "value": round(job_throughput(t_max, world, B, T, args.steps), 1),
        "unit": "audio-frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": args.compute, "data": "synthetic",
        "config": {"workload": f"Conformer-Transducer-Large encoder ({L} layers) + RNNTDecoder (LSTM 640, 1 layer, "
                               f"U={U} targets + SOS) + RNNTJoint (640 hidden, relu), "
                               f"B={B}/GPU, T={T}, U+1={U + 1}, V+1={V + 1}, logits fp32 "
                               f"({B * Tp * (U + 1) * (V + 1) * 4 / 1e9:.2f} GB per step)",
                   "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world} (replicas, no collective)"},
        "model_flops": {"GFLOP_per_step_per_gpu": round(tot / 1e9, 1), "encoder_GFLOP": round(f_enc / 1e9, 1),
                        "joint_GFLOP": round(f_joint / 1e9, 1), "prediction_net_GFLOP": round(f_pred / 1e9, 2),
                        "TFLOP/s_per_gpu": round(tot / (ms_step * 1e-3) / 1e12, 1),
                        "frac_of_peak": round(tot / (ms_step * 1e-3) / 1e12 / PEAK[args.compute], 4)},
        **({"breakdown": breakdown, "roofline": roof} if breakdown else {}),
    })


RNNT_TRAIN_METRIC = ("transducer training-step audio-frames/sec, Conformer-Transducer-Large B=16/GPU T=1600 U=100 "
                     "V=1024 (BASELINE config 4 workload, fwd+bwd)")


def run_rnnt_train(args, world, rank, dev, dist, barrier):
    """The config-4 workload as a training step (EncDecRNNTModel.training_step, rnnt_models.py:673-739, on
    the drop-in modules): Large-17 encoder in train mode (conformer_transducer_bpe.yaml regularisation:
    dropout 0.1, dropout_att 0.1) at B=16, T=1600; RNNTDecoder (LSTM 640, dropout 0.2) over U=100 targets;
    RNNTJoint (640, relu, dropout 0.2) to raw logits (B, 400, 101, 1025); native RNN-T loss (mean_batch);
    loss.backward() (loss gradient -> joint backward -> prediction-net BPTT -> encoder backward, per-layer
    gradient buckets over RCCL at N>1) and AdamW."""
    from conformer_amd import dist as cdist
    from nemo.collections.asr.losses import RNNTLoss
    from nemo.collections.asr.modules import ConformerEncoder, RNNTDecoder, RNNTJoint
    torch.manual_seed(0)
    d, H, L, B, T, U, V = 512, 8, args.layers, 16, 1600, 100, 1024
    enc = ConformerEncoder(feat_in=80, n_layers=L, d_model=d, n_heads=H, dropout=0.1, dropout_emb=0.0,
                           dropout_att=0.1).to(dev).train()
    enc.set_compute_mode(args.compute)
    dec = RNNTDecoder(prednet=dict(pred_hidden=640, pred_rnn_layers=1, dropout=0.2), vocab_size=V).to(dev).train()
    joint = RNNTJoint(jointnet=dict(encoder_hidden=d, pred_hidden=640, joint_hidden=640, activation="relu",
                                    dropout=0.2), num_classes=V, log_softmax=False).to(dev).train()
    joint.set_compute_mode(args.compute)
    if dist:
        cdist.convert_sync_batchnorm(enc)
    loss_fn = RNNTLoss(num_classes=V, reduction="mean_batch")
    params = [p for m in (enc, dec, joint) for p in m.parameters()]
    opt = torch.optim.AdamW(params, lr=1e-4, betas=(0.9, 0.98), weight_decay=1e-3, fused=True)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.randn(B, 80, T, device=dev, generator=g)
    lengths = torch.full((B,), T, dtype=torch.int64, device=dev)
    targets = torch.randint(0, V, (B, U), device=dev, generator=g)
    tlen = torch.full((B,), U, dtype=torch.int64, device=dev)
    if dist:
        cdist.enable_gradient_buckets(torch.nn.ModuleList([enc, dec, joint]))

    def step():
        opt.zero_grad(set_to_none=True)
        y, yl = enc(audio_signal=x, length=lengths)
        pred, _, _ = dec(targets=targets, target_length=tlen)
        logits = joint(encoder_outputs=y, decoder_outputs=pred)
        loss = loss_fn(log_probs=logits, targets=targets, input_lengths=yl, target_lengths=tlen)
        loss.backward()
        opt.step()
        return loss

    elapsed, loss = timed_loop(step, args.warmup, args.steps, barrier)
    finite = bool(torch.isfinite(loss).item())
    t_max = max_over_ranks(elapsed, dev, dist)
    ms_step = 1000.0 * t_max / args.steps
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from conformer_oracle import encoder_flops
    Tp = (((T - 1) // 2 + 1) - 1) // 2 + 1
    f_enc = encoder_flops(B, T, d, L)
    f_joint = 2 * B * Tp * d * 640 + 2 * B * (U + 1) * 640 * 640 + 2 * B * Tp * (U + 1) * 640 * (V + 1)
    f_pred = 2 * B * (U + 1) * (2 * 640) * (4 * 640)
    tot = 3 * (f_enc + f_joint + f_pred)
    emit(rank, dist, {
        "metric": RNNT_TRAIN_METRIC, "value": round(job_throughput(t_max, world, B, T, args.steps), 1),
        "unit": "audio-frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": args.compute, "data": "synthetic",
        "config": {"workload": f"Conformer-Transducer-Large training step: encoder ({L} layers, dropout 0.1, "
                               f"dropout_att 0.1) + RNNTDecoder (LSTM 640, dropout 0.2, U={U} + SOS) + RNNTJoint "
                               f"(640, relu, dropout 0.2, V+1={V + 1}, raw logits) + RNN-T loss + backward + AdamW, "
                               f"B={B}/GPU, T={T}",
                   "global_batch": B * world, "seq_len": T,
                   "parallelism": f"dp{world}" + (" (per-layer RCCL gradient buckets)" if dist else "")},
        "model_flops": {"GFLOP_per_step_per_gpu_(3x_fwd)": round(tot / 1e9, 1),
                        "TFLOP/s_per_gpu": round(tot / (ms_step * 1e-3) / 1e12, 1),
                        "frac_of_peak": round(tot / (ms_step * 1e-3) / 1e12 / PEAK[args.compute], 4)},
        "loss": round(float(loss.detach()), 4), "loss_finite": finite,
        "params": sum(p.numel() for p in params),
    })


DECODE_METRIC = "transducer greedy inference audio-frames/sec, Conformer-Transducer-Large B=16 T=1600 V=1024 (config 4 + SURVEY f2)"


def run_decode(args, world, rank, dev, dist, barrier):
    """Config-4 transducer inference: Large-17 encoder forward (B=16, T=1600) followed by greedy batch
    RNN-T decoding (GreedyBatchedRNNTInfer, max_symbols 30, conformer_transducer_bpe.yaml:172-177) with
    the LSTM prediction network (640, 1 layer) and the joint (640, relu, V=1024).  Random weights; the
    joint's blank logit is biased (+BLANK_BIAS) so the emission rate is speech-like (reported)."""
    from nemo.collections.asr.modules import ConformerEncoder, RNNTDecoder, RNNTJoint
    from nemo.collections.asr.parts.submodules.rnnt_greedy_decoding import GreedyBatchedRNNTInfer
    torch.manual_seed(0)
    d, H, L, B, T, V = 512, 8, args.layers, 16, 1600, 1024
    blank_bias = float(os.environ.get("BLANK_BIAS", "1.1"))
    enc = ConformerEncoder(feat_in=80, n_layers=L, d_model=d, n_heads=H).to(dev).eval()
    enc.set_compute_mode(args.compute)
    dec = RNNTDecoder(prednet=dict(pred_hidden=640, pred_rnn_layers=1), vocab_size=V).to(dev).eval()
    joint = RNNTJoint(jointnet=dict(encoder_hidden=d, pred_hidden=640, joint_hidden=640, activation="relu"),
                      num_classes=V).to(dev).eval()
    with torch.no_grad():
        joint.joint_net[-1].bias[V] += blank_bias
    greedy = GreedyBatchedRNNTInfer(dec, joint, blank_index=V, max_symbols_per_step=30)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.randn(B, 80, T, device=dev, generator=g)
    lengths = torch.full((B,), T, dtype=torch.int64, device=dev)
    dec_ms = []

    def step():
        y, yl = enc(audio_signal=x, length=lengths)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        hyps = greedy(encoder_output=y, encoded_lengths=yl)[0]
        dec_ms.append(1000.0 * (time.perf_counter() - t0))
        return hyps

    with torch.inference_mode():
        elapsed, hyps = timed_loop(step, args.warmup, args.steps, barrier)
    t_max = max_over_ranks(elapsed, dev, dist)
    ms_step = 1000.0 * t_max / args.steps
    Tp = (((T - 1) // 2 + 1) - 1) // 2 + 1
    ntok = sum(len(h.y_sequence) for h in hyps)
    emit(rank, dist, {
        "metric": DECODE_METRIC, "value": round(job_throughput(t_max, world, B, T, args.steps), 1),
        "unit": "audio-frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": f"{args.compute} encoder, fp32 decoder", "data": "synthetic",
        "config": {"workload": f"Conformer-Transducer-Large encoder ({L} layers, B={B}, T={T} -> T'={Tp}) + greedy "
                               f"batch RNN-T decoding (LSTM 640, joint 640 relu, V+1={V + 1}, max_symbols 30, "
                               f"blank logit bias +{blank_bias})",
                   "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world} (replicas, no collective)"},
        "decode": {"ms_per_step": round(sorted(dec_ms[-args.steps:])[len(dec_ms[-args.steps:]) // 2], 3),
                   "tokens_per_step": ntok, "tokens_per_frame": round(ntok / (B * Tp), 3),
                   "note": "median host wall time of the greedy decode (it synchronises: it polls a device done-flag)"},
    })


STREAM_METRIC = ("streaming audio-frames/sec, Conformer-XLarge buffered (400-frame buffer, 160-frame chunk), "
                 "B=64 streams (BASELINE config 5)")


def run_stream(args, world, rank, dev, dist, barrier):
    """BASELINE config 5: every step advances B=64 independent streams by one 1.6 s chunk (160 frames):
    device-resident shift + per-feature normalisation of the 4 s buffers (cfm_frame_buffer_step,
    BatchedFeatureFrameBufferer semantics, streaming_utils.py:686-818), then the stateless XL encoder
    (d1024, 8 heads, 24 layers) over the whole 400-frame buffer, as FrameBatchASR does.  `value`
    counts NEW audio frames (B x 160 per step): the stream's real-time throughput."""
    from types import SimpleNamespace
    from nemo.collections.asr.modules import ConformerEncoder
    from nemo.collections.asr.parts.utils.streaming_utils import BatchedFeatureFrameBufferer
    torch.manual_seed(0)
    d, H, L, B, Tbuf, n = 1024, 8, 24, 64, 400, 160
    enc = ConformerEncoder(feat_in=80, n_layers=L, d_model=d, n_heads=H).to(dev).eval()
    enc.set_compute_mode(args.compute)
    model = SimpleNamespace(_cfg=SimpleNamespace(sample_rate=16000, preprocessor=SimpleNamespace(
        window_stride=0.01, features=80)), device=dev)
    bb = BatchedFeatureFrameBufferer(model, frame_len=1.6, batch_size=B, total_buffer=4.0)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    chunks = torch.randn(8, B, 80, n, device=dev, generator=g) * 4.0 - 6.0   # synthetic log-mel chunks
    buf = torch.empty(B, 80, Tbuf, device=dev)
    lengths = torch.full((B,), Tbuf, dtype=torch.int64, device=dev)
    it = [0]

    def step():
        bb.step(chunks[it[0] % 8], out=buf)
        it[0] += 1
        return enc(audio_signal=buf, length=lengths)

    with torch.inference_mode():
        elapsed, (y, yl) = timed_loop(step, args.warmup, args.steps, barrier)
        assert torch.isfinite(y).all().item()
    t_max = max_over_ranks(elapsed, dev, dist)
    ms_step = 1000.0 * t_max / args.steps
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from conformer_oracle import encoder_flops
    fl = encoder_flops(B, Tbuf, d, L)
    emit(rank, dist, {
        "metric": STREAM_METRIC, "value": round(world * B * n * args.steps / t_max, 1), "unit": "audio-frames/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.compute, "data": "synthetic",
        "config": {"workload": f"Conformer-XLarge (d1024, 8 heads, {L} layers) buffered streaming: B={B} streams, "
                               f"{Tbuf}-frame buffer, {n}-frame chunk, device-resident buffer normalisation",
                   "global_batch": B * world, "seq_len": Tbuf, "parallelism": f"dp{world} (replicas, no collective)"},
        "buffer_frames_per_s": round(world * B * Tbuf * args.steps / t_max, 1),
        "model_flops": {"GFLOP_per_step_per_gpu": round(fl / 1e9, 1),
                        "TFLOP/s_per_gpu": round(fl / (ms_step * 1e-3) / 1e12, 1),
                        "frac_of_peak": round(fl / (ms_step * 1e-3) / 1e12 / PEAK[args.compute], 4)},
    })


CACHE_STREAM_METRIC = "cache-aware streaming audio-frames/sec, Conformer-XL B=64 streams, 160-frame chunks"


def run_cache_stream(args, world, rank, dev, dist, barrier):
    """the same 64 XL streams advancing by 160 new frames (1.6 s) per
    step, through the cache-aware chunked encoder (include/cfm_cache_stream.h): 40 new encoder frames
    per stream per step, 60 frames of attention history carried as per-layer key/value rings (the
    40 + 60 = 100 encoder frames the buffered path sees in its 400-frame buffer), conv / subsampling
    state carried too.  Causal variant of the encoder (parity unpinned, see the header); `value`
    counts NEW audio frames like --mode stream, so the two lines compare directly."""
    from nemo.collections.asr.modules import ConformerEncoder
    torch.manual_seed(0)
    d, H, L, B, n, left = 1024, 8, 24, 64, 160, 60
    enc = ConformerEncoder(feat_in=80, n_layers=L, d_model=d, n_heads=H).to(dev).eval()
    enc.set_compute_mode(args.compute)
    st = enc.cache_aware_streamer(batch_size=B, chunk_size=n // 4, left_context=left, device=dev)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    chunks = torch.randn(8, B, 80, n, device=dev, generator=g) * 4.0 - 6.0   # synthetic log-mel chunks
    it = [0]

    def step():
        y = st.step(chunks[it[0] % 8])
        it[0] += 1
        return y

    with torch.inference_mode():
        elapsed, (y, yl) = timed_loop(step, args.warmup, args.steps, barrier)
        assert torch.isfinite(y).all().item()
    t_max = max_over_ranks(elapsed, dev, dist)
    ms_step = 1000.0 * t_max / args.steps
    emit(rank, dist, {
        "metric": CACHE_STREAM_METRIC, "value": round(world * B * n * args.steps / t_max, 1),
        "unit": "audio-frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": args.compute, "data": "synthetic",
        "config": {"workload": f"Conformer-XLarge (d1024, 8 heads, {L} layers) cache-aware streaming: B={B} streams, "
                               f"{n}-frame chunks ({n // 4} encoder frames), left context {left}, causal variant",
                   "global_batch": B * world, "seq_len": n, "parallelism": f"dp{world} (replicas, no collective)"},
    })


MEL_METRIC = "preprocessor audio-frames/sec, AudioToMelSpectrogramPreprocessor (conformer_ctc_bpe.yaml) B=32 T=1000"


def run_mel(args, world, rank, dev, dist, barrier):
    """the conformer_ctc_bpe.yaml preprocessor (25 ms hann window, 10 ms hop, n_fft 512,
    80 mels, per_feature normalisation, pad_to 0) over B=32 utterances of 159,840 samples (16 kHz,
    1000 output frames each): raw samples in HBM -> normalised (B, 80, 1000) features, eval mode."""
    from nemo.collections.asr.modules import AudioToMelSpectrogramPreprocessor
    B, N = args.batch, 160 * (args.seq - 1)
    p = AudioToMelSpectrogramPreprocessor(sample_rate=16000, normalize="per_feature", window_size=0.025,
                                          window_stride=0.01, window="hann", features=80, n_fft=512, log=True,
                                          frame_splicing=1, dither=0.00001, pad_to=0, pad_value=0.0).to(dev).eval()
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    x = torch.randn(B, N, device=dev, generator=g) * 0.1
    L = torch.full((B,), N, dtype=torch.int64, device=dev)
    with torch.inference_mode():
        elapsed, (y, yl) = timed_loop(lambda: p(input_signal=x, length=L), args.warmup, args.steps, barrier)
        assert torch.isfinite(y).all().item()
    T = y.shape[-1]
    t_max = max_over_ranks(elapsed, dev, dist)
    ms_step = 1000.0 * t_max / args.steps
    algo = B * N * 4 + 2 * B * 80 * T * 4 * 2      # samples once; features written, re-read and re-written by the norm pass
    ach = algo / (ms_step * 1e-3) / 1e9
    emit(rank, dist, {
        "metric": MEL_METRIC, "value": round(world * B * T * args.steps / t_max, 1), "unit": "audio-frames/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
        "config": {"workload": f"AudioToMelSpectrogramPreprocessor 80-mel, n_fft 512, B={B}, {N} samples/utterance",
                   "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world} (replicas, no collective)"},
        "roofline": {"kernel": "mel_frames_kernel + mel_norm_rows_kernel (whole step)", "bound": "hbm",
                     "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                     "traffic": None, "per_launch": f"{algo / 1e6:.1f} MB algorithmic per step"},
    })


if __name__ == "__main__":
    main()
