#!/usr/bin/env python3
"""bench.py -- throughput of the bulk audio-effect hot path on MI355X.

One step = one 256-frame block (48 kHz) processed for every instance on every rank, inputs
already resident in HBM (a pool of distinct synthetic blocks, cycled, larger than the 256 MiB
Infinity Cache).  Default workload = BASELINE.json configs[1]: 65,536 stereo ChorusEffect
instances per GPU.  Multi-GPU: one process per GPU (torchrun), instances sharded with no
data-path collective (weak scaling); one RCCL all-reduce after the timed region gathers the
counters.

Prints ONE JSON line (rank 0): metric/value/unit/... plus
  roofline     : algorithmic bytes of the dominant kernel / its HIP-event-timed duration vs 8 TB/s
  cpu_baseline : the CPU oracle (port) or the compiled reference (reference) on host cores
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "stereo samples/s across N effect instances @48kHz; % HBM roofline; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
FP32_VALU_PEAK_TFLOPS = 157.3  # MI355X FP32 vector peak (MI355X_MICROARCH.md)
# The voice is VALU-bound (~5 B of HBM per sample): its roofline is FP32 operations, counted
# from the reference arithmetic per sample: 2 ADSR steps 6, amp 1, Port 3,
# SetFreq 1, polyBLEP saw 11, 0.5 gain 1, filter-env cutoff 3, Svf::SetFreq 8 + sin, two Svf
# passes 22, Low() average 3, output 1, sin and the three divisions 4 -> 64.
VOICE_FLOPS_PER_SAMPLE = 64.0
# MoogFilter voice: the same voice minus the Svf (27) plus daisysp::LadderFilter: SetAlpha/Qadjust
# 20, input drive 1, and per 4x-oversampled step: feedback sum 9, Pade tanh 6, four stages 24,
# accumulate 3 (x4 = 168) -> 216.
VOICE_MOOG_FLOPS_PER_SAMPLE = 216.0
VOICE_KINDS = ("voice", "voice_moog")
WORKLOADS = {
    # name: (kind, default instances per GPU, BASELINE config it restates)
    "chorus": ("chorus", 65536, "configs[1]: 65,536 ChorusEffect instances, 48 kHz, 256-sample blocks, 1xMI355X"),
    "dattorro": ("dattorro", 65536, "configs[2]: 65,536 dattorro-verb instances (full network), 48 kHz"),
    "voice": ("voice", 32768, "configs[3]: 262,144 synthlib voices = 32,768 per GPU x 8"),
    "voice_moog": ("voice_moog", 32768, "SURVEY 8f row 3: configs[3] with the Daisy firmware's MoogFilter "
                   "(daisysp::LadderFilter) voices, 32,768 per GPU"),
    "chain": ("chain", 16384, "configs[4]: 131,072 chorus->pitch-shift->dattorro chains = 16,384 per GPU x 8"),
    "pitchshift": ("pitchshift", 65536, "pitch-shift stage alone"),
    "fxrack": ("fxrack", 65536, "SURVEY 8f row 1: fxlib FxRack<2> (delay -> reverb -> filter -> master), 65,536 instances"),
    "voice_poly": ("voice", 32768, "SURVEY 8a A17: configs[3] voices summed into Polyvoice buses of 8 voices "
                   "(olfx_mix) inside every step"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="chorus", choices=sorted(WORKLOADS))
    ap.add_argument("--instances", type=int, default=0, help="instances per GPU (0 = workload default)")
    ap.add_argument("--block", type=int, default=256)
    ap.add_argument("--sample-rate", type=float, default=48000.0)
    ap.add_argument("--pool-bytes", type=float, default=1.2e9, help="bytes of distinct input blocks")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="wall budget of the CPU baseline (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cpu_count)")
    ap.add_argument("--traffic-json", default="", help="PMC traffic summary (tools/pmc_traffic.py)")
    return ap.parse_args()


def draw_params(kind: str, n: int, seed: int) -> np.ndarray:
    """Per-instance params, seeded uniform within the reference ranges."""
    rng = np.random.default_rng(seed)
    u = lambda lo, hi: rng.uniform(lo, hi, n).astype(np.float32)  # noqa: E731
    chorus = [u(0, 3), u(0, 1), u(0, .95), u(0, 1), u(0, 1), u(.08, 1), u(.01, 1), np.full(n, 10, np.float32)]
    pitch = [u(0, 3), np.full(n, 10, np.float32)]
    verb = [np.full(n, 0.1, np.float32), u(.5, .95), np.full(n, .75, np.float32), np.full(n, .625, np.float32),
            np.full(n, .70, np.float32), u(.25, .95), u(.05, .95)]
    voice = [u(100, 8000), u(0, .9), u(0, 1), u(0, 1), u(.001, .5), u(0, 1), u(.001, .5), u(0, 1), u(.001, .5),
             u(.2, 1), u(.001, .5), u(0, 1), u(.001, .5), u(0, 1), u(.001, .5), u(0, .05)]
    rack = [u(0.05, 1), u(0, .9), u(0, 1), u(100, 12000), u(0, .8), u(0, 1), u(100, 12000), u(0, .8),
            u(0, 1), rng.integers(0, 5, n).astype(np.float32), u(0, 1)]
    table = {"chorus": chorus, "pitchshift": pitch, "dattorro": verb, "voice": voice, "voice_moog": voice,
             "chain": chorus + pitch + verb, "fxrack": rack}
    return np.stack(table[kind])


def cpu_baseline(kind: str, block: int, sr: float, budget_s: float, threads: int) -> dict:
    """Time the CPU oracle (or the compiled reference for dattorro) on a bounded sample of the
    same workload: a bank of instances, 256-frame blocks, until the wall budget is spent."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    n = 8192 if kind not in VOICE_KINDS else 32768
    rng = np.random.default_rng(7)
    p = draw_params(kind, n, 7)
    x = (rng.random((2, block, n), dtype=np.float32) - 0.5)
    kind_used = "port"
    if kind == "dattorro":
        ref = O.ref_available()
        bank = O.Dattorro(n, ref=ref)
        kind_used = "reference" if ref else "port"
        for i in range(n):
            for f in range(7):
                bank.set(i, f, float(p[f, i]))
        step = lambda: bank.process(x, threads)  # noqa: E731
    elif kind in ("chorus", "pitchshift"):
        bank = O.Chorus(n, sr, 0 if kind == "chorus" else 1)
        for i in range(n):
            for f in range(p.shape[0]):
                bank.set(i, f if kind == "chorus" else (0, 7)[f], float(p[f, i]))
        step = lambda: bank.process(x, threads)  # noqa: E731
    elif kind == "fxrack":
        bank = O.FxRack(n, sr)
        for i in range(n):
            for f in range(p.shape[0]):
                bank.set(i, f, float(p[f, i]))
        step = lambda: bank.process(x, threads)  # noqa: E731
    elif kind in VOICE_KINDS:
        bank = O.Voice(n, sr, moog=kind == "voice_moog")
        for i in range(n):
            bank.config(i, p[:, i])
            bank.note(i, True, 36 + i % 60)
        step = lambda: bank.process(block, threads)  # noqa: E731
    else:  # chain: compose the three stages
        c1, c2, d = O.Chorus(n, sr), O.Chorus(n, sr, 1), O.Dattorro(n, ref=O.ref_available())
        step = lambda: d.process(c2.process(c1.process(x, threads), threads), threads)  # noqa: E731
    step()  # warm
    t0 = time.perf_counter()
    blocks = 0
    while True:
        step()
        blocks += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    frames = blocks * block * n
    return {"value": frames / el, "unit": "stereo samples/s" if kind not in VOICE_KINDS else "voice samples/s",
            "cores": threads, "kind": kind_used,
            "sample": f"{n} instances x {blocks} blocks x {block} frames ({el:.1f} s wall, {threads} OpenMP threads"
                      f"{', oracle/_ref = libs/dattorro-verb/verb.cpp -O2' if kind_used == 'reference' else ', oracle C restatement -O2'})"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from ol_dsp_amd.dist import RunStats, env_ranks, reduce_stats
    rank, world, local = env_ranks()
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import ol_dsp_amd as ofx
    kind, n_default, desc = WORKLOADS[args.workload]
    n = args.instances or n_default
    B = args.block
    eng = ofx.Engine(kind, n, sample_rate=args.sample_rate, block=B, device=local)
    eng.set_params(0, draw_params(kind, n, 1000 + rank))
    ich, och = eng.info.in_channels, eng.info.out_channels

    # input pool: distinct synthetic blocks (uniform +-0.5 white noise), generated on the device
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    blk_bytes = max(ich, 1) * B * n * 4
    pool_n = max(2, int(args.pool_bytes // blk_bytes)) if ich else 1
    pool = [torch.rand((ich, B, n), generator=gen, device=dev) - 0.5 for _ in range(pool_n)] if ich else [None]
    out = torch.empty((och, B, n), device=dev)
    if kind in VOICE_KINDS:   # NoteOn for every voice at block 0
        eng.note_events([(i, 1, 36 + (i * 7) % 61) for i in range(n)])
    bus = None
    if args.workload == "voice_poly":       # Polyvoice buses of 8 voices (Polyvoice.h:28-33)
        eng.mix_config([list(range(g, min(g + 8, n))) for g in range(0, n, 8)])
        bus = torch.zeros((B, eng.n_buses), device=dev)
    stream = torch.cuda.Stream(dev)        # dedicated non-default stream: events see the kernels
    torch.cuda.synchronize(dev)

    def step(k):
        eng.process(pool[k % pool_n], out=out, n_frames=B, stream=stream.cuda_stream)
        if bus is not None:
            eng.mix(out, bus, stream=stream.cuda_stream)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step(args.warmup + k)
        ev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    # the single collective of the run (RCCL over xGMI when world > 1): outside the timed region
    # sum |y| over the finite outputs (a voice whose Svf diverges -- possible in the reference
    # DaisySP arithmetic at high cutoff, low resonance and high drive -- yields inf/NaN there too;
    # DESIGN.md section 5); the count of non-finite samples is reported beside it
    finite = torch.isfinite(out)
    nonfinite = int((~finite).sum().item())
    checksum = float(torch.where(finite, out.abs(), torch.zeros_like(out)).sum().item())
    stats = reduce_stats(RunStats(elapsed, kern_ms, float(n) * B * args.steps, checksum), device=dev)
    elapsed, kern_ms, frames = stats.elapsed_s, stats.kernel_ms, stats.frames

    if rank == 0:
        value = frames / elapsed
        bpf = eng.algorithmic_bytes_per_frame
        per_launch_bytes = bpf * n * B
        achieved = per_launch_bytes / (kern_ms * 1e-3) / 1e9
        traffic = None
        tj = args.traffic_json or os.path.join(ROOT, "profiles", f"traffic_{args.workload}.json")
        if os.path.exists(tj):
            try:
                with open(tj) as f:
                    tr = json.load(f)
                if tr.get("instances") == n and tr.get("block") == B:
                    traffic = tr.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        if kind in VOICE_KINDS:
            fps = VOICE_MOOG_FLOPS_PER_SAMPLE if kind == "voice_moog" else VOICE_FLOPS_PER_SAMPLE
            tflops = fps * n * B / (kern_ms * 1e-3) / 1e12
            roofline = {"bound": "valu", "achieved": tflops, "peak": FP32_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": tflops / FP32_VALU_PEAK_TFLOPS, "traffic": traffic,
                        "kernel": eng.kernel_name, "kernel_ms": kern_ms,
                        "algorithmic_flops_per_frame": fps,
                        "algorithmic_bytes_per_frame": bpf, "hbm_gbs": achieved, "frames_per_launch": n * B}
        else:
            roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                        "kernel": eng.kernel_name, "kernel_ms": kern_ms,
                        "algorithmic_bytes_per_frame": bpf, "frames_per_launch": n * B}
        cpu = None
        if world == 1 and args.cpu_seconds > 0:
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            cpu = cpu_baseline(kind, B, args.sample_rate, args.cpu_seconds, threads)
        res = {
            "metric": METRIC,
            "value": value,
            "unit": "voice samples/s" if kind in VOICE_KINDS else "stereo samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (device-generated uniform +-0.5 noise pool, seeded per-instance params)",
            "config": {"workload": args.workload, "restates": desc, "instances_per_gpu": n,
                       "instances_total": n * world, "block": B, "sample_rate": args.sample_rate,
                       "input_pool_blocks": pool_n, "parallelism": f"instance-shard x{world} (no data-path collective)"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "output_checksum": stats.checksum,
            "output_nonfinite_rank0": nonfinite,
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
