#!/usr/bin/env python3
"""bench.py -- throughput of the bulk audio-effect hot path on MI355X.

One step = one 256-frame block (48 kHz) processed for every instance on every rank, inputs
already resident in HBM (a pool of distinct synthetic blocks, cycled, larger than the 256 MiB
Infinity Cache).  Default workload = BASELINE.json configs[1]: 65,536 stereo ChorusEffect
instances per GPU.  Multi-GPU: one process per GPU (torchrun); the job is `instances per GPU x
world` GLOBAL instances, each rank takes its contiguous shard (ol_dsp_amd.dist.shard) and derives
every instance's parameters and input stream from its global index (ol_dsp_amd.workload), so an
N-GPU run processes exactly the instances a one-GPU run of the same total would.  No data-path
collective (weak scaling); one RCCL all-reduce after each timed region gathers the counters.

Prints ONE JSON line (rank 0): metric/value/unit/... plus
  roofline     : algorithmic bytes of the dominant kernel / its HIP-event-timed duration vs 8 TB/s
                 (frac = read+write, frac_read = the read share: the north star's HBM-read roofline)
  cpu_baseline : the CPU oracle (port) or the compiled reference (reference) on all host cores
                 given to this process, at -O2 and -O0 (the reference's CMake default)
  cpu_c1       : BASELINE configs[0]: one chorus instance, one core, per-frame calls
  also         : the other BASELINE configs timed in the same run (dattorro = configs[2], the
                 north star's >= 64k chorus+reverb chains, configs[4]'s per-GPU shard, configs[3]'s
                 voices, the fxlib rack), each with its own roofline and cpu_baseline
"""
from __future__ import annotations

import argparse
import json
import os
import platform
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
    "chain_65536": ("chain", 65536, "north_star: >= 64k concurrent chorus+reverb instances on 1xMI355X "
                    "(fused chorus->pitch-shift->dattorro chains)"),
    "pitchshift": ("pitchshift", 65536, "pitch-shift stage alone"),
    "fxrack": ("fxrack", 65536, "SURVEY 8f row 1: fxlib FxRack<2> (delay -> reverb -> filter -> master), 65,536 instances"),
    "voice_poly": ("voice", 32768, "SURVEY 8a A17: configs[3] voices summed into Polyvoice buses of 8 voices "
                   "(olfx_mix) inside every step"),
    "voice_events": ("voice", 32768, "configs[3] voices with note events every block: NoteOn for 2.5 % and NoteOff "
                     "for 2.5 % of the voices (5 %), SynthVoice.h:245-256, applied at the block start"),
    "chain_cc": ("chain", 16384, "configs[4]'s per-GPU shard with a control change every block: one parameter of "
                 "1 % of the chains (163 scattered instances) set before each block, as a MIDI CC fanned out "
                 "to objects (olfx_set_param_list)"),
    "dattorro_rpd": ("dattorro", 65536, "configs[2] with a random per-instance pre-delay (SURVEY 8d: 'a variant "
                     "with random preDelay measures the gather path', verb.cpp:137-139)"),
    "chain_rpd": ("chain", 65536, "north_star chains (65,536) with a random per-instance reverb pre-delay"),
}
# parameter set of a workload (ol_dsp_amd.workload.RANGES key) where it is not the kind's own
PARAM_SET = {"dattorro_rpd": "dattorro_rpd", "chain_rpd": "chain_rpd"}
# the event-free workload a control leg is compared with (same kind and instances)
EVENT_FREE = {"voice_events": "voice", "chain_cc": "chain"}
DEFAULT_ALSO = "dattorro,chain_65536,chain,voice,voice_moog,fxrack,voice_events,chain_cc,dattorro_rpd,chain_rpd"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="chorus", choices=sorted(WORKLOADS))
    ap.add_argument("--instances", type=int, default=0, help="instances per GPU (0 = workload default)")
    ap.add_argument("--also", default=None,
                    help=f"comma list of extra workloads timed in the same run (default for chorus: {DEFAULT_ALSO}; "
                         "'' = none)")
    ap.add_argument("--block", type=int, default=256)
    ap.add_argument("--sample-rate", type=float, default=48000.0)
    ap.add_argument("--pool-bytes", type=float, default=1.0e9, help="bytes of distinct input blocks (> 256 MiB IC)")
    ap.add_argument("--cpu-seconds", type=float, default=4.0, help="wall budget of each -O2 CPU baseline (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this process may run on")
    ap.add_argument("--traffic-json", default="", help="PMC traffic summary (tools/pmc_traffic.py)")
    return ap.parse_args()


# ------------------------------------------------------------------------------------------------
# CPU baseline (rank 0, N=1): the oracle restatement or the compiled reference, bounded sample
# ------------------------------------------------------------------------------------------------
def host_facts() -> dict:
    """nproc (the cores this process is given: OMP_NUM_THREADS where set -- the GPU box's CPU share
    per GPU, which `nproc` reports too -- else the affinity mask), the machine's CPU count and model
    (lscpu)."""
    try:
        nproc = len(os.sched_getaffinity(0))
    except AttributeError:
        nproc = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        nproc = min(nproc, int(omp))
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": nproc, "host_cpus": os.cpu_count(), "cpu_model": model}


def _cpu_bank(kind: str, n: int, sr: float, o0: bool, ref: bool, pset: str = ""):
    import oracle as O
    from ol_dsp_amd.workload import instance_params, voice_notes
    p = instance_params(pset or kind, 0, n)
    if kind == "dattorro":
        bank = O.Dattorro(n, ref=ref, o0=o0)
        for i in range(n):
            for f in range(7):
                bank.set(i, f, float(p[f, i]))
        return lambda x, t: bank.process(x, t), bank
    if kind in ("chorus", "pitchshift"):
        bank = O.Chorus(n, sr, 0 if kind == "chorus" else 1, o0=o0)
        for i in range(n):
            for f in range(p.shape[0]):
                bank.set(i, f if kind == "chorus" else (0, 7)[f], float(p[f, i]))
        return lambda x, t: bank.process(x, t), bank
    if kind == "fxrack":
        bank = O.FxRack(n, sr, o0=o0)
        for i in range(n):
            for f in range(p.shape[0]):
                bank.set(i, f, float(p[f, i]))
        return lambda x, t: bank.process(x, t), bank
    if kind in VOICE_KINDS:
        bank = O.Voice(n, sr, moog=kind == "voice_moog", o0=o0)
        notes = voice_notes(0, n)
        for i in range(n):
            bank.config(i, p[:, i])
            bank.note(i, True, int(notes[i]))
        return lambda x, t: bank.process(x.shape[1], t), bank
    # chain: the composed stages, each a real bank with the chain's parameters
    c1, c2, d = O.Chorus(n, sr, 0, o0=o0), O.Chorus(n, sr, 1, o0=o0), O.Dattorro(n, ref=ref, o0=o0)
    for i in range(n):
        for f in range(8):
            c1.set(i, f, float(p[f, i]))
        c2.set(i, 0, float(p[8, i]))
        c2.set(i, 7, float(p[9, i]))
        for f in range(7):
            d.set(i, f, float(p[10 + f, i]))
    return lambda x, t: d.process(c2.process(c1.process(x, t), t), t), (c1, c2, d)


def cpu_baseline(kind: str, block: int, sr: float, budget_s: float, threads: int, pset: str = "") -> dict:
    """Time the CPU oracle (or, for the reverb, the reference verb.cpp compiled here) on a bounded
    sample of the same workload: the same global instances 0..n-1 with the same parameters and
    input streams, 256-frame blocks, OpenMP schedule(static) over instances, until the wall
    budget is spent; then the same at -O0 for a quarter of the budget."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from ol_dsp_amd.workload import noise_np
    n = 8192 if kind not in VOICE_KINDS else 32768
    ich = 0 if kind in VOICE_KINDS else 2
    x = noise_np(0, n, block, 2) if ich else np.zeros((1, block, n), np.float32)
    ref = kind in ("dattorro", "chain") and O.ref_available() and O.ref_available(o0=True)

    def timed(o0: bool, budget: float):
        step, _keep = _cpu_bank(kind, n, sr, o0, ref, pset)
        step(x, threads)  # warm
        t0 = time.perf_counter()
        blocks = 0
        while True:
            step(x, threads)
            blocks += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return blocks * block * n / el, blocks, el

    v2, b2, e2 = timed(False, budget_s)
    v0, b0, e0 = timed(True, max(0.5, budget_s / 4))
    src = ("oracle/_ref = libs/dattorro-verb/verb.cpp compiled here (reverb stage)" if ref
           else "oracle C restatement")
    res = {"value": v2, "unit": "stereo samples/s" if kind not in VOICE_KINDS else "voice samples/s",
           "cores": threads, "kind": "reference" if kind == "dattorro" and ref else "port",
           "sample": f"{n} instances x {b2} blocks x {block} frames ({e2:.1f} s wall, {threads} OpenMP threads, "
                     f"{src}, -O2 -ffp-contract=off)",
           "value_O0": v0, "sample_O0": f"{n} instances x {b0} blocks ({e0:.1f} s), -O0 (reference CMake default)"}
    res.update(host_facts())
    return res


def cpu_c1(sr: float, block: int) -> dict:
    """BASELINE configs[0]: one ChorusEffect instance, one core, 60 s of audio in
    256-frame blocks, one process() call per frame as in the reference's fx_test.cpp:45-54 loop."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from ol_dsp_amd.workload import instance_params
    p = instance_params("chorus", 0, 1)[:, 0]
    frames = int(60 * sr)
    out = {}
    for o0 in (False, True):
        t0 = time.perf_counter()
        nans, _ = O.chorus_c1(p, frames, block, sr, o0=o0)
        el = time.perf_counter() - t0
        out["value_O0" if o0 else "value"] = frames / el
        out["nan_outputs_O0" if o0 else "nan_outputs"] = nans
    out.update({"unit": "stereo samples/s", "cores": 1, "kind": "port",
                "sample": f"1 instance, {frames} frames (60 s @ {sr:.0f} Hz), {block}-frame blocks, per-frame "
                          "process() calls (fx_test.cpp:45-54 loop shape), oracle C restatement -O2 / -O0"})
    return out


# ------------------------------------------------------------------------------------------------
# GPU workloads
# ------------------------------------------------------------------------------------------------
def _traffic(name: str, n: int, B: int, override: str = ""):
    for tj in ([override] if override else []) + [os.path.join(ROOT, "profiles", f"traffic_{name}_{n}.json"),
                                                  os.path.join(ROOT, "profiles", f"traffic_{name}.json")]:
        if tj and os.path.exists(tj):
            try:
                with open(tj) as f:
                    tr = json.load(f)
                if tr.get("instances") == n and tr.get("block") == B:
                    return tr
            except Exception:
                pass
    return None


def run_workload(name: str, n_per_gpu: int, args, rank: int, world: int, dev, with_cpu: bool) -> dict:
    import torch

    import ol_dsp_amd as ofx
    from ol_dsp_amd.dist import RunStats, reduce_stats, shard
    from ol_dsp_amd.workload import instance_params, noise_torch, voice_notes

    kind, _, desc = WORKLOADS[name]
    total = n_per_gpu * world
    first, n = shard(total, world, rank)
    B = args.block
    eng = ofx.Engine(kind, n, sample_rate=args.sample_rate, block=B, device=dev.index or 0)
    pset = PARAM_SET.get(name, kind)
    eng.set_params(0, instance_params(pset, first, n))
    ich, och = eng.info.in_channels, eng.info.out_channels

    # input pool: distinct synthetic blocks of each global instance's own stream, on the device
    blk_bytes = max(ich, 1) * B * n * 4
    pool_n = max(2, int(args.pool_bytes // blk_bytes)) if ich else 1
    pool = noise_torch(first, n, B, ich, dev, blocks=pool_n) if ich else [None]
    out = torch.empty((och, B, n), device=dev)
    voice = kind in VOICE_KINDS
    notes = voice_notes(first, n)
    note_off = None
    if voice:   # NoteOn for every voice at block 0, NoteOff at the middle of the timed blocks
        eng.note_events(eng.make_events(np.arange(n), 1, notes))
        note_off = eng.make_events(np.arange(n), 0, notes)
    # control legs: the per-step calls are prebuilt (untimed), so a step is the library call only
    step_events = None
    if name == "voice_events":     # voices i % 40 == k % 40 get NoteOn, i % 40 == (k + 20) % 40 NoteOff
        gi = np.arange(first, first + n)
        step_events = []
        for k in range(40):
            on = np.nonzero(gi % 40 == k)[0]
            off = np.nonzero(gi % 40 == (k + 20) % 40)[0]
            ev_on = eng.make_events(on, 1, (notes[on] + 12 * (k & 1)) % 128)
            ev_off = eng.make_events(off, 0, notes[off])
            step_events.append(np.concatenate([ev_on, ev_off]))
    step_ccs = None
    if name == "chain_cc":         # chains i % 100 == k % 100 get a new value of one field per step
        from ol_dsp_amd.workload import uniform01
        gi = np.arange(first, first + n)
        fields = [("chorus_depth", .08, 1.0), ("chorus_mix", 0.0, 1.0), ("verb_decay", .25, .95),
                  ("verb_damping", .05, .95), ("pitch_shift", 0.0, 3.0)]
        step_ccs = []
        for k in range(100):
            sel = np.nonzero(gi % 100 == k)[0].astype(np.uint32)
            fname, lo, hi = fields[k % len(fields)]
            vals = (lo + (hi - lo) * uniform01(7, k, int(first), n)[sel]).astype(np.float32)
            step_ccs.append((eng.field(fname), sel, vals))
    bus = None
    if name == "voice_poly":       # Polyvoice buses of 8 voices (Polyvoice.h:28-33)
        eng.mix_config([list(range(g, min(g + 8, n))) for g in range(0, n, 8)])
        bus = torch.zeros((B, eng.n_buses), device=dev)
    stream = torch.cuda.Stream(dev)        # dedicated non-default stream: events see the kernels
    torch.cuda.synchronize(dev)
    K, W = args.steps, args.warmup
    # Kernel timing: ONE event pair on the launch stream around the K timed steps: GPU time per
    # step = the kernel's average launch duration plus the gap between launches.  (A pair per step
    # adds two timestamp markers between consecutive kernels -- ~3-4 us each on the command
    # processor, 10-20 % of a 35 us voice block, measured: tools/loop_probe.py.)  Only voice_poly,
    # whose steps run two kernels, times each kernel with its own pair.
    per_step = bus is not None
    region = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)] if per_step else None
    evm = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)] if per_step else None

    # The timed loop calls the C-ABI directly with prebuilt arguments (Engine.process's checks and
    # tensor handling cost ~20 us of Python per call, more than a voice block's kernel): the host
    # must stay ahead of the GPU, or the event pairs below would time the host's launch latency.
    import ctypes

    from ol_dsp_amd import _lib
    lib, h = eng.lib, eng.handle
    c_stream = ctypes.c_void_p(stream.cuda_stream)
    c_out = ctypes.c_void_p(out.data_ptr())
    proc_args = [(h, ctypes.c_void_p(p.data_ptr() if p is not None else 0), c_out, B, _lib.IO_DEVICE, c_stream)
                 for p in pool]
    ev_args = [(h, e_.ctypes.data_as(ctypes.POINTER(_lib.Event)), len(e_)) for e_ in step_events or []]
    cc_args = [(h, f, sel.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                vals.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(sel)) for f, sel, vals in step_ccs or []]

    def step(k, t=None):
        rc = 0
        if voice and k == W + K // 2:
            eng.note_events(note_off)
        if ev_args:
            rc |= lib.olfx_note_events(*ev_args[k % 40])
        if cc_args:
            rc |= lib.olfx_set_param_list(*cc_args[k % 100])
        if t is not None and per_step:
            ev[t][0].record(stream)
        rc |= lib.olfx_process(*proc_args[k % pool_n])
        if t is not None and per_step:
            ev[t][1].record(stream)
        if rc:
            _lib.check(rc, h)
        if bus is not None:
            if t is not None:
                evm[t][0].record(stream)
            eng.mix(out, bus, stream=stream.cuda_stream)
            if t is not None:
                evm[t][1].record(stream)

    for k in range(W):
        step(k)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    region[0].record(stream)
    for k in range(K):
        step(W + k, k)
    region[1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev])) if per_step else region[0].elapsed_time(region[1]) / K
    mix_ms = float(np.mean([a.elapsed_time(b) for a, b in evm])) if evm else None

    # sum |y| over the finite outputs of the last block (a voice whose Svf diverges -- possible in
    # the reference DaisySP arithmetic at high cutoff, low resonance and high drive -- yields
    # inf/NaN there too); the count of non-finite samples beside it
    finite = torch.isfinite(out)
    nonfinite = int((~finite).sum().item())
    checksum = float(torch.where(finite, out.abs(), torch.zeros_like(out)).sum().item())
    bus_sum = float(bus.abs().sum().item()) if bus is not None else None
    stats = reduce_stats(RunStats(elapsed, kern_ms, float(n) * B * K, checksum), device=dev)
    bpf, rbpf, kname = eng.algorithmic_bytes_per_frame, eng.algorithmic_read_bytes_per_frame, eng.kernel_name
    eng.close()
    del pool, out
    torch.cuda.empty_cache()
    if rank != 0:
        return {}

    elapsed, kern_ms, frames = stats.elapsed_s, stats.kernel_ms, stats.frames
    per_launch = n * B
    achieved = bpf * per_launch / (kern_ms * 1e-3) / 1e9
    achieved_r = rbpf * per_launch / (kern_ms * 1e-3) / 1e9
    tr = _traffic(name, n, B, args.traffic_json if name == args.workload else "")
    traffic = tr.get("hbm_bytes_per_launch") if tr else None
    # the PMC-measured HBM bytes of the same kernel (profiles/traffic_<workload>.json, separate
    # --pmc passes) over this run's kernel time: what HBM actually moved, against the peak
    measured = {}
    if tr and traffic:
        measured["hbm_gbs_measured"] = traffic / (kern_ms * 1e-3) / 1e9
        rd = tr.get("read_bytes_by_request_size")
        if rd:
            measured.update({"traffic_read": rd, "hbm_read_gbs_measured": rd / (kern_ms * 1e-3) / 1e9,
                             "frac_read_measured": rd / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS})
    timing = ("HIP event pair per step around olfx_process" if per_step else
              "one HIP event pair on the launch stream around the K timed steps / K (launch duration + launch gap)")
    if voice:
        fps = VOICE_MOOG_FLOPS_PER_SAMPLE if kind == "voice_moog" else VOICE_FLOPS_PER_SAMPLE
        tflops = fps * per_launch / (kern_ms * 1e-3) / 1e12
        roofline = {"bound": "valu", "achieved": tflops, "peak": FP32_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": tflops / FP32_VALU_PEAK_TFLOPS, "traffic": traffic,
                    "kernel": kname, "kernel_ms": kern_ms, "kernel_timing": timing, "algorithmic_flops_per_frame": fps,
                    "algorithmic_bytes_per_frame": bpf, "hbm_gbs": achieved, "frames_per_launch": per_launch}
    else:
        roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                    "achieved_read": achieved_r, "frac_read": achieved_r / HBM_PEAK_GBS,
                    "kernel": kname, "kernel_ms": kern_ms, "kernel_timing": timing,
                    "algorithmic_bytes_per_frame": bpf, "algorithmic_read_bytes_per_frame": rbpf,
                    "frames_per_launch": per_launch, **measured}
    res = {"metric": METRIC, "value": frames / elapsed,
           "unit": "voice samples/s" if voice else "stereo samples/s",
           "ms_per_step": elapsed / K * 1e3,
           "config": {"workload": name, "restates": desc, "instances_per_gpu": n_per_gpu,
                      "instances_total": total, "block": B, "sample_rate": args.sample_rate,
                      "input_pool_blocks": pool_n, "parallelism": f"instance-shard x{world} (no data-path collective)"},
           "roofline": roofline,
           "output_checksum": stats.checksum, "output_nonfinite_rank0": nonfinite}
    if mix_ms is not None:
        nb = (n + 7) // 8
        mix_bytes = 4.0 * n * B + 8.0 * nb * B          # voice reads + bus read-modify-write
        res["mix"] = {"kernel": "voice_mix_v2", "kernel_ms": mix_ms, "bound": "hbm",
                      "achieved": mix_bytes / (mix_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                      "frac": mix_bytes / (mix_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                      "algorithmic_bytes_per_launch": mix_bytes, "bus_checksum_rank0": bus_sum}
    if step_events is not None:
        res["control"] = {"events_per_block": int(np.mean([len(e) for e in step_events])),
                          "note": "NoteOn/NoteOff folded per voice on the host and applied by the voice kernel at "
                                  "the block start (olfx_engine.cpp fold_events, voice.hip voice_event)"}
    if step_ccs is not None:
        res["control"] = {"instances_changed_per_block": int(np.mean([len(c[1]) for c in step_ccs])),
                          "note": "changed coefficients re-derived on the host for those instances only and "
                                  "scattered on the device ahead of the block (control.hip coef_scatter)"}
    # the CPU baseline runs after every GPU leg (main): no leg is timed right after a many-thread
    # CPU run (a short-kernel leg measured 1.7x slow once, launch-bound behind it)
    res["cpu_baseline"] = None
    if with_cpu and world == 1 and args.cpu_seconds > 0:
        res["cpu_job"] = (kind, PARAM_SET.get(name, ""))
    return res


def run_cpu_jobs(jobs, reuse, args):
    """The deferred CPU baselines: jobs = [(result dict, kind, param set)], reuse = [(result dict,
    the dict whose baseline it reuses, its key)]."""
    threads = args.cpu_threads or host_facts()["nproc"]
    for target, kind, pset in jobs:
        target["cpu_baseline"] = cpu_baseline(kind, args.block, args.sample_rate, args.cpu_seconds, threads, pset)
    for target, src, key in reuse:
        if src.get("cpu_baseline"):
            target["cpu_baseline"] = dict(src["cpu_baseline"], reused_from=key)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from ol_dsp_amd.dist import env_ranks
    rank, world, local = env_ranks()
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    n = args.instances or WORKLOADS[args.workload][1]
    cpu_jobs, cpu_reuse = [], []
    main_res = run_workload(args.workload, n, args, rank, world, dev, with_cpu=True)
    if rank == 0 and "cpu_job" in main_res:
        cpu_jobs.append((main_res, *main_res.pop("cpu_job")))
    also = args.also if args.also is not None else (DEFAULT_ALSO if args.workload == "chorus" else "")
    also_res = {}
    for name in [a for a in also.split(",") if a]:
        twin = EVENT_FREE.get(name)
        tkey = twin if twin != "chain" else "chain_16384"
        # a control leg's CPU work per block is its twin's (the CPU oracle applies events and
        # parameters per instance at block boundaries): the twin's measured baseline is reused
        reuse = bool(twin and tkey in also_res)
        r = run_workload(name, WORKLOADS[name][1], args, rank, world, dev, with_cpu=not reuse)
        if rank == 0:
            key = name if name != "chain" else "chain_16384"
            also_res[key] = {k: r[k] for k in ("value", "unit", "ms_per_step", "config", "roofline", "control",
                                                "cpu_baseline", "output_checksum", "output_nonfinite_rank0") if k in r}
            if "cpu_job" in r:
                cpu_jobs.append((also_res[key], *r["cpu_job"]))
            elif reuse:
                cpu_reuse.append((also_res[key], also_res[tkey], tkey))
            base = EVENT_FREE.get(name)
            bkey = base if base != "chain" else "chain_16384"
            # the control leg's cost against its event-free twin (an `also` leg or the main workload)
            b = also_res.get(bkey) or (main_res if base == args.workload else None)
            if base and b is not None:
                also_res[key]["control"].update({
                    "event_free_kernel_ms": b["roofline"]["kernel_ms"], "event_free_ms_per_step": b["ms_per_step"],
                    "kernel_ms_ratio": r["roofline"]["kernel_ms"] / b["roofline"]["kernel_ms"],
                    "ms_per_step_ratio": r["ms_per_step"] / b["ms_per_step"]})

    if rank == 0:
        run_cpu_jobs(cpu_jobs, cpu_reuse, args)
        res = {
            "metric": METRIC,
            "value": main_res["value"],
            "unit": main_res["unit"],
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": main_res["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: per-(instance, channel) xorshift32 noise streams (SURVEY 8d seeds) in a device "
                    "pool; per-instance params hashed from the global instance index",
            "config": main_res["config"],
            "roofline": main_res["roofline"],
            "cpu_baseline": main_res["cpu_baseline"],
            "output_checksum": main_res["output_checksum"],
            "output_nonfinite_rank0": main_res["output_nonfinite_rank0"],
        }
        if "mix" in main_res:
            res["mix"] = main_res["mix"]
        if world == 1 and args.cpu_seconds > 0 and args.workload == "chorus":
            res["cpu_c1"] = cpu_c1(args.sample_rate, args.block)
        if also_res:
            res["also"] = also_res
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
