#!/usr/bin/env python3
"""bench.py -- throughput of the bulk audio-effect hot path on MI355X.

One step = one 256-frame block (48 kHz) processed for every instance on every rank, inputs
already resident in HBM (a pool of distinct synthetic blocks, cycled, larger than the 256 MiB
Infinity Cache).  Default workload = BASELINE.json configs[1]: 65,536 stereo ChorusEffect
instances per GPU.

Multi-GPU: one process per GPU.  Under torchrun the ranks come from the environment; without a
launcher, `--gpus N` (N > 1) starts the N rank processes itself (ol_dsp_amd.dist.launch_ranks),
before anything touches the GPU.  The job is `instances per GPU x world` GLOBAL instances, each
rank takes its contiguous shard (ol_dsp_amd.dist.shard) and derives every instance's parameters
and input stream from its global index (ol_dsp_amd.workload), so an N-GPU run processes exactly
the instances a one-GPU run of the same total would.  No data-path collective (weak scaling); one
RCCL all-reduce after each timed region gathers the counters.

Repetitions ("median of 5"): every leg is built first and kept alive; then each leg
runs --reps timed regions of exactly --steps steps (barrier + device sync on both sides, max over
ranks), the leg order rotated by one leg per repetition, after at least --leg-warmup untimed steps
before a leg's first region and --rep-warmup before each later one.  Every reported time is the
median region, with the min-max range beside it.

Prints ONE compact JSON line (rank 0; the whole record, every leg in full, goes to --full-json):
  roofline     : algorithmic bytes of the dominant kernel / its HIP-event-timed duration vs 8 TB/s
                 (frac = read+write, frac_read = the read share: the north star's HBM-read roofline)
  cpu_baseline : the CPU oracle (port) or the compiled reference (reference) on all host cores
                 given to this process, at -O2 (value) and -O0 (value_O0, the reference's default)
  parity       : UNTIMED, after all legs: sampled instances (first, last, wave edges) of the last
                 timed block against the CPU oracle replaying the same W+K blocks (inputs read back
                 from the device pool, the same control/note schedule) -- bit-exact for the reverb,
                 chorus, pitch-shift, chain and rack, max rel err vs 1e-5 for the voices
  cpu_c1       : BASELINE configs[0]: one chorus instance, one core, per-frame calls
  also         : the other BASELINE configs timed in the same run, one compact entry each (the
                 north star's 65,536 chains last)
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
VOICE_TOL = 1e-5      # max |gpu - ref| / max(|ref|, rms(ref)) per voice (tests/test_gpu_parity.py)
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
# legs in print order; the north star's 65,536 chains last (the end of the line survives any tail cut)
# (dattorro / dattorro_rpd and chain_rpd / chain_65536 adjacent: each pair on the same box state)
DEFAULT_ALSO = ("voice_poly,voice_events,chain_cc,voice_moog,fxrack,voice,chain,dattorro,dattorro_rpd,"
                "chain_rpd,chain_65536")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without torchrun, N > 1 launches the N rank processes itself")
    ap.add_argument("--steps", type=int, default=200, help="steps (blocks) in each timed region")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5,
                    help="timed regions per leg (SURVEY 8d: median of 5), leg order rotated between them")
    ap.add_argument("--leg-warmup", type=int, default=50,
                    help="untimed steps before a leg's first region at least (the sustained clock: "
                         "profiles/r5/chorus_launch_durations.txt)")
    ap.add_argument("--rep-warmup", type=int, default=10, help="untimed steps before each later region of a leg")
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
    ap.add_argument("--no-parity", action="store_true", help="skip the untimed oracle parity check per leg")
    ap.add_argument("--traffic-json", default="", help="PMC traffic summary (tools/pmc_traffic.py)")
    ap.add_argument("--full-json", default=os.path.join(ROOT, "gpurun_out", "bench_full.json"),
                    help="where the full (verbose) record of every leg is written ('' = nowhere)")
    ap.add_argument("--stub", action="store_true",
                    help="CPU launcher check: a no-GPU stand-in leg over gloo (tests/test_bench_launch.py)")
    return ap.parse_args(argv)


def _r(x, sig: int = 4):
    """Round for the compact line (significant digits)."""
    if x is None or isinstance(x, (bool, int, str)):
        return x
    x = float(x)
    return float(f"{x:.{sig}g}") if np.isfinite(x) else None


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


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    return O


def _rcp_table():
    """The committed v_rcp_f32 model of gfx950 (tests/golden/rcp_f32_gfx950.npz through
    oracle/rcp_model.py, sha256-checked: the voice oracle's kernel-arithmetic mode,
    oracle/voice_ref.c); None when the fixture is absent."""
    try:
        _oracle()
        import rcp_model
        return rcp_model.load()
    except (OSError, ValueError, ImportError):
        return None


def _oracle_bank(kind: str, p: np.ndarray, sr: float, o0: bool = False, ref: bool = False, notes=None,
                 frames: int = 256, kernel_arith: bool = False):
    """CPU oracle bank of `kind` for params p [fields][m] (columns = instances): (step, banks,
    setter).  step(x [ch][frames][m] or None, threads) -> [och][frames][m]; setter(j, field, v)
    sets one C-ABI field of instance j (the chain's fields route to their stage)."""
    O = _oracle()
    n = p.shape[1]
    if kind == "dattorro":
        bank = O.Dattorro(n, ref=ref, o0=o0)
        for i in range(n):
            for f in range(7):
                bank.set(i, f, float(p[f, i]))
        return (lambda x, t=1: bank.process(x, t)), bank, (lambda j, f, v: bank.set(j, f, v))
    if kind in ("chorus", "pitchshift"):
        bank = O.Chorus(n, sr, 0 if kind == "chorus" else 1, o0=o0)
        fmap = (lambda f: f) if kind == "chorus" else (lambda f: (0, 7)[f])
        for i in range(n):
            for f in range(p.shape[0]):
                bank.set(i, fmap(f), float(p[f, i]))
        return (lambda x, t=1: bank.process(x, t)), bank, (lambda j, f, v: bank.set(j, fmap(f), v))
    if kind == "fxrack":
        bank = O.FxRack(n, sr, o0=o0)
        for i in range(n):
            for f in range(p.shape[0]):
                bank.set(i, f, float(p[f, i]))
        return (lambda x, t=1: bank.process(x, t)), bank, (lambda j, f, v: bank.set(j, f, v))
    if kind in VOICE_KINDS:
        bank = O.Voice(n, sr, moog=kind == "voice_moog", o0=o0, kernel_arith=kernel_arith)
        for i in range(n):
            bank.config(i, p[:, i])
            if notes is not None:
                bank.note(i, True, int(notes[i]))
        return (lambda x, t=1: bank.process(frames if x is None else x.shape[1], t)), bank, None
    # chain: the composed stages, each a real bank with the chain's parameters
    c1, c2, d = O.Chorus(n, sr, 0, o0=o0), O.Chorus(n, sr, 1, o0=o0), O.Dattorro(n, ref=ref, o0=o0)

    def setter(j, f, v):
        if f < 8:
            c1.set(j, f, v)
        elif f < 10:
            c2.set(j, (0, 7)[f - 8], v)
        else:
            d.set(j, f - 10, v)
    for i in range(n):
        for f in range(p.shape[0]):
            setter(i, f, float(p[f, i]))
    return (lambda x, t=1: d.process(c2.process(c1.process(x, t), t), t)), (c1, c2, d), setter


def cpu_baseline(kind: str, block: int, sr: float, budget_s: float, threads: int, pset: str = "") -> dict:
    """Time the CPU oracle (or, for the reverb, the reference verb.cpp compiled here) on a bounded
    sample of the same workload: the same global instances 0..n-1 with the same parameters and
    input streams, 256-frame blocks, OpenMP schedule(static) over instances, until the wall
    budget is spent; then the same at -O0 for a quarter of the budget."""
    O = _oracle()
    from ol_dsp_amd.workload import instance_params, noise_np, voice_notes
    n = 8192 if kind not in VOICE_KINDS else 32768
    ich = 0 if kind in VOICE_KINDS else 2
    x = noise_np(0, n, block, 2) if ich else None
    ref = kind in ("dattorro", "chain") and O.ref_available() and O.ref_available(o0=True)
    p = instance_params(pset or kind, 0, n)
    notes = voice_notes(0, n) if kind in VOICE_KINDS else None

    def timed(o0: bool, budget: float):
        step, _keep, _ = _oracle_bank(kind, p, sr, o0, ref, notes, block)
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
    O = _oracle()
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
# Untimed on-box parity of each leg's last timed block (the oracle as the checker)
# ------------------------------------------------------------------------------------------------
def sample_instances(n: int) -> np.ndarray:
    """First, last, and the edges of waves (32 chorus instances, 64 reverb/voice lanes) and of the
    middle of the shard."""
    idx = {0, 1, 31, 32, 63, 64, 127, n // 2 - 1, n // 2, n - 65, n - 64, n - 33, n - 32, n - 1}
    return np.array(sorted(i for i in idx if 0 <= i < n), np.int64)


def parity_check(job: dict, sr: float) -> dict:
    """Replay the leg's W+K blocks for the sampled instances on the CPU oracle and compare the
    last block with what the GPU produced (job filled in by Leg.finish)."""
    kind, idx, B = job["kind"], job["idx"], job["block"]
    m = len(idx)
    voice = kind in VOICE_KINDS
    xs, pool_n = job.get("pool"), job.get("pool_n", 1)

    def replay(kernel_arith=False):
        step, _banks, setter = _oracle_bank(kind, job["params"], sr, notes=job.get("notes"), frames=B,
                                            kernel_arith=kernel_arith)
        bank = _banks if voice else None
        y = None
        for b in range(job["blocks"]):
            if voice:
                if b == job.get("note_off_block", -1):
                    for j in range(m):
                        bank.note(j, False, int(job["notes"][j]))
                for j, on, note in job.get("events", lambda b: [])(b):
                    bank.note(j, on, note)
            for j, f, v in job.get("ccs", lambda b: [])(b):
                setter(j, f, v)
            y = step(None if voice else xs[b % pool_n])
        return y

    y = replay()
    g = job["gpu"]
    res = {"instances": m, "blocks": job["blocks"]}
    if voice:
        fin = np.isfinite(y).all(axis=(0, 1)) & np.isfinite(g).all(axis=(0, 1))
        same_fin = bool(np.array_equal(np.isfinite(y), np.isfinite(g)))
        a = g[0][:, fin].T.astype(np.float64)
        r = y[0][:, fin].T.astype(np.float64)
        rms = np.sqrt(np.mean(r ** 2, axis=1, keepdims=True)) + 1e-30
        err = float(np.max(np.abs(a - r) / np.maximum(np.abs(r), rms))) if a.size else 0.0
        res.update({"check": f"max_rel_err<={VOICE_TOL:g}", "max_rel_err": err,
                    "ok": bool(same_fin and err <= VOICE_TOL), "finite_instances": int(fin.sum())})
        # and bit-exact against the oracle's kernel-arithmetic mode (the measured v_rcp_f32 model)
        tab = _rcp_table()
        if tab is not None:
            O = _oracle()
            O.set_rcp_table(tab)
            try:
                yk = replay(kernel_arith=True)
            finally:
                O.set_rcp_table(None)
            fk = np.isfinite(yk)
            bad = int(np.count_nonzero(yk[fk].view(np.uint32) != np.ascontiguousarray(g)[fk].view(np.uint32)))
            exact = bool(np.array_equal(fk, np.isfinite(g)) and bad == 0)
            res.update({"check": f"bit-exact(karith)+rel<={VOICE_TOL:g}",
                        "mismatched_samples_kernel_arith": bad, "ok": res["ok"] and exact})
    else:
        bad = int(np.count_nonzero(np.ascontiguousarray(g).view(np.uint32) != np.ascontiguousarray(y).view(np.uint32)))
        res.update({"check": "bit-exact", "ok": bad == 0, "mismatched_samples": bad})
    if "bus_gpu" in job:     # the mix kernel on the last block: bit-exact against Polyvoice's += order
        O = _oracle()
        bus_ref = O.mix_ref(job["bus_voices"], job["bus_lists"])
        bad = int(np.count_nonzero(bus_ref.view(np.uint32) != job["bus_gpu"].view(np.uint32)))
        res["buses"] = {"check": "bit-exact", "buses": len(job["bus_lists"]), "mismatched_samples": bad}
        res["ok"] = res["ok"] and bad == 0
    return res


# ------------------------------------------------------------------------------------------------
# GPU workloads
# ------------------------------------------------------------------------------------------------
_LIB_SHA = []


def _lib_sha256() -> str:
    """sha256 of the libolfx.so this process runs (the traffic files' build stamp)."""
    if not _LIB_SHA:
        import hashlib

        from ol_dsp_amd import _lib
        with open(_lib.LIB_PATH, "rb") as f:
            _LIB_SHA.append(hashlib.sha256(f.read()).hexdigest())
    return _LIB_SHA[0]


def _traffic(name: str, n: int, B: int, override: str = "", kernel: str = ""):
    """The PMC traffic summary of this workload's kernel (tools/pmc_traffic.py), if one was recorded
    for the same instance count, block and kernel AND with the same build: the file's
    `libolfx_sha256` must be the hash of the library this process runs (counters
    of an older build are never attached to the current kernel)."""
    for tj in ([override] if override else []) + [os.path.join(ROOT, "profiles", f"traffic_{name}_{n}.json"),
                                                  os.path.join(ROOT, "profiles", f"traffic_{name}.json")]:
        if tj and os.path.exists(tj):
            try:
                with open(tj) as f:
                    tr = json.load(f)
                kernels = tr.get("counters_per_kernel") or {}
                # a launch sequence ("a+b") needs a summary of every kernel in it
                same_kernel = not kernel or all(any(part in k for k in kernels) for part in kernel.split("+"))
                if (tr.get("instances") == n and tr.get("block") == B and same_kernel
                        and tr.get("libolfx_sha256") == _lib_sha256()):
                    return tr
            except Exception:
                pass
    return None


class StubLeg:
    """--stub: the launcher's CPU check.  No engine and no GPU: each rank 'processes' its shard (a
    host sleep per step) through the same repetition, rotation and per-region all-reduce (gloo) as a
    real leg."""

    def __init__(self, name: str, n_per_gpu: int, args, rank: int, world: int):
        from ol_dsp_amd.dist import shard
        self.name, self.n_per_gpu, self.args, self.rank, self.world = name, n_per_gpu, args, rank, world
        self.total = n_per_gpu * world
        self.first, self.n = shard(self.total, world, rank)
        self.reps = []

    def warm(self, steps: int) -> None:
        time.sleep(0.001 * steps)

    def timed(self, steps: int) -> None:
        from ol_dsp_amd.dist import RunStats, reduce_stats
        import torch.distributed as dist
        if dist.is_initialized():
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            time.sleep(0.001)
        elapsed = time.perf_counter() - t0
        if dist.is_initialized():
            dist.barrier()
        self.reps.append(reduce_stats(RunStats(elapsed, elapsed * 1e3 / steps, float(self.n) * self.args.block * steps,
                                               0.0, 1.0)))

    def finish(self) -> dict:
        from ol_dsp_amd.dist import RunStats, reduce_stats
        st = reduce_stats(RunStats(0.0, 0.0, 0.0, float(self.first), 1.0))   # the shard starts: distinct shards
        if self.rank != 0:
            return {}
        res = _rep_summary(self.reps, self.args.steps)
        res.update({"metric": METRIC, "unit": "stereo samples/s", "output_checksum": st.checksum,
                    "config": {"workload": self.name, "instances_per_gpu": self.n_per_gpu, "instances_total": self.total,
                               "block": self.args.block, "parallelism": f"instance-shard x{self.world} (stub: no GPU)"},
                    "roofline": None, "cpu_baseline": None, "parity": None, "output_nonfinite_rank0": 0})
        return res


def _median(v):
    s = sorted(v)
    m = len(s)
    return s[m // 2] if m % 2 else 0.5 * (s[m // 2 - 1] + s[m // 2])


def _rep_summary(reps, steps: int) -> dict:
    """The leg's repetitions (each a barrier-bracketed region of `steps` steps, max over ranks):
    value and ms_per_step from the median region, the kernel time median, the min-max spread."""
    el = [r.elapsed_s for r in reps]
    km = [r.kernel_ms for r in reps]
    frames = reps[0].frames                     # per region, summed over ranks
    e_med, k_med = _median(el), _median(km)
    return {"value": frames / e_med, "ms_per_step": e_med / steps * 1e3, "frames": frames,
            "ranks_reporting": int(reps[0].ranks), "kernel_ms_median": k_med,
            "reps": {"n": len(reps), "steps_each": steps, "kernel_ms": km, "elapsed_s": el,
                     "kernel_ms_min": min(km), "kernel_ms_max": max(km),
                     "kernel_spread": (max(km) - min(km)) / k_med if k_med > 0 else None}}


class Leg:
    """One workload on this rank's GPU: its engine, input pool and prebuilt per-step calls, kept
    alive across the repetitions so that main() can interleave the legs.  `warm(W)` runs W untimed
    steps; `timed(K)` one region of exactly K steps bracketed by a barrier and a device sync on both
    sides (max over ranks, one all-reduce after it); `finish()` the untimed checks and the result.
    Steps are numbered over the whole run (inputs from the pool, event / control schedules, the
    voices' NoteOff at the middle block), so the parity replay follows every block the engine ran."""

    def __init__(self, name: str, n_per_gpu: int, args, rank: int, world: int, dev, with_cpu: bool,
                 total_blocks: int):
        import torch

        import ol_dsp_amd as ofx
        from ol_dsp_amd.dist import shard
        from ol_dsp_amd.workload import instance_params, noise_torch, voice_notes

        self.name, self.args, self.rank, self.world, self.dev = name, args, rank, world, dev
        self.with_cpu = with_cpu
        kind, _, desc = WORKLOADS[name]
        self.kind, self.desc, self.n_per_gpu = kind, desc, n_per_gpu
        self.total = n_per_gpu * world
        first, n = shard(self.total, world, rank)
        self.first, self.n = first, n
        B = self.B = args.block
        eng = self.eng = ofx.Engine(kind, n, sample_rate=args.sample_rate, block=B, device=dev.index or 0)
        self.pset = PARAM_SET.get(name, kind)
        params = self.params = instance_params(self.pset, first, n)
        eng.set_params(0, params)
        ich, och = eng.info.in_channels, eng.info.out_channels
        self.ich = ich

        # input pool: distinct synthetic blocks of each global instance's own stream, on the device
        blk_bytes = max(ich, 1) * B * n * 4
        self.pool_n = pool_n = max(2, int(args.pool_bytes // blk_bytes)) if ich else 1
        self.pool = noise_torch(first, n, B, ich, dev, blocks=pool_n) if ich else [None]
        self.out = torch.empty((och, B, n), device=dev)
        self.voice = voice = kind in VOICE_KINDS
        self.notes = notes = voice_notes(first, n)
        self.note_off = None
        self.note_off_block = total_blocks // 2
        if voice:   # NoteOn for every voice at block 0, NoteOff at the middle block of the run
            eng.note_events(eng.make_events(np.arange(n), 1, notes))
            self.note_off = eng.make_events(np.arange(n), 0, notes)
        # control legs: the per-step calls are prebuilt (untimed), so a step is the library call only
        gi = self.gi = np.arange(first, first + n)
        self.step_events = None
        if name == "voice_events":     # voices i % 40 == k % 40 get NoteOn, i % 40 == (k + 20) % 40 NoteOff
            self.step_events = []
            for k in range(40):
                on = np.nonzero(gi % 40 == k)[0]
                off = np.nonzero(gi % 40 == (k + 20) % 40)[0]
                ev_on = eng.make_events(on, 1, (notes[on] + 12 * (k & 1)) % 128)
                ev_off = eng.make_events(off, 0, notes[off])
                self.step_events.append(np.concatenate([ev_on, ev_off]))
        self.step_ccs = None
        if name == "chain_cc":         # chains i % 100 == k % 100 get a new value of one field per step
            from ol_dsp_amd.workload import uniform01
            fields = [("chorus_depth", .08, 1.0), ("chorus_mix", 0.0, 1.0), ("verb_decay", .25, .95),
                      ("verb_damping", .05, .95), ("pitch_shift", 0.0, 3.0)]
            self.step_ccs = []
            for k in range(100):
                sel = np.nonzero(gi % 100 == k)[0].astype(np.uint32)
                fname, lo, hi = fields[k % len(fields)]
                vals = (lo + (hi - lo) * uniform01(7, k, int(first), n)[sel]).astype(np.float32)
                self.step_ccs.append((eng.field(fname), sel, vals))
        self.bus = None
        if name == "voice_poly":       # Polyvoice buses of 8 voices (Polyvoice.h:28-33)
            self.bus_lists = [list(range(g, min(g + 8, n))) for g in range(0, n, 8)]
            eng.mix_config(self.bus_lists)
            self.bus = torch.zeros((B, eng.n_buses), device=dev)
        self.stream = torch.cuda.Stream(dev)       # dedicated non-default stream: events see the kernels
        torch.cuda.synchronize(dev)

        # The timed loop calls the C-ABI directly with prebuilt arguments (Engine.process's checks and
        # tensor handling cost ~20 us of Python per call, more than a voice block's kernel): the host
        # must stay ahead of the GPU, or the event pair would time the host's launch latency.
        import ctypes

        from ol_dsp_amd import _lib
        self._lib = _lib
        self.lib, self.h = eng.lib, eng.handle
        c_stream = ctypes.c_void_p(self.stream.cuda_stream)
        c_out = ctypes.c_void_p(self.out.data_ptr())
        self.proc_args = [(self.h, ctypes.c_void_p(p.data_ptr() if p is not None else 0), c_out, B, _lib.IO_DEVICE,
                           c_stream) for p in self.pool]
        self.ev_args = [(self.h, e_.ctypes.data_as(ctypes.POINTER(_lib.Event)), len(e_))
                        for e_ in self.step_events or []]
        self.cc_args = [(self.h, f, sel.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                         vals.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(sel))
                        for f, sel, vals in self.step_ccs or []]
        self.k = 0                     # steps run so far (= blocks processed)
        self.reps = []

    def step(self) -> None:
        k = self.k
        rc = 0
        if self.voice and k == self.note_off_block:
            self.eng.note_events(self.note_off)
        if self.ev_args:
            rc |= self.lib.olfx_note_events(*self.ev_args[k % 40])
        if self.cc_args:
            rc |= self.lib.olfx_set_param_list(*self.cc_args[k % 100])
        rc |= self.lib.olfx_process(*self.proc_args[k % self.pool_n])
        if rc:
            self._lib.check(rc, self.h)
        if self.bus is not None:
            self.eng.mix(self.out, self.bus, stream=self.stream.cuda_stream)
        self.k += 1

    def warm(self, steps: int) -> None:
        import torch
        for _ in range(steps):
            self.step()
        torch.cuda.synchronize(self.dev)

    def timed(self, steps: int) -> None:
        """One region of exactly `steps` steps.  Kernel time: ONE event pair on the launch stream
        around the region (GPU time per step = the launch duration plus the gap between launches; a
        pair per step would add two timestamp markers between consecutive kernels, ~3-4 us each on
        the command processor, 10-20 % of a 35 us voice block: notes r5 §4)."""
        import torch

        from ol_dsp_amd.dist import RunStats, reduce_stats
        dev = self.dev
        region = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        torch.cuda.synchronize(dev)
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        region[0].record(self.stream)
        for _ in range(steps):
            self.step()
        region[1].record(self.stream)
        torch.cuda.synchronize(dev)
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        kern_ms = region[0].elapsed_time(region[1]) / steps
        self.reps.append(reduce_stats(RunStats(elapsed, kern_ms, float(self.n) * self.B * steps, 0.0, 1.0), device=dev))

    def finish(self) -> dict:
        import torch

        from ol_dsp_amd.dist import RunStats, reduce_stats
        args, dev, n, B, eng = self.args, self.dev, self.n, self.B, self.eng
        K = args.steps
        out, bus, stream = self.out, self.bus, self.stream
        # sum |y| over the finite outputs of the last block (a voice whose Svf diverges -- possible in
        # the reference DaisySP arithmetic at high cutoff, low resonance and high drive -- yields
        # inf/NaN there too); the count of non-finite samples beside it
        finite = torch.isfinite(out)
        nonfinite = int((~finite).sum().item())
        checksum = float(torch.where(finite, out.abs(), torch.zeros_like(out)).sum().item())
        bus_sum = float(bus.abs().sum().item()) if bus is not None else None
        mix_ms = None
        if bus is not None:            # the mix alone, K launches between one event pair (untimed for value)
            scratch = torch.zeros_like(bus)
            for _ in range(args.warmup):
                eng.mix(out, scratch, stream=stream.cuda_stream)
            mreg = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            mreg[0].record(stream)
            for _ in range(K):
                eng.mix(out, scratch, stream=stream.cuda_stream)
            mreg[1].record(stream)
            torch.cuda.synchronize(dev)
            mix_ms = reduce_stats(RunStats(0.0, mreg[0].elapsed_time(mreg[1]) / K, 0.0, 0.0, 1.0), device=dev).kernel_ms
            for r in self.reps:
                r.kernel_ms = max(r.kernel_ms - mix_ms, 1e-6)

        # untimed parity material: the last block of sampled instances, the pool blocks they read
        # (read back from the device: exactly the timed inputs) and the leg's event / control schedule
        parity_job = None
        if self.rank == 0 and not args.no_parity:
            if bus is not None:        # two whole buses (first, last) so the mix can be checked too
                nb = len(self.bus_lists)
                idx = np.array(sorted(set(self.bus_lists[0]) | set(self.bus_lists[nb - 1])), np.int64)
            else:
                idx = sample_instances(n)
            ti = torch.from_numpy(idx).to(dev)
            parity_job = {"kind": self.kind, "idx": idx, "block": B, "blocks": self.k,
                          "params": np.ascontiguousarray(self.params[:, idx]),
                          "gpu": out.index_select(2, ti).cpu().numpy()}
            if self.ich:
                parity_job["pool"] = [np.ascontiguousarray(p.index_select(2, ti).cpu().numpy()) for p in self.pool]
                parity_job["pool_n"] = self.pool_n
            notes, gi = self.notes, self.gi
            if self.voice:
                parity_job["notes"] = notes[idx].astype(np.int64)
                parity_job["note_off_block"] = self.note_off_block
            if self.step_events is not None:
                pos = {int(i): j for j, i in enumerate(idx)}
                sched = []
                for k in range(40):
                    on = [(pos[int(i)], True, int((notes[i] + 12 * (k & 1)) % 128)) for i in idx if gi[i] % 40 == k]
                    off = [(pos[int(i)], False, int(notes[i])) for i in idx if gi[i] % 40 == (k + 20) % 40]
                    sched.append(on + off)
                parity_job["events"] = lambda b, s=sched: s[b % 40]
            if self.step_ccs is not None:
                pos = {int(i): j for j, i in enumerate(idx)}
                sched = []
                for f, sel, vals in self.step_ccs:
                    sched.append([(pos[int(i)], f, float(v)) for i, v in zip(sel, vals) if int(i) in pos])
                parity_job["ccs"] = lambda b, s=sched: s[b % 100]
            if bus is not None:        # the mix of the last block into zeroed buses (untimed)
                bus_chk = torch.zeros_like(bus)
                eng.mix(out, bus_chk, stream=stream.cuda_stream)
                torch.cuda.synchronize(dev)
                pos = {int(i): j for j, i in enumerate(idx)}
                lists = [self.bus_lists[0], self.bus_lists[nb - 1]]
                parity_job["bus_lists"] = [[pos[v] for v in bl] for bl in lists]
                parity_job["bus_voices"] = parity_job["gpu"][0]
                parity_job["bus_gpu"] = np.ascontiguousarray(bus_chk[:, [0, nb - 1]].cpu().numpy())

        cs = reduce_stats(RunStats(0.0, 0.0, 0.0, checksum, 1.0), device=dev)
        bpf, rbpf, kname = eng.algorithmic_bytes_per_frame, eng.algorithmic_read_bytes_per_frame, eng.kernel_name
        eng.close()
        del self.pool, self.out
        self.bus = None
        torch.cuda.empty_cache()
        if self.rank != 0:
            return {}

        res = _rep_summary(self.reps, K)
        kern_ms = res.pop("kernel_ms_median")
        voice = self.voice
        per_launch = n * B
        achieved = bpf * per_launch / (kern_ms * 1e-3) / 1e9
        achieved_r = rbpf * per_launch / (kern_ms * 1e-3) / 1e9
        tr = _traffic(self.name, n, B, args.traffic_json if self.name == args.workload else "", kname)
        traffic = tr.get("hbm_bytes_per_launch") if tr else None
        # the PMC-measured HBM bytes of the same kernel (profiles/traffic_<workload>.json, separate
        # --pmc passes) over this run's kernel time: what HBM actually moved, against the peak
        measured = {"traffic_build": (tr or {}).get("libolfx_sha256", "none recorded for this libolfx.so")[:16]}
        if tr and traffic:
            measured["hbm_gbs_measured"] = traffic / (kern_ms * 1e-3) / 1e9
            rd = tr.get("read_bytes_by_request_size")
            if rd:
                measured.update({"traffic_read": rd, "hbm_read_gbs_measured": rd / (kern_ms * 1e-3) / 1e9,
                                 "frac_read_measured": rd / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS})
        timing = ("median over the repetitions of one HIP event pair around the K timed steps / K, less the mix's "
                  "own time (one pair around K mix launches after the timed regions)" if bus is not None else
                  "median over the repetitions of one HIP event pair on the launch stream around the K timed steps / K "
                  "(launch duration + launch gap)")
        if voice:
            fps = VOICE_MOOG_FLOPS_PER_SAMPLE if self.kind == "voice_moog" else VOICE_FLOPS_PER_SAMPLE
            tflops = fps * per_launch / (kern_ms * 1e-3) / 1e12
            roofline = {"bound": "valu", "achieved": tflops, "peak": FP32_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": tflops / FP32_VALU_PEAK_TFLOPS, "traffic": traffic,
                        "kernel": kname, "kernel_ms": kern_ms, "kernel_timing": timing,
                        "algorithmic_flops_per_frame": fps, "algorithmic_bytes_per_frame": bpf, "hbm_gbs": achieved,
                        "frames_per_launch": per_launch}
        else:
            roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                        "achieved_read": achieved_r, "frac_read": achieved_r / HBM_PEAK_GBS,
                        "kernel": kname, "kernel_ms": kern_ms, "kernel_timing": timing,
                        "algorithmic_bytes_per_frame": bpf, "algorithmic_read_bytes_per_frame": rbpf,
                        "frames_per_launch": per_launch, **measured}
        res.update({"metric": METRIC, "unit": "voice samples/s" if voice else "stereo samples/s",
                    "config": {"workload": self.name, "restates": self.desc, "instances_per_gpu": self.n_per_gpu,
                               "instances_total": self.total, "block": B, "sample_rate": args.sample_rate,
                               "input_pool_blocks": self.pool_n,
                               "parallelism": f"instance-shard x{self.world} (no data-path collective)"},
                    "roofline": roofline, "output_checksum": cs.checksum, "output_nonfinite_rank0": nonfinite})
        if mix_ms is not None:
            nb = (n + 7) // 8
            mix_bytes = 4.0 * n * B + 8.0 * nb * B          # voice reads + bus read-modify-write
            res["mix"] = {"kernel": "voice_mix_v4", "kernel_ms": mix_ms, "bound": "hbm",
                          "achieved": mix_bytes / (mix_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                          "frac": mix_bytes / (mix_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                          "algorithmic_bytes_per_launch": mix_bytes, "bus_checksum_rank0": bus_sum}
        if self.step_events is not None:
            res["control"] = {"events_per_block": int(np.mean([len(e) for e in self.step_events])),
                              "note": "NoteOn/NoteOff folded per voice on the host and applied by the voice kernel at "
                                      "the block start (olfx_engine.cpp fold_events, voice.hip voice_event)"}
        if self.step_ccs is not None:
            res["control"] = {"instances_changed_per_block": int(np.mean([len(c[1]) for c in self.step_ccs])),
                              "note": "changed coefficients re-derived on the host for those instances only and "
                                      "scattered on the device ahead of the block (control.hip coef_scatter)"}
        # the CPU baseline and the parity replay run after every GPU leg (main): no leg is timed right
        # after a many-thread CPU run (a short-kernel leg measured 1.7x slow once, launch-bound behind it)
        res["cpu_baseline"] = None
        res["parity"] = None
        if self.with_cpu and self.world == 1 and args.cpu_seconds > 0:
            res["cpu_job"] = (self.kind, PARAM_SET.get(self.name, ""))
        if parity_job is not None:
            res["parity_job"] = parity_job
        return res


def run_cpu_jobs(jobs, reuse, parity_jobs, args):
    """The deferred CPU work: baselines (jobs = [(result dict, kind, param set)], reuse = [(result
    dict, the dict whose baseline it reuses, its key)]) and the parity replays ([(result dict,
    job)])."""
    threads = args.cpu_threads or host_facts()["nproc"]
    for target, job in parity_jobs:
        try:
            target["parity"] = parity_check(job, args.sample_rate)
        except Exception as e:                 # a checker failure is reported, never hidden
            target["parity"] = {"ok": False, "error": f"{type(e).__name__}: {e}"}
    for target, kind, pset in jobs:
        target["cpu_baseline"] = cpu_baseline(kind, args.block, args.sample_rate, args.cpu_seconds, threads, pset)
    for target, src, key in reuse:
        if src.get("cpu_baseline"):
            target["cpu_baseline"] = dict(src["cpu_baseline"], reused_from=key)


# ------------------------------------------------------------------------------------------------
# The compact line
# ------------------------------------------------------------------------------------------------
def _compact_parity(p):
    if not p:
        return p
    if "error" in p:
        return {"ok": False, "error": p["error"][:120]}
    out = {"ok": p["ok"], "check": p["check"], "inst": p["instances"], "blocks": p["blocks"]}
    if "max_rel_err" in p:
        out["max_rel_err"] = _r(p["max_rel_err"], 3)
    if p.get("mismatched_samples"):
        out["mismatched"] = p["mismatched_samples"]
    if "buses" in p:
        out["buses_bit_exact"] = p["buses"]["mismatched_samples"] == 0
    return out


def compact_leg(r: dict) -> dict:
    """One leg in ~250 bytes: instances, kernel, time, throughput, roofline fractions, measured
    traffic per frame, the CPU baseline and the parity verdict."""
    rf = r["roofline"]
    if rf is None:                  # --stub
        return {"n": r["config"]["instances_per_gpu"], "value": _r(r["value"]), "ranks": r["ranks_reporting"]}
    c = {"n": r["config"]["instances_per_gpu"], "kernel": rf["kernel"], "kernel_ms": _r(rf["kernel_ms"]),
         "value": _r(r["value"]), "bound": rf["bound"], "frac": _r(rf["frac"], 3)}
    reps = r.get("reps")
    if reps:                        # the repetitions' kernel-time range around the median
        c["ms_range"] = [_r(reps["kernel_ms_min"]), _r(reps["kernel_ms_max"])]
    if rf["bound"] == "hbm":
        c["frac_read"] = _r(rf["frac_read"], 3)
        if rf.get("traffic"):
            c["traffic_B_per_frame"] = _r(rf["traffic"] / rf["frames_per_launch"], 4)
    if "mix" in r:
        c["mix"] = {"kernel_ms": _r(r["mix"]["kernel_ms"]), "frac": _r(r["mix"]["frac"], 3)}
    if "control" in r and "kernel_ms_ratio" in r["control"]:
        c["vs_event_free"] = _r(r["control"]["kernel_ms_ratio"], 4)
    cb = r.get("cpu_baseline")
    if cb:
        c["cpu_baseline"] = {"value": _r(cb["value"]), "kind": cb["kind"], "cores": cb["cores"]}
    c["parity"] = _compact_parity(r.get("parity"))
    return c


def _box_copy_rate(torch, dev):
    """The box's device-to-device copy rate (2 GiB, read + write bytes), untimed and after the legs: a
    reference for comparing lines from different boxes, whose HBM rates differ."""
    try:
        a = torch.empty(1 << 29, dtype=torch.float32, device=dev)
        b = torch.empty_like(a)
        for _ in range(3):
            b.copy_(a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        gbs = 2 * a.numel() * 4 * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9
        del a, b
        return {"copy_gbs": _r(gbs, 1), "what": "torch device copy of 2 GiB, read + write bytes, after the legs"}
    except Exception as ex:       # informational only
        return {"copy_gbs": None, "error": str(ex)[:80]}


def main():
    args = parse()
    from ol_dsp_amd.dist import env_ranks, launch_ranks, self_command
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no torchrun around us: start the N rank processes here, before anything touches the GPU
        sys.exit(launch_ranks(self_command(), args.gpus))

    import torch
    import torch.distributed as dist

    rank, world, local = env_ranks()
    # under a launcher (WORLD_SIZE set, 1 included) the ranks form a process group: RCCL over xGMI
    # ("nccl") on the GPUs, gloo for the CPU stub
    grouped = world > 1 or "WORLD_SIZE" in os.environ
    if args.stub:
        if grouped:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cpu")
    else:
        if grouped:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)

    n = args.instances or WORKLOADS[args.workload][1]
    also = args.also if args.also is not None else (DEFAULT_ALSO if args.workload == "chorus" and not args.stub else "")
    also_names = [a for a in also.split(",") if a]
    R, K = max(1, args.reps), args.steps
    W0 = max(args.warmup, args.leg_warmup)       # before a leg's first region: the sustained clock
    Wr = args.rep_warmup                         # before each later region of the leg
    total_blocks = W0 + R * K + (R - 1) * Wr
    # every leg is built first and kept alive, then the regions run leg after leg, the order rotated
    # by one leg per repetition (each leg's regions see different neighbours and clock states)
    specs = [(args.workload, n, True, args.workload)]
    for name in also_names:
        twin = EVENT_FREE.get(name)
        tkey = twin if twin != "chain" else "chain_16384"
        # a control leg's CPU work per block is its twin's (the CPU oracle applies events and
        # parameters per instance at block boundaries): the twin's measured baseline is reused
        reuse = bool(twin and (twin in also_names or twin == args.workload))
        specs.append((name, WORKLOADS[name][1], not reuse, name if name != "chain" else "chain_16384"))
    if args.stub:
        legs = [StubLeg(name, npg, args, rank, world) for name, npg, _, _ in specs]
    else:
        legs = [Leg(name, npg, args, rank, world, dev, with_cpu, total_blocks) for name, npg, with_cpu, _ in specs]
    m = len(legs)
    for r in range(R):
        for leg in legs[r % m:] + legs[:r % m]:
            leg.warm(W0 if r == 0 else Wr)
            leg.timed(K)
    results = [leg.finish() for leg in legs]
    main_res = results[0]
    box = _box_copy_rate(torch, dev) if rank == 0 and not args.stub else None
    also_res = {key: res for (_, _, _, key), res in zip(specs[1:], results[1:])}
    cpu_jobs, cpu_reuse, parity_jobs = [], [], []
    if rank == 0 and not args.stub:
        for (name, _, with_cpu, key), r in zip(specs, results):
            if "cpu_job" in r:
                cpu_jobs.append((r, *r.pop("cpu_job")))
            elif name in EVENT_FREE and not with_cpu:
                twin = EVENT_FREE[name]
                cpu_reuse.append((r, twin if twin != "chain" else "chain_16384"))
            if "parity_job" in r:
                parity_jobs.append((r, r.pop("parity_job")))
        # the control legs against their event-free twins (an `also` leg or the main workload)
        for key, r in also_res.items():
            base = EVENT_FREE.get(key)
            if not base:
                continue
            bkey = base if base != "chain" else "chain_16384"
            b = also_res.get(bkey) or (main_res if base == args.workload else None)
            if b is not None:
                r["control"].update({
                    "event_free_kernel_ms": b["roofline"]["kernel_ms"], "event_free_ms_per_step": b["ms_per_step"],
                    "kernel_ms_ratio": r["roofline"]["kernel_ms"] / b["roofline"]["kernel_ms"],
                    "ms_per_step_ratio": r["ms_per_step"] / b["ms_per_step"]})
        cpu_reuse = [(r, also_res.get(tkey) or (main_res if tkey == args.workload else {}), tkey)
                     for r, tkey in cpu_reuse]

    if rank == 0:
        run_cpu_jobs(cpu_jobs, cpu_reuse, parity_jobs, args)
        rf = main_res["roofline"]
        res = {
            "metric": METRIC,
            "value": main_res["value"],
            "unit": main_res["unit"],
            "n_gpus": world,
            "steps": args.steps,
            "warmup": W0,
            "ms_per_step": main_res["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: per-(instance, channel) xorshift32 noise (SURVEY 8d seeds) in a device pool; "
                    "per-instance params hashed from the global instance index",
            "config": {k: main_res["config"][k] for k in ("workload", "instances_per_gpu", "instances_total", "block",
                                                          "parallelism") if k in main_res["config"]},
            "frames": main_res["frames"],
            "ranks_reporting": main_res["ranks_reporting"],
            "reps": {"n": R, "warmup_between": Wr, "leg_order": "rotated by one leg per repetition" if m > 1 else "one leg",
                     "kernel_ms": [_r(v) for v in main_res["reps"]["kernel_ms"]],
                     "kernel_spread": _r(main_res["reps"]["kernel_spread"], 3)},
        }
        if rf is not None:
            keep = ("bound", "achieved", "peak", "unit", "frac", "traffic", "achieved_read", "frac_read", "kernel",
                    "kernel_ms", "algorithmic_bytes_per_frame", "algorithmic_read_bytes_per_frame",
                    "frames_per_launch", "frac_read_measured")
            res["roofline"] = {k: (_r(rf[k], 5) if isinstance(rf[k], float) else rf[k]) for k in keep if k in rf}
        else:
            res["roofline"] = None
        cb = main_res.get("cpu_baseline")
        res["cpu_baseline"] = ({k: (_r(v) if isinstance(v, float) else v) for k, v in cb.items()
                                if k not in ("sample_O0",)} if cb else None)
        res["parity"] = _compact_parity(main_res.get("parity"))
        res["output_checksum"] = main_res["output_checksum"]
        if "mix" in main_res:
            res["mix"] = main_res["mix"]
        if box:
            res["box"] = box
        full = dict(res, roofline=rf, cpu_baseline=cb, parity=main_res.get("parity"))
        if world == 1 and args.cpu_seconds > 0 and args.workload == "chorus" and not args.stub:
            c1 = cpu_c1(args.sample_rate, args.block)
            full["cpu_c1"] = c1
            res["cpu_c1"] = {"value": _r(c1["value"]), "value_O0": _r(c1["value_O0"]), "cores": 1, "kind": "port"}
        if also_res:
            full["also"] = also_res
            res["also"] = {k: compact_leg(v) for k, v in also_res.items()}
            res["all_parity_ok"] = all((v.get("parity") or {}).get("ok", False) for v in
                                       [main_res] + list(also_res.values())) if not (args.no_parity or args.stub) else None
        if args.full_json:
            try:
                os.makedirs(os.path.dirname(args.full_json), exist_ok=True)
                with open(args.full_json, "w") as f:
                    json.dump(full, f, indent=1, default=str)
                res["full_json"] = os.path.relpath(args.full_json, ROOT)
            except OSError:
                pass
        print(json.dumps(res), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
