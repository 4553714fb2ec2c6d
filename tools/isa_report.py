#!/usr/bin/env python3
"""Compile one .hip file for gfx950 with saved temps and report, per kernel: VGPR/AGPR/spills,
instruction mix, and scratch (spill) instructions inside loops.
Usage: python tools/isa_report.py ol_dsp_amd/csrc/chorus.hip [kernel-substring] [-DX=Y ...]"""
import collections, os, re, subprocess, sys, tempfile

src = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-D") else ""
defs = [a for a in sys.argv[2:] if a.startswith("-D")]
sub = "" if sub == "-v" else sub
d = tempfile.mkdtemp()
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                "-fno-gpu-flush-denormals-to-zero", "--save-temps", "-c", os.path.abspath(src), "-o", os.path.join(d, "x.o")] + defs,
               cwd=d, check=True, capture_output=True)
asm = [f for f in os.listdir(d) if f.endswith("gfx950.s")][0]
s = open(os.path.join(d, asm)).read()
for m in re.finditer(r"^(_Z\w+):", s, flags=re.M):
    name = m.group(1)
    if sub not in name or "kd" in name:
        continue
    end = s.find(".Lfunc_end", m.end())
    body = s[m.end():end].split("\n")
    ins, inloop, w0loop = [], 0, 0
    loop = False
    ctx = []
    for l in body:
        t = l.strip()
        if re.match(r"^\.LBB\d+_\d+:", t):
            loop = "in Loop" in t
            continue
        if not t or t.startswith((".", ";")):
            continue
        ins.append(t)
        if "scratch_" in t and loop:
            inloop += 1
            if "-v" in sys.argv:
                print("   loop spill:", t[:90])
        if loop and t.startswith("s_waitcnt") and "vmcnt(0)" in t:
            w0loop += 1
    c = collections.Counter(i.split()[0] for i in ins)
    meta = s[s.find(".name:           " + name):][:2000]
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", meta) or [None, "?"])[1]
    print(f"{name}: vgpr {g('vgpr_count')} agpr {g('agpr_count')} vspill {g('vgpr_spill_count')} sspill {g('sgpr_spill_count')} "
          f"| valu {sum(v for k, v in c.items() if k.startswith('v_'))} lds {sum(v for k, v in c.items() if k.startswith('ds_'))} "
          f"vmem {sum(v for k, v in c.items() if k.startswith(('buffer_', 'global_')))} scratch {sum(v for k, v in c.items() if 'scratch' in k)} "
          f"(in loops {inloop}) vmcnt(0) in loops {w0loop}")
