#!/usr/bin/env python3
"""Diagnostic builds of the fused chain from source edits -> build/ab/chain_<name>.so (A/B timing
only: the variants compute wrong audio on purpose).  The kernel sources stay clean.
Usage: python tools/chain_variant_build.py <name>
  nodt : the reverb role skips its network (outputs its input): the pipeline at the C and P roles' pace
  nop  : the pitch role skips its stage (passes its input on): is P on the critical path?
  v6 (chain_block_v6, round 6; the edits also reach dattorro_block_v5 in that build):
  notank : the tank halves skip their taps, arithmetic and ring writes (partials = x, outputs x)
  nodi   : the DI role skips its taps and ring writes (x = its input)
  noc    : the chorus roles skip their stage (zeros on)
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ol_dsp_amd", "csrc")


def edit_nodt(s):
    a = "                    dt_step(T + s, f0 + s + 4 < nf, xin, o_l, o_r);"
    assert a in s
    return s.replace(a, "                    for (int k = 0; k < 4; ++k) { o_l[k] = xin[k]; o_r[k] = xin[k]; }", 1)


def edit_nop(s):
    a = "                sp.template chunk<P>(x, C, Cn, [&](int k, float2 v) { y[k] = v; });"
    assert a in s
    return s.replace(a, "                for (int k = 0; k < kChunk; ++k) y[k] = x[k];")


def edit_notank(s):
    a = s.index("        SPLIT_TAPS(SPLIT_PREFETCH)\n        ap1.prefetch(a, t, i);\n        ap1.resolve();\n")
    s = s[:a] + s[a:].replace("        SPLIT_TAPS(SPLIT_PREFETCH)\n        ap1.prefetch(a, t, i);\n        ap1.resolve();\n", "", 1)
    b = s.index("            float y = x[k] + fb.get(k) * g_decay;")
    e = s.index("            n5[k] = t5.get(k); n6[k] = t6.get(k); n7[k] = t7.get(k);")
    s = s[:b] + "            pm[k] = x[k]; n5[k] = 0.f; n6[k] = 0.f; n7[k] = 0.f;\n" + s[e + len("            n5[k] = t5.get(k); n6[k] = t6.get(k); n7[k] = t7.get(k);"):]
    for r in ("kAP1", "kDL1", "kAP2", "kDL2"):
        line = f"        *grpu<Hf::{r}>(a, gw, i) = f4(w_{r[1:].lower()});\n"
        assert line in s, line
        s = s.replace(line, "", 1)
    return s


def edit_nodi(s):
    a = "                    dt::di_compute(xpd, lp_pre, g_pre, g_in1, g_in2, in0, in1, in2, in3, w0, w1, w2, w3, xo);"
    assert a in s
    s = s.replace(a, "                    for (int k = 0; k < 4; ++k) xo[k] = xin[k];", 1)
    for l in ("IN0", "IN1", "IN2", "IN3"):
        line = f"                    *dt::grpu<DT_{l}>(d, gw, i) = dt::f4(w{l[-1]});\n"
        assert line in s, line
        s = s.replace(line, "", 1)
    b = "                    in0.prefetch(d, t, i); in1.prefetch(d, t, i); in2.prefetch(d, t, i); in3.prefetch(d, t, i);\n"
    assert b in s
    return s.replace(b, "", 1)


def edit_noc(s):
    a = s.index("__global__ __launch_bounds__(kChain6Threads, 1) void chain_block_v6")
    c = "                s1.template chunk<decltype(par)::value>(x, xn, C, Cn, [&](int k, float v) { y[k] = v; }, prefetch, xq);"
    assert c in s[a:]
    return s[:a] + s[a:].replace(c, "                for (int k = 0; k < kChunk; ++k) y[k] = 0.f;", 1)


EDITS = {"nodt": ("chain.hip", edit_nodt), "nop": ("chain.hip", edit_nop), "notank": ("dattorro_stage.h", edit_notank),
         "nodi": ("chain.hip", edit_nodi), "noc": ("chain.hip", edit_noc)}


def main():
    name = sys.argv[1]
    fname, fn = EDITS[name]
    dst = os.path.join(ROOT, "build", "ab", "src_chain_" + name)
    shutil.rmtree(dst, ignore_errors=True)
    os.makedirs(os.path.join(dst, "ol_dsp_amd"), exist_ok=True)
    shutil.copytree(SRC, os.path.join(dst, "ol_dsp_amd", "csrc"), ignore=shutil.ignore_patterns("obj"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(dst, "include"))
    p = os.path.join(dst, "ol_dsp_amd", "csrc", fname)
    src = open(p).read()
    open(p, "w").write(fn(src))
    out = os.path.join(ROOT, "build", "ab", "chain_" + name + ".so")
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(dst, "ol_dsp_amd", "csrc"), f"OUT={out}", "-B"], check=True)
    print(out)


if __name__ == "__main__":
    main()
