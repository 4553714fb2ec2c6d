#!/usr/bin/env python3
"""Diagnostic builds of the fused chain from source edits -> build/ab/chain_<name>.so (A/B timing
only: the variants compute wrong audio on purpose).  The kernel sources stay clean.
Usage: python tools/chain_variant_build.py <name>
  nodt : the reverb role skips its network (outputs its input): the pipeline at the C and P roles' pace
  nop  : the pitch role skips its stage (passes its input on): is P on the critical path?
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
    return s.replace(a, "                for (int k = 0; k < kChunk; ++k) y[k] = x[k];", 1)


EDITS = {"nodt": ("chain.hip", edit_nodt), "nop": ("chain.hip", edit_nop)}


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
