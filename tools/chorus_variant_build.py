#!/usr/bin/env python3
"""Diagnostic builds of the chorus stage from source edits -> build/ab/<name>.so (A/B timing only:
some variants compute wrong audio on purpose).  The kernel sources stay clean.
Usage: python tools/chorus_variant_build.py <name>
  lbs   : stores_and_next issues chunk c+1's plan and line loads BEFORE the ring stores (wrong
          audio: fresh lines lack psv_c and x_{c+1}) -- is the store -> load order in the vector
          memory counter what the next chunk waits for?
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ol_dsp_amd", "csrc")


def edit_lbs(s):
    a = '''        if (FULL) {
            stage_run(psv, kPsvBase);
            coop_store(false, kPsvBase, w0, C);
        }'''
    b = '''        pl = plan_chunk_l<kWin>(lfo0 + (uint64_t)C * lfo_inc, lfo_inc, lfo_off, ps0 + (uint64_t)C * ps_inc,
                                ps_inc, Cn > 0 ? Cn : 4, D, wi, wf, pmaxu, cmaxd, FULL);
        load_lines<PAR ^ 1>(pl, w0 + (uint32_t)C, false);
'''
    assert a in s
    s = s.replace(a, b + a, 1)
    c = '''        pl = plan_chunk_l<kWin>(lfo0 + (uint64_t)C * lfo_inc, lfo_inc, lfo_off, ps0 + (uint64_t)C * ps_inc,
                                ps_inc, Cn > 0 ? Cn : 4, D, wi, wf, pmaxu, cmaxd, FULL);
        // the line loads below read positions the stores above just wrote (other lanes of this
        // wave): vector memory operations of a wave reach the L1/L2 in issue order, as for the
        // v10 chunk-start input store and the loads after it
        load_lines<PAR ^ 1>(pl, w0 + (uint32_t)C, false);'''
    assert c in s
    return s.replace(c, "", 1)


def edit_desync(s):
    # the second wave of each SIMD (odd wave slot, HW_ID bits 3:0) starts about half a chunk late, so
    # the two waves of a SIMD are out of phase (one staging through LDS while the other computes)
    a = "    Stage st;\n    st.init(a, lds + wib * Stage::kRegion, lane, inst0);"
    assert a in s
    b = ("    if (__builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11)) & 1u) {\n"
         "        __builtin_amdgcn_s_sleep(127);\n        __builtin_amdgcn_s_sleep(40);\n    }\n")
    return s.replace(a, b + a, 1)


EDITS = {"lbs": ("chorus_stage_l.h", edit_lbs), "desync": ("chorus.hip", edit_desync)}


def main():
    name = sys.argv[1]
    fname, fn = EDITS[name]
    dst = os.path.join(ROOT, "build", "ab", "src_" + name)
    shutil.rmtree(dst, ignore_errors=True)
    os.makedirs(os.path.join(dst, "ol_dsp_amd"), exist_ok=True)
    shutil.copytree(SRC, os.path.join(dst, "ol_dsp_amd", "csrc"), ignore=shutil.ignore_patterns("obj"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(dst, "include"))
    p = os.path.join(dst, "ol_dsp_amd", "csrc", fname)
    src = open(p).read()
    open(p, "w").write(fn(src))
    out = os.path.join(ROOT, "build", "ab", name + ".so")
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(dst, "ol_dsp_amd", "csrc"), f"OUT={out}", "-B"], check=True)
    print(out)


if __name__ == "__main__":
    main()
