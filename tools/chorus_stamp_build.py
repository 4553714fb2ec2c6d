#!/usr/bin/env python3
"""Diagnostic build: chorus_block_v11 with per-phase cycle stamps (s_memtime) -> build/ab/chstamp.so.

The kernel sources stay clean: this copies ol_dsp_amd/csrc to build/ab/src_chstamp, inserts the
stamps at fixed anchors of chorus_stage_l.h / chorus.hip, and builds.  Each wave accumulates, per
phase of the chunk, the cycles between consecutive stamps; at the end its first instance's channel-0
output rows 0..NPH-1 hold the sums (the audio is garbage in this build).  A stamp is an SMEM read
with an lgkmcnt wait, so it also drains the wave's LDS operations at that point: read the phase
split as "where each wave's time goes", not as an exact profile.  tools/chorus_stamps.py reads it.
Usage: python tools/chorus_stamp_build.py
"""
import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ol_dsp_amd", "csrc")
DST = os.path.join(ROOT, "build", "ab", "src_chstamp")
OUT = os.path.join(ROOT, "build", "ab", "chstamp.so")

PHASES = ["loop", "stageC", "stageAB", "prefetch", "pitch", "psvwin", "st_psv", "chorus", "out", "st_x", "st_plan",
          "st_lines"]


def stamp(k):
    return ("{ const uint64_t st_t = __builtin_amdgcn_s_memtime(); st_acc[%d] += st_t - st_last; "
            "st_last = st_t; }\n        " % k)


def main():
    shutil.rmtree(DST, ignore_errors=True)
    os.makedirs(os.path.join(DST, "ol_dsp_amd"), exist_ok=True)
    shutil.copytree(SRC, os.path.join(DST, "ol_dsp_amd", "csrc"), ignore=shutil.ignore_patterns("obj"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(DST, "include"))
    p = os.path.join(DST, "ol_dsp_amd", "csrc", "chorus_stage_l.h")
    s = open(p).read()
    ins = [("        // tap C first: psv_{c-1}", 0),
           ("        stage_tap<PAR, 0>();\n        stage_tap<PAR, 1>();", 1),
           ("        started = true;", 2),
           ("        const bool fast = C == kChunk && __all(cur.okA && cur.okB);", 3),
           ("            if (FULL) {\n#pragma unroll\n                for (int k = 0; k < kChunk; ++k) wC[min(k - cur.sC, kWin) * kRow] = psv[k];", 4),
           ("        stores_and_next<PAR>(psv, x, xn, xq, w0, C, Cn, lfo0, ps0);", 5),
           ("        if (fast) {\n            // C. the chorus tap", 6),
           ("        wpos = w0 + (uint32_t)C;", 7)]
    # inside stores_and_next: psv -> ring (6), x rows -> ring + own frames (9), plan (10), line loads (11)
    ins += [("        if (COOP) {                              // x_{c+1}: rows -> staging -> ring and lanes", 6),
            ("        pl = plan_chunk_l<kWin>(lfo0 + (uint64_t)C * lfo_inc", 9),
            ("        load_lines<PAR ^ 1>(pl, w0 + (uint32_t)C, false);\n    }", 10)]
    for anchor, k in ins:
        assert anchor in s, anchor
        if k == 10:      # after the line loads: stamp 11 too
            s = s.replace(anchor, stamp(k) + anchor.replace("\n    }", "\n        " + stamp(11).rstrip() + "\n    }"), 1)
        else:
            s = s.replace(anchor, stamp(k) + anchor, 1)
    s = s.replace("    PlanL pl;\n    uint32_t wpos;", "    PlanL pl;\n    uint64_t st_acc[%d], st_last;\n    uint32_t wpos;" % len(PHASES), 1)
    s = s.replace("        strag_slot = kWin;\n    }", "        strag_slot = kWin;\n        for (int q = 0; q < %d; ++q) st_acc[q] = 0;\n"
                  "        st_last = __builtin_amdgcn_s_memtime();\n    }" % len(PHASES), 1)
    open(p, "w").write(s)
    p = os.path.join(DST, "ol_dsp_amd", "csrc", "chorus.hip")
    s = open(p).read()
    anchor = "#pragma unroll\n        for (int k = 0; k < kChunk; ++k) x[k] = xn[k];\n    };"
    assert anchor in s
    s = s.replace(anchor, "        { const uint64_t st_t = __builtin_amdgcn_s_memtime(); st.st_acc[8] += st_t - st.st_last; st.st_last = st_t; }\n" + anchor, 1)
    anchor = "    st.finish(a);\n}"
    assert anchor in s
    s = s.replace(anchor, "    st.finish(a);\n    if (lane == 0)\n        for (int q = 0; q < %d; ++q) a.out[(size_t)q * a.n + inst0] = (float)st.st_acc[q];\n}" % len(PHASES), 1)
    open(p, "w").write(s)
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(DST, "ol_dsp_amd", "csrc"), f"OUT={OUT}", "-B"], check=True)
    print(OUT)


if __name__ == "__main__":
    main()
