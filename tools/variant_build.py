#!/usr/bin/env python3
"""Experimental builds of libolfx.so from literal source edits -> build/ab/<name>.so, for same-box
A/B timing (tools/libs_occ.sh, tools/ab.sh with OLFX_LIB).  The kernel sources stay untouched.
Usage: python tools/variant_build.py <name> <file> <old> <new> [<file> <old> <new> ...]
  (<file> relative to ol_dsp_amd/csrc; every <old> must occur; all occurrences are replaced)
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ol_dsp_amd", "csrc")


def main():
    name, edits = sys.argv[1], sys.argv[2:]
    if len(edits) % 3:
        sys.exit("edits come in triples: <file> <old> <new>")
    dst = os.path.join(ROOT, "build", "ab", "src_" + name)
    shutil.rmtree(dst, ignore_errors=True)
    os.makedirs(os.path.join(dst, "ol_dsp_amd"), exist_ok=True)
    shutil.copytree(SRC, os.path.join(dst, "ol_dsp_amd", "csrc"), ignore=shutil.ignore_patterns("obj"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(dst, "include"))
    for k in range(0, len(edits), 3):
        p = os.path.join(dst, "ol_dsp_amd", "csrc", edits[k])
        s = open(p).read()
        if edits[k + 1] not in s:
            sys.exit(f"{edits[k]}: not found: {edits[k + 1]!r}")
        open(p, "w").write(s.replace(edits[k + 1], edits[k + 2]))
    out = os.path.join(ROOT, "build", "ab", name + ".so")
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(dst, "ol_dsp_amd", "csrc"), f"OUT={out}", "-B"], check=True)
    print(out)


if __name__ == "__main__":
    main()
