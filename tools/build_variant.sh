#!/usr/bin/env bash
# tools/build_variant.sh -- build libolfx.so from a git revision (or the working tree, rev "wt")
# with extra flags into build/ab/<name>.so, for A/B timing on the GPU box (tools/ab.sh).
# Usage: bash tools/build_variant.sh <name> <rev|wt> [EXTRA flags...]
set -eu
name=$1; rev=$2; shift 2
root=$(git rev-parse --show-toplevel)
dst=$root/build/ab/src_$name
rm -rf "$dst"; mkdir -p "$dst/ol_dsp_amd/csrc" "$dst/include"
if [ "$rev" = wt ]; then
  find "$root"/ol_dsp_amd/csrc -maxdepth 1 -type f -exec cp {} "$dst/ol_dsp_amd/csrc/" \; ; cp "$root"/include/* "$dst/include/"
else
  git -C "$root" archive "$rev" ol_dsp_amd/csrc include | tar -x -C "$dst"
fi
make -s -j8 -C "$dst/ol_dsp_amd/csrc" OUT="$root/build/ab/$name.so" EXTRA="$*" -B 2>&1 | grep -v warning || true
ls -la "$root/build/ab/$name.so"
