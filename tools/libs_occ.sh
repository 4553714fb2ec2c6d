#!/usr/bin/env bash
# tools/libs_occ.sh -- kernel time against instances (tools/occ_scale.sh) for several builds of
# libolfx.so on one box.  Usage: bash tools/libs_occ.sh "<workloads>" "<instance counts>" <lib>...
# (lib paths relative to the repo root; "main" = ol_dsp_amd/libolfx.so)
set -u
w=$1; ns=$2; shift 2
for lib in "$@"; do
  [ "$lib" = main ] && lib=ol_dsp_amd/libolfx.so
  echo "## $lib"
  OLFX_LIB=$PWD/$lib bash tools/occ_scale.sh "$w" "$ns" || exit 1
done
