#!/bin/bash
# Build a whole-library variant for scripts/ab_libs.sh: copies antidote_amd/csrc (reusing its
# objects) to /tmp/amvar_<NAME>/antidote_amd/csrc, overlays the files given as SRC=DST pairs (DST relative to
# csrc; SRC a path or git:<rev>:<path>), adds EXTRA_FLAGS, builds, and installs
# scripts/ab/lib_<NAME>.so.   scripts/build_variant.sh old git:HEAD:antidote_amd/csrc/am_lanes.hip=am_lanes.hip
set -eu
cd "$(dirname "$0")/.."
NAME=$1; shift
W=/tmp/amvar_$NAME
rm -rf $W && mkdir -p $W/antidote_amd/csrc $W/include
cp -a antidote_amd/csrc/. $W/antidote_amd/csrc/
cp -a include/. $W/include/
for pair in "$@"; do
  src=${pair%%=*}; dst=${pair#*=}
  case $src in
    git:*) rev_path=${src#git:}; git show "$rev_path" > $W/antidote_amd/csrc/$dst ;;
    *) cp "$src" $W/antidote_amd/csrc/$dst ;;
  esac
done
# objects are newer than the overlaid sources otherwise; extra flags rebuild everything
for pair in "$@"; do dst=${pair#*=}; touch $W/antidote_amd/csrc/$dst; done
if [ -n "${EXTRA_FLAGS:-}" ]; then touch $W/antidote_amd/csrc/*.hip; fi
make -s -j8 -C $W/antidote_amd/csrc OUT=$W/antidote_amd HIPFLAGS_EXTRA="${EXTRA_FLAGS:-}" >/dev/null
mkdir -p scripts/ab
cp $W/antidote_amd/libantidote_mat.so scripts/ab/lib_$NAME.so
echo "scripts/ab/lib_$NAME.so"
