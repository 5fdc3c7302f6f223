#!/bin/bash
# Build the current csrc tree (or a given source dir) into an A/B library
#   bash profiles/build_variant.sh <name> [src_dir] [-- EXTRA hipcc flags]
# -> voxelraymarcher_amd/ab/libvr_<name>.so  (compare with profiles/ab_probe.py)
set -eu
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/voxelraymarcher_amd/csrc
if [ $# -gt 0 ] && [ "$1" != "--" ]; then SRC=$1; shift; fi
[ $# -gt 0 ] && [ "$1" == "--" ] && shift
EXTRA="$*"
T=$(mktemp -d /tmp/vr_variant.XXXX)
mkdir -p "$T/pkg"
cp -r "$SRC" "$T/pkg/csrc"
rm -rf "$T/pkg/csrc/build"
ln -s "$ROOT/include" "$T/include"
make -s -C "$T/pkg/csrc" ../libvr.so INC="$T/include" EXTRA="$EXTRA" > "$T/build.log" 2>&1 || { cat "$T/build.log"; exit 1; }
mkdir -p "$ROOT/voxelraymarcher_amd/ab"
cp "$T/pkg/libvr.so" "$ROOT/voxelraymarcher_amd/ab/libvr_$NAME.so"
rm -rf "$T"
echo "built voxelraymarcher_amd/ab/libvr_$NAME.so"
