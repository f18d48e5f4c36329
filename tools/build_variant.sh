#!/usr/bin/env bash
# Build an experiment library from the working tree with some source files replaced:
#   tools/build_variant.sh NAME [csrc_file=replacement_path ...]  ->  variants/NAME.so
set -euo pipefail
root=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
d=/tmp/var_$name
rm -rf "$d" && mkdir -p "$d/thor-slam_amd" "$d/include"
cp -r "$root/thor-slam_amd/csrc" "$d/thor-slam_amd/" && rm -rf "$d/thor-slam_amd/csrc/build"
cp "$root/include/tslam.h" "$d/include/"
for kv in "$@"; do cp "${kv#*=}" "$d/thor-slam_amd/csrc/${kv%%=*}"; done
mkdir -p "$root/variants"
make -s -C "$d/thor-slam_amd/csrc" -j8 OUT="$root/variants/$name.so" 2>&1 | grep -E "error|warning" || true
ls -la "$root/variants/$name.so"
