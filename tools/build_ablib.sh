#!/bin/bash
# An A/B build of libnc_gpuhash.so with extra -D flags, into abl/<name>.so
# (git-ignored, travels with gpurun), from a copy of the current sources:
#   tools/build_ablib.sh NAME "-DFOO=1 -DBAR=0"
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; DEFS=${2:-}
W=$(mktemp -d /tmp/ablXXXX)
mkdir -p "$W/twemproxy_amd"
cp -r "$ROOT/twemproxy_amd/csrc" "$W/twemproxy_amd/" && rm -rf "$W/twemproxy_amd/csrc/build"
cp -r "$ROOT/include" "$W/"
make -s -C "$W/twemproxy_amd/csrc" -j8 \
    HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$W/include -I$W/twemproxy_amd/csrc -Wall -Wno-unused-function $DEFS" \
    "$W/twemproxy_amd/csrc/../libnc_gpuhash.so" 2>&1 | grep -i " error" || true
mkdir -p "$ROOT/abl"
cp "$W/twemproxy_amd/libnc_gpuhash.so" "$ROOT/abl/$NAME.so"
rm -rf "$W"
echo "abl/$NAME.so"
