#!/bin/bash
# Development tool: build an A/B variant of libwxalign.so into build/.
# Usage: tools/build_variant.sh NAME [extra hipcc flags...]   (e.g. -DWX_DEV_V32 -DWX_PHASE_TIMING)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p "$ROOT/build"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math "$@" -I"$ROOT/include" \
  -o "$ROOT/build/$NAME.so" "$ROOT"/whisperx_amd/csrc/wx_align.hip "$ROOT"/whisperx_amd/csrc/wx_emission.hip \
  "$ROOT"/whisperx_amd/csrc/wx_vad.hip
