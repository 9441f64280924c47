#!/bin/bash
# Development tool: build an A/B variant of libwxalign.so into build/ (parallel shards, as
# whisperx_amd._lib.build).  Usage: tools/build_variant.sh NAME [extra hipcc flags...]
# (e.g. -DWX_DEV_V32 -DWX_PHASE_TIMING; a phase-timing build compiles the DP as one TU)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p "$ROOT/build"
cd "$ROOT" && python3 -c "import sys; from whisperx_amd import _lib; _lib.build(force=True, out=sys.argv[1], flags=sys.argv[2:])" \
  "$ROOT/build/$NAME.so" "$@"
