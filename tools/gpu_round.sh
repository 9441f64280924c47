#!/bin/bash
# GPU-box command chain used during development: gpu tests, default bench, a 2-rank gloo
# rehearsal of the multi-rank bench path.  Each GPU step under its own time limit; stops at
# the first failure.  Usage: tools/gpu_round.sh TAG [tests|bench|multi]...
set -o pipefail
TAG=${1:-x}; shift
O=gpurun_out
mkdir -p $O
steps=("$@")
[ ${#steps[@]} -eq 0 ] && steps=(tests bench)
for step in "${steps[@]}"; do
  case $step in
    tests) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/${TAG}_gputests.log 2>&1 || { echo "tests failed"; tail -30 $O/${TAG}_gputests.log; exit 1; } ; tail -3 $O/${TAG}_gputests.log ;;
    bench) timeout -k 10 600 python bench.py > $O/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -30 $O/${TAG}_bench.log; exit 1; } ; tail -1 $O/${TAG}_bench.log | cut -c1-600 ;;
    multi) WX_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --no-cpu --no-scale --no-e2e > $O/${TAG}_multi.log 2>&1 || { echo "multi failed"; tail -30 $O/${TAG}_multi.log; exit 1; } ; tail -1 $O/${TAG}_multi.log | cut -c1-600 ;;
  esac
done
