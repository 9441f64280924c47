set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_gputests.log 2>&1 || { tail -40 gpurun_out/r4_gputests.log; exit 1; }
tail -3 gpurun_out/r4_gputests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench.log 2>&1 || { tail -20 gpurun_out/r4_bench.log; exit 1; }
tail -1 gpurun_out/r4_bench.log | cut -c1-3000
for i in 1 2; do timeout -k 10 180 python tools/legs.py e2e --steps 5 --warmup 2 2>&1 | tail -1; done
