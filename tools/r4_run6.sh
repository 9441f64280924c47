set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_vad_producer.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_vadtests.log 2>&1 || { tail -40 gpurun_out/r4_vadtests.log; exit 1; }
tail -3 gpurun_out/r4_vadtests.log
for e in "X=1" "WX_NO_SHARED_SINC=1" "X=1"; do env $e timeout -k 10 180 python tools/legs.py vad1h --steps 5 --warmup 1 2>&1 | tail -1 | sed "s/^/$e /"; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gputests.log 2>&1 || { tail -40 gpurun_out/r4_gputests.log; exit 1; }
tail -2 gpurun_out/r4_gputests.log
