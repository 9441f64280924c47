set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_gputests.log 2>&1 || { tail -40 gpurun_out/r4_gputests.log; exit 1; }
tail -2 gpurun_out/r4_gputests.log
for e in "X=1" "WX_NO_ADDLN=1" "X=1" "WX_NO_ADDLN=1"; do env $e timeout -k 10 180 python tools/legs.py e2e --steps 5 --warmup 2 2>&1 | tail -1 | sed "s/^/$e /"; done
timeout -k 10 200 python tools/satbench.py --libs build/libt_p4.so,build/libt_cs.so,build/libt_ts.so,build/libt_p4.so,build/libt_cs.so,build/libt_ts.so --cases b64,b16,b64p2,sat1499 --steps 20 > gpurun_out/r4cs.log 2>&1; cat gpurun_out/r4cs.log
timeout -k 10 300 python tools/satbench.py --libs build/libph_cs.so,build/libph_ts.so --cases b64 --phases --parts 4 --steps 20 > gpurun_out/r4cs_ph.log 2>&1; grep -E "b64 |exit_max|seg_exit|walk_" gpurun_out/r4cs_ph.log
