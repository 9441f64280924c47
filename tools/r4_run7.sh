set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gputests.log 2>&1 || { tail -40 gpurun_out/r4_gputests.log; exit 1; }
tail -2 gpurun_out/r4_gputests.log
timeout -k 10 250 python tools/satbench.py --libs build/libt_p4.so,whisperx_amd/libwxalign.so --cases b64,rag64,sat3000,sat1499 --steps 10 > gpurun_out/r4fin.log 2>&1; cat gpurun_out/r4fin.log
