set -o pipefail
timeout -k 10 250 python tools/satbench.py --libs build/libt_p4.so,build/libt_cs.so,build/libt_ts.so,build/libt_p4.so,build/libt_cs.so,build/libt_ts.so --cases rag64,b64,b16,b64p2 --steps 20 > gpurun_out/r4rag.log 2>&1; cat gpurun_out/r4rag.log
