set -o pipefail
timeout -k 10 250 python tools/satbench.py --libs build/libt_p4.so,build/libt_ov1.so,build/libt_p4.so,build/libt_ov1.so --cases b64,b16,rag64 --steps 20 > gpurun_out/r4ov1.log 2>&1; cat gpurun_out/r4ov1.log
