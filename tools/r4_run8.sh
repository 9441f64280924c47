set -o pipefail
timeout -k 10 250 python tools/satbench.py --libs build/libt_p4.so,build/libt_ch.so,build/libt_p4.so,build/libt_ch.so --cases b64,b16,rag64,b64p2 --steps 20 > gpurun_out/r4ch.log 2>&1; cat gpurun_out/r4ch.log
