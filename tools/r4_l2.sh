set -o pipefail
R=$(pwd)
timeout -k 10 200 python tools/satbench.py --libs build/libt_p4.so,build/libt_l2.so,build/libt_p4.so,build/libt_l2.so --cases b64,b16,rag64 --steps 20 > gpurun_out/r4l2.log 2>&1; cat gpurun_out/r4l2.log
for v in p4 l2; do
  WX_LIB_PATH=$R/build/libt_$v.so bash tools/profile_round2.sh l2$v cfg2 > gpurun_out/l2$v.log 2>&1 || { tail gpurun_out/l2$v.log; exit 1; }
  python tools/pmcsum.py gpurun_out/prof_l2$v/cfg2/fetch align_dp | sed "s/^/$v fetch /"
  python tools/pmcsum.py gpurun_out/prof_l2$v/cfg2/write align_dp | sed "s/^/$v write /"
done
rm -rf gpurun_out/prof_l2p4 gpurun_out/prof_l2l2
