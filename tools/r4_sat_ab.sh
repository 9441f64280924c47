#!/bin/bash
# A/B of saturated-kernel variants (development tool): per variant library build/libt_<v>.so,
# rocprof kernel stats of tools/legs.py sat3000 and one PMC pass for the effective clock
# (GRBM_GUI_ACTIVE / 8 / duration) and the VALU instruction count.
set -o pipefail
export TMPDIR=/tmp
for v in "$@"; do
  WX_LIB_PATH=build/libt_$v.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sat_$v -o sat -- \
    python tools/legs.py sat3000 --steps 5 --warmup 2 > gpurun_out/sat_$v.log 2>&1 || { tail -5 gpurun_out/sat_$v.log; exit 1; }
  grep "sat3000:" gpurun_out/sat_$v.log
  WX_LIB_PATH=build/libt_$v.so timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv \
    -d gpurun_out/satpmc_$v -o pmc -- python tools/legs.py sat3000 --steps 2 --warmup 1 > gpurun_out/satpmc_$v.log 2>&1 \
    || { tail -5 gpurun_out/satpmc_$v.log; exit 1; }
  python tools/pmcsum.py gpurun_out/satpmc_$v align_dp_kernel
  find gpurun_out/sat_$v -name "*kernel_stats.csv" -exec grep -h align_dp {} \; | cut -c1-160
done
find gpurun_out -name "*kernel_trace.csv" -delete
