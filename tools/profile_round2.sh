#!/bin/bash
# Round profiles on the GPU box (development tool).  Per leg (cfg2 = the bench headline,
# sat3000 = saturated fused DP, trellis3000 = materialised get_trellis): a rocprofv3 kernel
# trace with stats, then separate PMC passes (FETCH_SIZE; WRITE_SIZE; SQ busy/VALU counters).
# Usage: tools/profile_round2.sh ROUND LEG...   Outputs: gpurun_out/prof_ROUND/LEG/
set -o pipefail
RND=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for LEG in "$@"; do
  O=$R/gpurun_out/prof_$RND/$LEG
  mkdir -p "$O"
  case $LEG in trellis3000) RX=trellis_kernel ;; *) RX=align_dp ;; esac
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o prof -- python3 "$R/tools/legs.py" $LEG --steps 20 > "$O/stats.log" 2>&1 || { echo "$LEG stats failed"; tail -5 "$O/stats.log"; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $RX --output-format csv -d "$O/fetch" -o p -- python3 "$R/tools/legs.py" $LEG --steps 5 > "$O/fetch.log" 2>&1 || { echo "$LEG fetch failed"; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $RX --output-format csv -d "$O/write" -o p -- python3 "$R/tools/legs.py" $LEG --steps 5 > "$O/write.log" 2>&1 || { echo "$LEG write failed"; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM --kernel-include-regex $RX --output-format csv -d "$O/sq" -o p -- python3 "$R/tools/legs.py" $LEG --steps 5 > "$O/sq.log" 2>&1 || { echo "$LEG sq failed"; exit 1; }
  grep "ms per launch" "$O/stats.log"
done
