#!/bin/bash
# PMC passes over one satbench case (development tool).  Usage: tools/pmc.sh CASE OUTDIR [LIB]
# One rocprofv3 --pmc run per counter group (rocprofv3 does not split groups over passes).
set -e
CASE=${1:-sat3000}; OUT=${2:-gpurun_out/pmc}; LIB=${3:-}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/$OUT"
[ -n "$LIB" ] && export WX_LIB_PATH=$(readlink -f "$LIB")
cd /tmp && export TMPDIR=/tmp
i=0
while read -r G; do
  [ -z "$G" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --kernel-include-regex align_dp_kernel --output-format csv \
      -d "$R/$OUT/p$i" -o p -- python3 "$R/tools/satbench.py" --child --cases "$CASE" --steps 3 > "$R/$OUT/p$i.log" 2>&1
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS
SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA
SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_VALU_ADD_F32 SQ_INSTS_BRANCH SQ_CYCLES SQ_LEVEL_WAVES
GROUPS
