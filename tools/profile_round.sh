#!/bin/bash
# Round profiles and kernel A/Bs on the GPU box (development tool; replaces the round-specific
# profile_round2.sh / profile_round3.sh / r4_bench.sh / r4_sat_ab.sh).
#
#   tools/profile_round.sh profile ROUND [LEG...]
#       per DP leg (default: cfg2 sat3000 trellis3000; cfg2 = the bench headline, sat3000 = the
#       saturated fused DP, trellis3000 = materialised get_trellis): a rocprofv3 kernel trace with
#       stats, then separate PMC passes (FETCH_SIZE; WRITE_SIZE; SQ busy / VALU counters: one
#       counter group per run, rocprofv3 does not split groups); then the kernel stats of the VAD
#       producer over 1 h (vad1h) and of align() end to end (e2e); condensed by
#       tools/summarize_profiles.py into gpurun_out/profiles_ROUND/ (raw traces deleted: gpurun
#       brings back <= 64 MiB), and the default bench line into gpurun_out/ROUND_bench.log.
#   tools/profile_round.sh sat-ab VARIANT...
#       saturated-kernel variants built by tools/build_variant.sh (build/libt_VARIANT.so): kernel
#       stats of tools/legs.py sat3000 and one PMC pass for the effective clock
#       (GRBM_GUI_ACTIVE / 8 / duration) and the VALU instruction count.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
MODE=$1; shift
cd /tmp && export TMPDIR=/tmp

dp_legs() {
  local RND=$1; shift
  for LEG in "$@"; do
    local O=$R/gpurun_out/prof_$RND/$LEG RX=align_dp
    mkdir -p "$O"
    [ "$LEG" = trellis3000 ] && RX=trellis_kernel
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o prof -- python3 "$R/tools/legs.py" $LEG --steps 20 > "$O/stats.log" 2>&1 || { echo "$LEG stats failed"; tail -5 "$O/stats.log"; return 1; }
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $RX --output-format csv -d "$O/fetch" -o p -- python3 "$R/tools/legs.py" $LEG --steps 5 > "$O/fetch.log" 2>&1 || { echo "$LEG fetch failed"; return 1; }
    timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $RX --output-format csv -d "$O/write" -o p -- python3 "$R/tools/legs.py" $LEG --steps 5 > "$O/write.log" 2>&1 || { echo "$LEG write failed"; return 1; }
    timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM --kernel-include-regex $RX --output-format csv -d "$O/sq" -o p -- python3 "$R/tools/legs.py" $LEG --steps 5 > "$O/sq.log" 2>&1 || { echo "$LEG sq failed"; return 1; }
    timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_CMD_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --kernel-include-regex $RX --output-format csv -d "$O/lds" -o p -- python3 "$R/tools/legs.py" $LEG --steps 5 > "$O/lds.log" 2>&1 || { echo "$LEG lds failed"; return 1; }
    grep "ms per launch" "$O/stats.log"
  done
}

stats_leg() {  # kernel stats of one tools/legs.py leg into gpurun_out/prof_ROUND/LEG
  local RND=$1 LEG=$2 O=$R/gpurun_out/prof_$1/$2
  mkdir -p "$O"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o prof -- python3 "$R/tools/legs.py" $LEG --steps 3 > "$O/stats.log" 2>&1 || { echo "$LEG stats failed"; tail -5 "$O/stats.log"; return 1; }
  grep "ms per launch" "$O/stats.log"
}

case $MODE in
  profile)
    RND=${1:?round}; shift
    LEGS=${*:-cfg2 cfg5 sat3000 trellis3000}
    dp_legs "$RND" $LEGS || exit 1
    stats_leg "$RND" vad1h || exit 1
    stats_leg "$RND" e2e || exit 1
    stats_leg "$RND" e2e5 || exit 1
    cd "$R" && python3 tools/summarize_profiles.py "$RND" > "gpurun_out/summarize_$RND.log" 2>&1 || { echo "summarize failed"; tail -20 "gpurun_out/summarize_$RND.log"; exit 1; }
    # per-kernel rooflines of the producers from the same kernel traces
    T_VAD=$(find "gpurun_out/prof_$RND/vad1h/stats" -name "*kernel_trace.csv" | head -1)
    [ -n "$T_VAD" ] && python3 tools/vad_roofline.py "$T_VAD" --out "profiles/${RND}_vad_roofline.json" > /dev/null
    T_E2E=$(find "gpurun_out/prof_$RND/e2e/stats" -name "*kernel_trace.csv" | head -1)
    [ -n "$T_E2E" ] && python3 tools/forward_roofline.py "$T_E2E" --out "profiles/${RND}_forward_roofline.json" > /dev/null
    mkdir -p "gpurun_out/profiles_$RND" && cp profiles/${RND}_* "gpurun_out/profiles_$RND/"
    for LEG in vad1h e2e e2e5; do
      find "gpurun_out/prof_$RND/$LEG/stats" -name "*kernel_stats.csv" -exec cp {} "gpurun_out/profiles_$RND/${RND}_${LEG}_kernel_stats.csv" \;
    done
    rm -rf "gpurun_out/prof_$RND"
    timeout -k 10 600 python3 bench.py > "gpurun_out/${RND}_bench.log" 2>&1 || { echo "bench failed"; tail -20 "gpurun_out/${RND}_bench.log"; exit 1; }
    tail -n 1 "gpurun_out/${RND}_bench.log" | cut -c1-400
    ;;
  sat-ab)
    cd "$R"
    for v in "$@"; do
      WX_LIB_PATH=build/libt_$v.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sat_$v -o sat -- \
        python3 tools/legs.py sat3000 --steps 5 --warmup 2 > gpurun_out/sat_$v.log 2>&1 || { tail -5 gpurun_out/sat_$v.log; exit 1; }
      grep "sat3000:" gpurun_out/sat_$v.log
      WX_LIB_PATH=build/libt_$v.so timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv \
        -d gpurun_out/satpmc_$v -o pmc -- python3 tools/legs.py sat3000 --steps 2 --warmup 1 > gpurun_out/satpmc_$v.log 2>&1 \
        || { tail -5 gpurun_out/satpmc_$v.log; exit 1; }
      python3 tools/pmcsum.py gpurun_out/satpmc_$v align_dp_kernel
      find gpurun_out/sat_$v -name "*kernel_stats.csv" -exec grep -h align_dp {} \; | cut -c1-160
    done
    find gpurun_out -name "*kernel_trace.csv" -delete
    ;;
  *) echo "usage: tools/profile_round.sh profile ROUND [LEG...] | sat-ab VARIANT..."; exit 2 ;;
esac
