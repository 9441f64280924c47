#!/bin/bash
# Round-3 profiles on the GPU box (development tool): tools/profile_round2.sh's legs (kernel
# stats + FETCH_SIZE / WRITE_SIZE / SQ passes), the VAD producer's kernel stats over 1 h, then
# the end-to-end align() leg's kernel stats, then the default bench line.  Usage: tools/profile_round3.sh ROUND
set -o pipefail
RND=${1:-r3}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$R/tools/profile_round2.sh" "$RND" cfg2 sat3000 trellis3000 || exit 1
O=$R/gpurun_out/prof_$RND/vad1h
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o prof -- python3 "$R/tools/legs.py" vad1h --steps 3 > "$O/stats.log" 2>&1 || { echo "vad1h stats failed"; tail -5 "$O/stats.log"; exit 1; }
grep "ms per launch" "$O/stats.log"
O2=$R/gpurun_out/prof_$RND/e2e
mkdir -p "$O2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O2/stats" -o prof -- python3 "$R/tools/legs.py" e2e --steps 3 > "$O2/stats.log" 2>&1 || { echo "e2e stats failed"; tail -5 "$O2/stats.log"; exit 1; }
grep "ms per launch" "$O2/stats.log"
# condense on the box (gpurun brings back <= 64 MiB of gpurun_out/): summaries into
# gpurun_out/profiles_$RND/, the raw traces deleted
cd "$R" && python3 tools/summarize_profiles.py "$RND" > "gpurun_out/summarize_$RND.log" 2>&1 || { echo "summarize failed"; tail -20 "gpurun_out/summarize_$RND.log"; exit 1; }
mkdir -p "gpurun_out/profiles_$RND" && cp profiles/${RND}_* "gpurun_out/profiles_$RND/"
find "$O/stats" -name "*kernel_stats.csv" -exec cp {} "gpurun_out/profiles_$RND/${RND}_vad1h_kernel_stats.csv" \;
find "$O2/stats" -name "*kernel_stats.csv" -exec cp {} "gpurun_out/profiles_$RND/${RND}_e2e_kernel_stats.csv" \;
rm -rf "gpurun_out/prof_$RND"
cd "$R" && timeout -k 10 600 python3 bench.py > "gpurun_out/${RND}_bench.log" 2>&1 || { echo "bench failed"; tail -20 "gpurun_out/${RND}_bench.log"; exit 1; }
tail -n 1 "gpurun_out/${RND}_bench.log" | cut -c1-400
