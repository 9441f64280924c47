#!/bin/bash
# Round profiles on the GPU box (development tool): kernel stats of the bench step, two PMC
# passes (FETCH_SIZE / WRITE_SIZE) for the headline kernel, then the bench line that reads
# the traffic file.  Usage: tools/profile_round.sh ROUND (e.g. r1).  Outputs: gpurun_out/prof_ROUND/
set -e
RND=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/prof_$RND
mkdir -p "$O"
KSUB=$(cd "$R" && python3 -c "from whisperx_amd import _lib; n=_lib.align_dp_plan(64,300,500,32)[0]; print(n.split('(')[0].replace('void ',''))")
echo "headline kernel: $KSUB"
CMD="python3 bench.py --no-cpu --no-e2e --no-scale --steps 10"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o prof -- python3 "$R/bench.py" --no-cpu --no-e2e --no-scale --steps 50 > "$O/stats.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex align_dp --output-format csv -d "$O/fetch" -o p -- python3 "$R/bench.py" --no-cpu --no-e2e --no-scale --steps 10 > "$O/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex align_dp --output-format csv -d "$O/write" -o p -- python3 "$R/bench.py" --no-cpu --no-e2e --no-scale --steps 10 > "$O/write.log" 2>&1
cd "$R"
python3 tools/traffic_summary.py "$O/fetch" "$O/write" "$KSUB" "$O/${RND}_pmc_traffic.json" "rocprofv3 --pmc FETCH_SIZE (pass 1) / --pmc WRITE_SIZE (pass 2) -- $CMD"
cp "$O/${RND}_pmc_traffic.json" "$R/profiles/${RND}_pmc_traffic.json"
find "$O/stats" -name "*kernel_stats.csv" -exec cp {} "$O/${RND}_rocprof_kernel_stats.csv" \;
timeout -k 10 600 python3 bench.py > "$O/${RND}_bench.log" 2>&1
tail -1 "$O/${RND}_bench.log" > "$O/${RND}_bench.json"
cat "$O/${RND}_bench.json"
