set -o pipefail
timeout -k 10 600 python bench.py > gpurun_out/r4_bench_final.log 2>&1 || { tail -20 gpurun_out/r4_bench_final.log; exit 1; }
tail -1 gpurun_out/r4_bench_final.log > gpurun_out/r4_bench_final.json
python -c "import json; d=json.load(open('gpurun_out/r4_bench_final.json')); print(d['ms_per_step'], d['roofline']['avg_launch_us']); [print(k, {kk: vv for kk, vv in v.items() if not isinstance(vv, (dict, list))} if isinstance(v, dict) else v) for k, v in d['extra'].items()]" | cut -c1-400
