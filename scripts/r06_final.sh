#!/bin/bash
# Round-6 closing evidence of the product build, in two calls:
#   bash scripts/r06_final.sh pmc    fabric traffic by request size per config
#                                    (pmc_fetch_split.sh) as bench.py --pmc-json
#                                    lines, and the SQ issue/wait split of the
#                                    one-wavefront kernel (pmc_sq_r02.sh +
#                                    sq_summary.py, with the build digest)
#   bash scripts/r06_final.sh bench  GPU parity tests, smoke(), the driver's
#                                    command for configs 2-6, the rocprofv3
#                                    kernel-trace stats of the config-2 driver
#                                    command and of the config 2 / 4 / 5 kernels
#                                    alone, config 4's single-catalog latency
#                                    (c4_latency.py) and the served path's
#                                    pieces (pipe_timing.py)
# Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${2:-r06_final}
mkdir -p $OUT
if [ "$1" = pmc ]; then
  bash scripts/pmc_fetch_split.sh "2 3 6 5 4" $OUT/fetch_split || exit 1
  OUT=$OUT python3 - <<'PY' || exit 1
import json, os
out = os.environ["OUT"]
d = json.load(open(out + "/fetch_split/fetch_split.json"))
with open(out + "/pmc_traffic.jsonl", "w") as f:
    for c, v in d.items():
        f.write(json.dumps({"config": int(c), "problems": v["problems"],
                            "hbm_bytes_per_dispatch": v["read_bytes_by_size"] + v["write_bytes"],
                            "fetch_bytes_per_run": v["read_bytes_by_size"], "write_bytes_per_run": v["write_bytes"],
                            "algorithmic_bytes_per_run": v["algorithmic_bytes_per_run"],
                            "traffic_over_algorithmic": v["traffic_over_algorithmic"],
                            "l2_hit_rate": v["l2"]["hit_rate"],
                            "correction": "exact request sizes (scripts/pmc_fetch_split.sh)"}) + "\n")
PY
  cat $OUT/pmc_traffic.jsonl
  rm -rf gpurun_out/sq
  bash scripts/pmc_sq_r02.sh "2 3 6 4" > $OUT/sq.log 2>&1 || exit 1
  python3 scripts/sq_summary.py gpurun_out/sq > $OUT/sq_split.json || exit 1
  head -c 600 $OUT/sq_split.json
  exit 0
fi
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -1 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
cat $OUT/smoke.log
for c in 2 3 4 5 6; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --config $c > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/bench_c$c.json').read().strip().splitlines()[-1]); print('config $c', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'cpu', d['cpu_baseline']['value'], 'frac', d['roofline']['frac'], 't/a', d['roofline']['traffic_over_algorithmic'], 'lat', d['latency']['gpu_ms_median'], d['latency']['cpu_1thread_ms_median'], 'e2e', d.get('end_to_end', {}).get('res_per_s'), 'e2e_dev', d.get('end_to_end_device', {}).get('res_per_s'), 'dev_lower', d.get('end_to_end_device', {}).get('lowering_res_per_s'), 'api', d.get('solve_batch_api', {}).get('res_per_s'), 'exact', d['verified_bit_exact_vs_oracle'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c2 -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-steps 0 > $OUT/trace_c2.json 2> $OUT/trace_c2.err || exit 1
for c in 2 4 5; do
  ks=10; [ $c = 4 ] && ks=4
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace_c$c -o run -- \
    python3 bench.py --config $c --kernel-only --kernel-steps $ks --no-cpu > $OUT/ktrace_c$c.json 2> $OUT/ktrace_c$c.err || exit 1
done
timeout -k 10 300 python -u scripts/c4_latency.py 20 > $OUT/c4_latency.jsonl 2> $OUT/c4_latency.err || exit 1
tail -1 $OUT/c4_latency.jsonl
timeout -k 10 300 python -u scripts/pipe_timing.py 2 10000 > $OUT/pipe_timing.txt 2>&1 || exit 1
echo "closing run done"
