#!/bin/bash
# Round-6 GPU call: parity tests, smoke(), the driver's command for the given
# configs, config 4's single-catalog latency (scripts/c4_latency.py) and the
# rocprofv3 kernel-trace stats of the config 2 and 4 kernels alone.
#   bash scripts/r06_gpu.sh TAG [tests|notests] [configs...]
# Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
MODE=$1; shift
CONFIGS=${*:-2 4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$MODE" = tests ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -1 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit 1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
  cat $OUT/smoke.log
fi
for c in $CONFIGS; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --config $c > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/bench_c$c.json').read().strip().splitlines()[-1]); print('config $c', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'frac', d['roofline']['frac'], 'lat', d['latency']['gpu_ms_median'], d['latency']['cpu_1thread_ms_median'], 'e2e', d.get('end_to_end', {}).get('res_per_s'), 'api', d.get('solve_batch_api', {}).get('res_per_s'), 'place', d['config'].get('placements'), 'h2d/step', d['pcie']['h2d_bytes_per_step'], 'exact', d['verified_bit_exact_vs_oracle'])"
done
if [[ " $CONFIGS " == *" 4 "* ]]; then
  timeout -k 10 300 python -u scripts/c4_latency.py 20 > $OUT/c4_latency.jsonl 2> $OUT/c4_latency.err || exit 1
  tail -1 $OUT/c4_latency.jsonl
fi
for c in $CONFIGS; do
  ks=10; [ $c = 4 ] && ks=4
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace_c$c -o run -- \
    python3 bench.py --config $c --kernel-only --kernel-steps $ks --no-cpu > $OUT/ktrace_c$c.json 2> $OUT/ktrace_c$c.err || exit 1
done
echo "r06 gpu call done"
