#!/bin/bash
# Device lowering (dp_lower_device): its parity tests first, then the whole
# GPU suite, then the driver's command for the given configs (the line's
# end_to_end_device leg) and the rocprofv3 kernel-trace stats of the
# config-2 device lowering.
#   bash scripts/r06_dlower.sh TAG [configs...]
# Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
CONFIGS=${*:-2 3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_device_lowering.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $OUT/dl_tests.log 2>&1
rc=$?; tail -12 $OUT/dl_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -1 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit 1
for c in $CONFIGS; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --config $c > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/bench_c$c.json').read().strip().splitlines()[-1]); print('config $c', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'e2e', d['end_to_end']['res_per_s'], 'e2e_dev', d['end_to_end_device'], 'api', d['solve_batch_api']['res_per_s'], 'host_lower', d['host_lowering_res_per_s'], 'exact', d['verified_bit_exact_vs_oracle'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dtrace_c2 -o run -- \
  python3 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu --e2e-steps 5 --kernel-steps 0 > $OUT/dtrace_c2.json 2> $OUT/dtrace_c2.err || exit 1
echo "dlower call done"
