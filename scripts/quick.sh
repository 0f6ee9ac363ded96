#!/bin/bash
# Iteration pass: GPU parity tests, bench on configs 2 and 3, phase profile.
#   usage (via gpurun): bash scripts/quick.sh <tag> [steps]
TAG=${1:-q}; STEPS=${2:-40}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps $STEPS --cpu-seconds 1 > $OUT/bench2.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config 3 --steps 20 --cpu-seconds 1 > $OUT/bench3.log 2>&1 && \
timeout -k 10 200 python -u scripts/phases.py 2 10000 > $OUT/ph2.jsonl 2> $OUT/ph2.err
rc=$?
tail -2 $OUT/gpu_tests.log
for f in $OUT/bench2.log $OUT/bench3.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d.get('verified_bit_exact_vs_oracle'))" $f; done
exit $rc
