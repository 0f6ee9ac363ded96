#!/bin/bash
# Round 5: M_LDSG for latency-bound chunks only (placement.hpp kLdsgMaxProblems):
# GPU tests, config 5 host to host (auto vs never), the largest config-5
# catalogs one at a time, and the bench latency leg of config 5.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r05/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/ldsg_latency.py 20 300 > gpurun_out/r05/ldsg_lat_auto.txt 2>&1 || exit 1
tail -1 gpurun_out/r05/ldsg_lat_auto.txt | cut -c1-400
bash scripts/ab_env.sh 5 2 - DEPPY_LDSG=0 || exit 1
timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 5 --cpu-seconds 3 --e2e-steps 0 > gpurun_out/r05/bench_c5.json 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r05/bench_c5.json').read().strip().splitlines()[-1]); print(d['value'], d['latency'], d.get('verified_bit_exact_vs_oracle'))"
