#!/bin/bash
# Interleaved A/B of environment settings on one box (bench.py host to host
# with the driver's --steps 20 --warmup 5, plus the kernel-only rate):
#   scripts/ab_env.sh <config> <rounds> "<VAR=val ...>" ...   ("-" = none)
set -o pipefail
export TMPDIR=/tmp
CFG=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out/ab
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    envs=""; [ "$v" != "-" ] && envs="$v"
    env $envs timeout -k 10 200 python bench.py --config $CFG --steps 20 --warmup 5 --kernel-steps 30 --no-cpu --e2e-steps 0 > gpurun_out/ab/run.json 2>&1 || { echo "run $v failed"; tail -5 gpurun_out/ab/run.json; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab/run.json').read().strip().splitlines()[-1]); print('[$v]', 'config $CFG', 'h2h', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'serial_ms', d['kernel_only']['serial_launch_ms'])" | tee -a gpurun_out/ab/ab_env_c$CFG.txt
  done
done
