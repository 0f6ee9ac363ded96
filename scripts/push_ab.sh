#!/bin/bash
# One-wavefront A/B of a kernel change against the previous build, on one box:
# GPU parity tests of the current build; phase stamps of both stamps builds
# (libdeppy_hip_stamps.so vs the variant named by $3) on configs 2 and 6; then
# configs 2, 3 and 6 host to host and kernel only, interleaved twice.
#   usage: bash scripts/push_ab.sh <tag> <release variant lib> <stamps variant lib> [bench]
# ("bench": the bench lines only)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-push_ab}
VAR=${2:-libdeppy_hip_head.so}
SVAR=${3:-libdeppy_hip_stamps_head.so}
mkdir -p $OUT
if [ "$4" != bench ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
for cfg in 2 6; do
  for v in new old; do
    lib=libdeppy_hip_stamps.so; [ $v = old ] && lib=$SVAR
    DEPPY_PHASES_FORM=packed DEPPY_STAMPS_LIB=$lib timeout -k 10 200 python -u scripts/phases.py $cfg 10000 > $OUT/ph_c${cfg}_$v.jsonl 2> $OUT/ph_c${cfg}_$v.err || exit 1
    python3 -c "
import json; d=[json.loads(l) for l in open('$OUT/ph_c${cfg}_$v.jsonl')][-1]; a=d['sat_A']
print('[$v] config $cfg phases: total', a['total_mean'], 'push_guess', a['push_guess'][0], 'push_pre', a['push_pre'][0], 'pushes', a['pushes'][0], 'rounds', a['round_total'][0], 'loop_gap', a['loop_gap'][0])"
  done
done
fi
for rep in 1 2; do
  for cfg in 2 3 6; do
    for v in new old; do
      envs=""; [ $v = old ] && envs="DEPPY_VARIANT_LIB=$VAR"
      env $envs timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 5 --kernel-steps 30 --no-cpu --e2e-steps 0 > $OUT/run.json 2>&1 || exit 1
      python3 -c "import json; d=json.loads(open('$OUT/run.json').read().strip().splitlines()[-1]); print('[$v] config $cfg', 'h2h', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'serial_ms', d['kernel_only']['serial_launch_ms'], 'identical', d['kernel_only']['identical_to_host_path'])" | tee -a $OUT/ab.txt
    done
  done
done
exit 0
