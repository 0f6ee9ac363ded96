#!/bin/bash
# Two-watched-literal lists on the one-wavefront path (-DDP_TWL_LDS=1, built
# as deppy_amd/libdeppy_hip_twl.so) against the occurrence lists (the
# product library): GPU parity tests of each, then interleaved kernel-only
# and host-to-host rates of configs 2, 3 and 6; then config 2 with one launch
# per residency class (DEPPY_CEILINGS=fine, merge only at equal residency),
# serial on the chunk's stream or spread over sibling streams (DEPPY_SPREAD=1),
# only with FINE=1 in the environment.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_twl}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_occ.log 2>&1
rc=$?; tail -1 $OUT/tests_occ.log; [ $rc -eq 0 ] || exit 1
DEPPY_VARIANT_LIB=libdeppy_hip_twl.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_twl.log 2>&1
rc=$?; tail -1 $OUT/tests_twl.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2.json 2>$OUT/bench_c2.err || exit 1
tail -c 300 $OUT/bench_c2.json; echo
for rep in 1 2; do
for cfg in 2 3 6; do
  for v in occ twl; do
    envs=""; [ $v = twl ] && envs="DEPPY_VARIANT_LIB=libdeppy_hip_twl.so"
    env $envs timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 5 --kernel-steps 30 --no-cpu --e2e-steps 0 > $OUT/c${cfg}_$v.json 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open('$OUT/c${cfg}_$v.json').read().strip().splitlines()[-1]); print('[$v] config $cfg', 'h2h', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'serial_ms', d['kernel_only']['serial_launch_ms'])" | tee -a $OUT/ab.txt
  done
done
done
[ -n "$FINE" ] || exit 0
for rep in 1 2; do
  for v in "-" "DEPPY_CEILINGS=fine DEPPY_BUCKET_MERGE=0.99" "DEPPY_CEILINGS=fine DEPPY_BUCKET_MERGE=0.99 DEPPY_SPREAD=1"; do
    envs=""; [ "$v" != "-" ] && envs="$v"
    env $envs timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 5 --kernel-steps 30 --no-cpu --e2e-steps 0 > $OUT/fine.json 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open('$OUT/fine.json').read().strip().splitlines()[-1]); print('[$v] config 2', 'h2h', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'serial_ms', d['kernel_only']['serial_launch_ms'], 'chunks', d['pipeline'])" | tee -a $OUT/ab_fine.txt
  done
done
exit 0
