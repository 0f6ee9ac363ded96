#!/bin/bash
# Config 4 single-catalog latency on the same 20 catalogs, three builds on one
# box: the round-2 tree (_ab/r02: its own binding and oracle, extracted with
# `git archive 520402c deppy_amd oracle include` and built in place), the
# round-3 final library (scripts/mkvariant.sh 48e5159 r03) and the current
# build.  Interleaved twice.  scripts/c4_latency.py prints one line per
# catalog (host to host, kernel alone, one oracle thread) and the medians.
# Then the phase stamps of the current build (python -m deppy_amd.build --stamps).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-c4_latency}
M=${2:-20}
mkdir -p $OUT
for rep in 1 2; do
  (cd _ab/r02 && timeout -k 10 300 python -u scripts/c4_latency.py $M) > $OUT/r02_$rep.jsonl 2>&1 || exit 1
  tail -1 $OUT/r02_$rep.jsonl
  DEPPY_VARIANT_LIB=libdeppy_hip_r03.so timeout -k 10 300 python -u scripts/c4_latency.py $M > $OUT/r03_$rep.jsonl 2>&1 || exit 1
  tail -1 $OUT/r03_$rep.jsonl
  timeout -k 10 300 python -u scripts/c4_latency.py $M > $OUT/head_$rep.jsonl 2>&1 || exit 1
  tail -1 $OUT/head_$rep.jsonl
done
# phase stamps of the current build (diagnostic library): one catalog alone
# and 16 together
timeout -k 10 300 python -u scripts/phases.py 4 1,16 > $OUT/phases_c4.jsonl 2> $OUT/phases_c4.err || exit 1
# config 4's kernel-only leg with 8, 16 and 24 resident batches in flight
for kd in 8 16 24; do
  timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 3 --kernel-steps 12 --kernel-depth $kd --no-cpu --e2e-steps 0 > $OUT/kdepth_$kd.json 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/kdepth_$kd.json').read().strip().splitlines()[-1]); print('kernel depth $kd', 'h2h', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'serial_ms', d['kernel_only']['serial_launch_ms'])"
done
exit 0
