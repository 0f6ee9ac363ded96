#!/bin/bash
# Same-box A/B of library variants: alternating bench runs per config.
#   usage (via gpurun): bash scripts/ab.sh <tag> "<configs>" <steps> lib1 lib2 ...
TAG=$1; CONFIGS=$2; STEPS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in ${REPS:-1 2}; do
  for c in $CONFIGS; do
    for lib in "$@"; do
      DEPPY_VARIANT_LIB=$lib timeout -k 10 150 python -u bench.py --config $c --steps $STEPS --warmup 8 --cpu-seconds 1 > $OUT/$lib.$c.$rep.log 2>&1 || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified_bit_exact_vs_oracle'])" $OUT/$lib.$c.$rep.log "$lib config$c rep$rep"
    done
  done
done
