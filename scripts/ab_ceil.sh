#!/bin/bash
# LDS bucket ceilings A/B (DEPPY_LDS_CEILINGS, KiB lists; "-" = built-in).
#   usage (via gpurun): bash scripts/ab_ceil.sh <tag> "<configs>" <steps> "<list> <list> ..."
TAG=$1; CONFIGS=$2; STEPS=$3; LISTS=$4
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for c in $CONFIGS; do
    for v in $LISTS; do
      if [ "$v" = "-" ]; then unset DEPPY_LDS_CEILINGS; else export DEPPY_LDS_CEILINGS=$v; fi
      timeout -k 10 200 python -u bench.py --config $c --steps $STEPS --warmup 4 --cpu-seconds 1 > $OUT/$v.$c.$rep.log 2>&1 || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified_bit_exact_vs_oracle'])" $OUT/$v.$c.$rep.log "$v config$c rep$rep"
    done
  done
done
