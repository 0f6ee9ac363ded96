#!/bin/bash
# Bucket ceilings x merge ratio A/B for config 5, now that footprints under
# 160 KiB / 12 take the 4-waves-per-SIMD build.  Variants are "ceilings@merge"
# ("-" = built-in for either part).
#   usage (via gpurun): bash scripts/ab_dense.sh <tag> <config> <steps> "<variant> ..."
TAG=$1; C=$2; STEPS=$3; VARS=$4
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for v in $VARS; do
    cl=${v%@*}; mg=${v#*@}
    if [ "$cl" = "-" ]; then unset DEPPY_LDS_CEILINGS; else export DEPPY_LDS_CEILINGS=$cl; fi
    if [ "$mg" = "-" ]; then unset DEPPY_BUCKET_MERGE; else export DEPPY_BUCKET_MERGE=$mg; fi
    timeout -k 10 200 python -u bench.py --config $C --steps $STEPS --warmup 4 --no-cpu > $OUT/$rep.$v.log 2>&1 || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('verified_bit_exact_vs_oracle'))" $OUT/$rep.$v.log "$v config$C rep$rep"
  done
done
