#!/bin/bash
# Phase stamps of the one-wavefront kernel with occurrence lists
# (libdeppy_hip_stamps.so) and with two-watched-literal lists
# (libdeppy_hip_stamps_twl.so: python -m deppy_amd.build --stamps
# -DDP_TWL_LDS=1, copied under that name) on configs 2, 3 and 6, 10k
# catalogs each: cycles per round, rounds, watch entries visited per catalog
# (n_watch_1lit + n_flat_entries); records packed (P16D), as bench.py sends them.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-twl_phases}
mkdir -p $OUT
for cfg in 2 3 6; do
  for v in occ twl; do
    lib=libdeppy_hip_stamps.so; [ $v = twl ] && lib=libdeppy_hip_stamps_twl.so
    DEPPY_PHASES_FORM=packed DEPPY_STAMPS_LIB=$lib timeout -k 10 200 python -u scripts/phases.py $cfg 10000 > $OUT/c${cfg}_$v.jsonl 2> $OUT/c${cfg}_$v.err || exit 1
    echo "config $cfg $v done"
  done
done
