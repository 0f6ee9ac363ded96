#!/bin/bash
# Device lowering A/B: the packing's stream at high priority (default) vs a
# normal stream (DEPPY_DL_PACK_PRIORITY=0), config 2, with a kernel and
# memory-copy trace of the default.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
for r in 1 2; do
  DEPPY_DL_TIMES=0 timeout -k 10 200 python -u scripts/dl_probe.py 2 10000 20 >> $OUT/ab.txt 2>&1 || exit 1
  DEPPY_DL_PACK_PRIORITY=0 timeout -k 10 200 python -u scripts/dl_probe.py 2 10000 20 | sed 's/^/normal-priority /' >> $OUT/ab.txt 2>&1 || exit 1
done
cat $OUT/ab.txt
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/tr -o run -- \
  python3 scripts/dl_probe.py 2 10000 10 > $OUT/tr.log 2>&1 || exit 1
echo done
