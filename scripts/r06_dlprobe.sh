#!/bin/bash
# Device lowering alone: its parity tests, call times (scripts/dl_probe.py,
# with DEPPY_DL_TIMES=1 phase times) for configs 2, 3, 6 and a rocprofv3
# kernel + memory-copy trace of config 2's calls.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_device_lowering.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/dl_tests.log 2>&1
rc=$?; tail -1 $OUT/dl_tests.log; [ $rc -eq 0 ] || exit 1
for c in 2 3 6; do
  DEPPY_DL_TIMES=1 timeout -k 10 200 python -u scripts/dl_probe.py $c 10000 20 > $OUT/probe_c$c.txt 2>&1 || exit 1
  tail -3 $OUT/probe_c$c.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/tr -o run -- \
  python3 scripts/dl_probe.py 2 10000 10 > $OUT/tr.log 2>&1 || exit 1
echo done
