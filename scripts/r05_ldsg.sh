#!/bin/bash
# Round 5: the all-LDS multi-wave placement (M_LDSG).  GPU parity tests, then
# config 5 host to host / kernel only with M_LDSG (default), without it
# (DEPPY_LDSG=0: the HBM-read multi-wave groups, as in round 4), and with
# every 16-bit catalog on one wavefront (DEPPY_GROUP_ABOVE=163840).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r05/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05/tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab_env.sh 5 ${1:-2} - DEPPY_LDSG=0 DEPPY_GROUP_ABOVE=163840
