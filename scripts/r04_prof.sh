#!/bin/bash
# Round-4 profiles of the product build: rocprofv3 kernel-trace stats and the
# FETCH_SIZE / WRITE_SIZE passes per config (scripts/profile_r02.sh), the SQ
# issue / wait split and instruction mix (scripts/pmc_sq_r02.sh), LDS
# counters of config 2 (scripts/pmc_lds.sh), and the counter list of this
# ROCm for the fetch breakdown.  Every GPU step has its own kill timeout and
# the steps are chained, so the first failure ends the call.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/sq
timeout -s KILL 60 rocprofv3 -L > gpurun_out/prof/counters.txt 2>&1 || true
bash scripts/profile_r02.sh "${1:-2 3 6}" && \
bash scripts/pmc_sq_r02.sh "${2:-2 3 6}" && \
python3 scripts/sq_summary.py gpurun_out/sq > gpurun_out/sq/sq_split.json && \
bash scripts/pmc_lds.sh lds_c2 --kernel-only --kernel-steps 6
rc=$?
cat gpurun_out/prof/pmc_traffic.jsonl; head -c 1500 gpurun_out/sq/sq_split.json
exit $rc
