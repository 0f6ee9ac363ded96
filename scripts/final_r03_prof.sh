#!/bin/bash
# Round-3 closing profiles of the final build: rocprofv3 kernel-trace stats
# and FETCH_SIZE / WRITE_SIZE passes per config (scripts/profile_r03.sh), and
# the SQ issue / wait split of configs 2 and 4 (scripts/pmc_sq_r02.sh).
set -o pipefail
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/sq
bash scripts/profile_r03.sh "${1:-2 3 5 6 4}" || exit 1
bash scripts/pmc_sq_r02.sh "2 4" || exit 1
python3 scripts/sq_summary.py gpurun_out/sq > gpurun_out/sq/sq_split.json || exit 1
cat gpurun_out/prof/pmc_traffic.jsonl
