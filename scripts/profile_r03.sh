#!/bin/bash
# Round-3 kernel profiles: for each BASELINE config, rocprofv3 kernel-trace
# stats of the solve kernel alone (bench.py --kernel-only: records resident in
# HBM, K + 1 serial launches), then one PMC pass each for
# FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md: separate passes).
# Usage: scripts/profile_r03.sh "2 3 5 4"
set -o pipefail
export TMPDIR=/tmp
K=10
mkdir -p gpurun_out/prof
for cfg in ${1:-2 3 5 4}; do
  case $cfg in 4) ks=4;; *) ks=$K;; esac
  cmd="python3 bench.py --config $cfg --kernel-only --kernel-steps $ks --no-cpu --pmc-json none"
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/c${cfg}_trace -o run -- $cmd \
    > gpurun_out/prof/c${cfg}_trace.json 2> gpurun_out/prof/c${cfg}_trace.err || { echo "trace $cfg failed"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/c${cfg}_fetch -o run -- $cmd \
    > /dev/null 2> gpurun_out/prof/c${cfg}_fetch.err || { echo "fetch $cfg failed"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/c${cfg}_write -o run -- $cmd \
    > /dev/null 2> gpurun_out/prof/c${cfg}_write.err || { echo "write $cfg failed"; exit 1; }
  python3 scripts/pmc_traffic.py gpurun_out/prof/c${cfg}_fetch gpurun_out/prof/c${cfg}_write $((ks + 1)) $cfg \
    gpurun_out/prof/c${cfg}_trace.json >> gpurun_out/prof/pmc_traffic.jsonl || exit 1
  echo "config $cfg done"
done
