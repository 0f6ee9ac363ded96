#!/bin/bash
# Round-2 evidence: bench lines (host to host + kernel only + CPU baseline)
# for every config, then kernel-trace stats and PMC traffic per config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 2 3 5 4; do
  st=50; [ $c = 3 ] && st=20; [ $c = 5 ] && st=10; [ $c = 4 ] && st=4
  timeout -k 10 400 python -u bench.py --config $c --steps $st --kernel-steps 8 > gpurun_out/final_c$c.json 2> gpurun_out/final_c$c.err || exit 1
  echo "bench $c done"
done
rm -rf gpurun_out/prof && bash scripts/profile_r02.sh "2 3 5 4" > gpurun_out/profile.log 2>&1
