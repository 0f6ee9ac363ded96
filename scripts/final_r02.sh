#!/bin/bash
# Round-2 evidence: per config, rocprofv3 kernel-trace stats of the solve
# kernel alone and its FETCH/WRITE PMC passes (scripts/profile_r02.sh), then
# the bench lines (host to host + kernel only + CPU baseline), whose
# roofline.traffic comes from those PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof
bash scripts/profile_r02.sh "${1:-2 3 5 4}" > gpurun_out/profile.log 2>&1 || { tail -5 gpurun_out/profile.log; exit 1; }
for c in ${1:-2 3 5 4}; do
  st=50; [ $c = 3 ] && st=20; [ $c = 5 ] && st=10; [ $c = 4 ] && st=4
  timeout -k 10 400 python -u bench.py --config $c --steps $st --kernel-steps 24 \
    --pmc-json gpurun_out/prof/pmc_traffic.jsonl > gpurun_out/final_c$c.json 2> gpurun_out/final_c$c.err || exit 1
  echo "bench $c done"
done
