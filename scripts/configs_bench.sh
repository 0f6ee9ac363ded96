#!/bin/bash
# Bench lines for the non-headline workloads (configs 3, 4, 5) plus the kernel
# stats of config 3 and 5.  Every GPU step has its own time limit; && ends the
# call at the first failure.
#   usage (via gpurun): bash scripts/configs_bench.sh <tag>
set -o pipefail
TAG=${1:-cfg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python -u bench.py --config 3 --steps 30 > $OUT/bench3.log 2>&1 && \
timeout -k 10 240 python -u bench.py --config 5 --steps 20 > $OUT/bench5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 > $OUT/bench4.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof3 -o prof -- python3 bench.py --no-cpu --config 3 --steps 10 --warmup 2 > $OUT/prof3.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5 -o prof -- python3 bench.py --no-cpu --config 5 --steps 5 --warmup 1 > $OUT/prof5.log 2>&1
rc=$?
for f in $OUT/bench3.log $OUT/bench5.log $OUT/bench4.log; do [ -f $f ] && tail -1 $f; done
exit $rc
