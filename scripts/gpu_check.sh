#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats and the
# two PMC passes for HBM traffic.  Every GPU step has its own time limit and the
# steps are chained with && so the first failure ends the call.
#   usage (via gpurun): bash scripts/gpu_check.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-run}; shift
BARGS="$@"
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py $BARGS > $OUT/bench.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- python3 bench.py --no-cpu --steps 10 --warmup 2 $BARGS > $OUT/prof.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 bench.py --no-cpu --steps 5 --warmup 0 --depth 1 $BARGS > $OUT/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- python3 bench.py --no-cpu --steps 5 --warmup 0 --depth 1 $BARGS > $OUT/pmc_write.log 2>&1
rc=$?
[ $rc -eq 0 ] && python scripts/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write 9 > $OUT/pmc_traffic.json
tail -3 $OUT/gpu_tests.log; cat $OUT/bench.log | tail -2
exit $rc
