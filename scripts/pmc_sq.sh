#!/bin/bash
# SQ / SQC counter passes over the bench's solve kernel (one pass per block
# budget; each pass under its own kill timeout).  usage: bash scripts/pmc_sq.sh <tag> [bench args]
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --no-cpu --steps 5 --warmup 0 --depth 1 $@"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_IFETCH SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $OUT/sq -o sq -- $B > $OUT/sq.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $OUT/sqc -o sqc -- $B > $OUT/sqc.log 2>&1 && \
python scripts/pmc_sum.py $OUT/sq $OUT/sqc > $OUT/sq_summary.json
rc=$?
cat $OUT/sq_summary.json
exit $rc
