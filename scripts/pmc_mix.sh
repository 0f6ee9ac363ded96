#!/bin/bash
# Instruction-mix counter passes over the bench's solve kernel under load
# (pipelined steps).  One pass per SQ budget (8 counters), each under its own
# kill timeout.   usage: bash scripts/pmc_mix.sh <tag> [bench args]
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --no-cpu --steps 12 --warmup 0 --depth 3 $@"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/a -o a -- $B > $OUT/a.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $OUT/b -o b -- $B > $OUT/b.log 2>&1 && \
python scripts/pmc_sum.py $OUT/a $OUT/b > $OUT/mix.json
rc=$?
cat $OUT/mix.json
exit $rc
