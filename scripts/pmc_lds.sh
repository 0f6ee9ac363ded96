#!/bin/bash
# LDS and memory-path counter passes over the bench's solve kernel (north_star:
# "rocprof counters showing coalesced clause-array reads and LDS hit behaviour").
# One pass per block budget, each under its own kill timeout.
#   usage: bash scripts/pmc_lds.sh <tag> [bench args]
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --no-cpu --steps 5 --warmup 0 --depth 1 $@"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $OUT/lds -o lds -- $B > $OUT/lds.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TA_FLAT_READ_WAVEFRONTS_sum TA_FLAT_READ_LDS_WAVEFRONTS_sum --output-format csv -d $OUT/mem -o mem -- $B > $OUT/mem.log 2>&1 && \
python scripts/pmc_sum.py $OUT/lds $OUT/mem > $OUT/lds_summary.json
rc=$?
cat $OUT/lds_summary.json
exit $rc
