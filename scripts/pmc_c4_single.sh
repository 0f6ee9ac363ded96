#!/bin/bash
# Counters of config-4 catalogs solved one at a time (scripts/c4_latency.py:
# each catalog alone, host to host, then resident): L2 hits and misses, the
# reads' destinations, and the SQ issue / wait split of the lone 8-wave
# workgroup.  One rocprofv3 --pmc pass per counter group, each under its own
# kill timeout; scripts/pmc_sum.py sums the solve kernel's dispatches.
#   usage: bash scripts/pmc_c4_single.sh [catalogs] [out_dir]
set -o pipefail
export TMPDIR=/tmp
M=${1:-4}
OUT=${2:-gpurun_out/c4_single}
mkdir -p $OUT
pass() {  # pass <name> <counters...>
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
    python3 scripts/c4_latency.py $M > $OUT/$name.jsonl 2> $OUT/$name.err || { echo "pass $name failed"; return 1; }
}
pass l2 TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_READ_sum && \
pass ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum && \
pass sqa SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS && \
pass sqb SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
for p in l2 ea sqa sqb; do echo "$p $(python3 scripts/pmc_sum.py $OUT/$p)"; done | tee $OUT/summary.txt
