#!/bin/bash
# SQ issue / wait split of the solve kernel per config (one PMC pass each,
# kernel-only serial launches): wave cycles, issuing, waiting on s_waitcnt,
# issue stalls, and the instruction mix.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sq
for cfg in ${1:-2 4}; do
  case $cfg in 4) ks=2;; *) ks=6;; esac
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
    --output-format csv -d gpurun_out/sq/c${cfg}_a -o run -- python3 bench.py --config $cfg --kernel-only --kernel-steps $ks --no-cpu \
    > /dev/null 2> gpurun_out/sq/c${cfg}_a.err || { echo "sq a $cfg failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    --output-format csv -d gpurun_out/sq/c${cfg}_b -o run -- python3 bench.py --config $cfg --kernel-only --kernel-steps $ks --no-cpu \
    > /dev/null 2> gpurun_out/sq/c${cfg}_b.err || { echo "sq b $cfg failed"; exit 1; }
  echo "config $cfg done"
done
