#!/bin/bash
# Where the solve kernel's L2-to-fabric traffic comes from, per config
# (bench.py --kernel-only: records resident in HBM, serial launches).  One
# rocprofv3 --pmc pass per counter group, each under its own kill timeout:
#   size  TCC_EA0_RDREQ by request size (32 / 64 / 128 B) and in total
#   dest  reads served by DRAM, 32 B reads by destination, uncached reads
#   wr    writes in total, 64 B writes, writes to host memory (IO: the
#         results the kernel writes into mapped pinned memory), to DRAM
#   sqc   instruction and scalar-data requests the SQC sends to L2
#   l2    L2 requests, hits and misses
# scripts/fetch_split.py turns the sums into bytes per run.
#   usage: bash scripts/pmc_fetch_split.sh "<configs>" [out_dir]
set -o pipefail
export TMPDIR=/tmp
OUT=${2:-gpurun_out/fetch_split}
mkdir -p $OUT
pass() {  # pass <cfg> <name> <counters...>
  local cfg=$1 name=$2; shift 2
  local ks=6; [ $cfg = 4 ] && ks=2
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/c${cfg}_$name -o run -- \
    python3 bench.py --config $cfg --kernel-only --kernel-steps $ks --no-cpu > $OUT/c${cfg}_$name.json 2> $OUT/c${cfg}_$name.err \
    || { echo "pass $name of config $cfg failed"; return 1; }
}
for cfg in ${1:-3 6 2}; do
  pass $cfg size TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum && \
  pass $cfg dest TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_IO_32B_sum TCC_EA0_RD_UNCACHED_32B_sum && \
  pass $cfg wr TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_WRITE_IO_32B_sum TCC_EA0_WRREQ_DRAM_sum && \
  pass $cfg sqc SQC_TC_INST_REQ SQC_TC_DATA_READ_REQ SQC_ICACHE_MISSES SQC_DCACHE_MISSES && \
  pass $cfg l2 TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_READ_sum || exit 1
  echo "config $cfg done"
done
python3 scripts/fetch_split.py $OUT > $OUT/fetch_split.json && cat $OUT/fetch_split.json
