#!/bin/bash
# Round 5, config 4: L2 hit rate and fabric traffic with 2-byte watch entries
# (the build) and with 8-byte ones (DEPPY_VARIANT_LIB=libdeppy_hip_went8.so):
# four catalogs alone (scripts/c4_latency.py) and the 256-catalog batch
# (bench.py --kernel-only).  One rocprofv3 --pmc pass per counter group.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_c4_pmc
mkdir -p $OUT
one() {  # one <tag> <name> <counters...>
  local tag=$1 name=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/${tag}_single_$name -o run -- \
    python3 scripts/c4_latency.py 4 > $OUT/${tag}_single_$name.jsonl 2> $OUT/${tag}_single_$name.err || { echo "pass $tag $name failed"; return 1; }
}
batch() {  # batch <tag> <name> <counters...>
  local tag=$1 name=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/${tag}_batch_$name -o run -- \
    python3 bench.py --config 4 --kernel-only --kernel-steps 2 --no-cpu > $OUT/${tag}_batch_$name.json 2> $OUT/${tag}_batch_$name.err || { echo "pass $tag $name failed"; return 1; }
}
for tag in head went8; do
  if [ $tag = went8 ]; then export DEPPY_VARIANT_LIB=libdeppy_hip_went8.so; fi
  one $tag l2 TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_READ_sum || exit 1
  one $tag sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
  batch $tag size TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum || exit 1
  batch $tag wr TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_WRITE_IO_32B_sum TCC_EA0_WRREQ_DRAM_sum || exit 1
  batch $tag l2 TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_READ_sum || exit 1
  for d in $OUT/${tag}_*; do [ -d $d ] && echo "$(basename $d) $(python3 scripts/pmc_sum.py $d)"; done | tee -a $OUT/summary.txt
done
