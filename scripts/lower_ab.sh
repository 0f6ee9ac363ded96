#!/bin/bash
# Host lowering A/B on the GPU box's CPU share: two builds of a standalone
# lowering benchmark (scripts/lower_bench_main.cpp linked with lower.cpp and
# gen.cpp, in _lprof/), interleaved, one thread and the whole share.
#   usage: bash scripts/lower_ab.sh <binary A> <binary B>
A=${1:-_lprof/lprof_base}; B=${2:-_lprof/lprof_new}
for rep in 1 2 3; do
  for t in 1 16; do
    for bin in $A $B; do
      for cfg in 2 3; do
        n=10000; [ $cfg = 3 ] && n=100000
        echo "$(basename $bin) threads=$t $(DEPPY_HOST_THREADS=$t timeout -k 5 120 $bin $cfg $n 20)"
      done
    done
  done
done
