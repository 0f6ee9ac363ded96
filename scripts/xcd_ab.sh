#!/bin/bash
# A/B of the XCD-contiguous launch order (DEPPY_XCD_ORDER = LDS threshold in
# bytes, 0 = LPT everywhere): kernel-only rate, then FETCH_SIZE / WRITE_SIZE
# per solve run (separate PMC passes) for each config.
#   usage: scripts/xcd_ab.sh "<configs>" <setting> ...
set -o pipefail
export TMPDIR=/tmp
CFGS=$1; shift
mkdir -p gpurun_out/xcd
for s in "$@"; do
  export DEPPY_XCD_ORDER=$s
  for cfg in $CFGS; do
    O=gpurun_out/xcd/s${s}_c$cfg
    mkdir -p $O
    timeout -k 10 150 python bench.py --config $cfg --steps 3 --warmup 1 --kernel-steps 30 --no-cpu --e2e-steps 0 > $O/bench.json 2>&1 || { echo "bench $s $cfg failed"; tail -3 $O/bench.json; exit 1; }
    cmd="python3 bench.py --config $cfg --kernel-only --kernel-steps 6 --no-cpu --pmc-json none"
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $cmd > /dev/null 2> $O/fetch.err || { echo "fetch $s $cfg failed"; exit 1; }
    timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $cmd > $O/kernel_only.json 2> $O/write.err || { echo "write $s $cfg failed"; exit 1; }
    python3 scripts/pmc_traffic.py $O/fetch $O/write 7 $cfg $O/kernel_only.json > $O/traffic.json || exit 1
    python3 -c "
import json
b=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); t=json.load(open('$O/traffic.json'))
print('xcd=$s config $cfg kernel_only', b['kernel_only']['res_per_s'], 'fetch', t['fetch_bytes_per_run'], 'write', t['write_bytes_per_run'], 'alg', t['algorithmic_bytes_per_run'], 'ratio', t['traffic_over_algorithmic'])" | tee -a gpurun_out/xcd/summary.txt
  done
done
