#!/bin/bash
# Round-5 probe: is config 2's host-to-host rate bound by PCIe?  The same
# batch as packed (P16D, ~1.93 KB/catalog) and U16 (~3.8 KB/catalog) records,
# and packed with 32 jobs in flight; --no-cpu, no end-to-end leg.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_h2h
mkdir -p $OUT
for rep in 1 2; do
  for v in packed u16 packed_d32; do
    extra="--record-form packed"
    [ $v = u16 ] && extra="--record-form u16"
    [ $v = packed_d32 ] && extra="--record-form packed --depth 32"
    timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu --e2e-steps 0 $extra > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/${v}_$rep.json').read().strip().splitlines()[-1]); print('$v rep $rep value', d['value'], 'ms', d['ms_per_step'], 'h2d_GBs', d['pcie']['h2d_GBs'], 'bytes', d['pcie']['h2d_bytes_per_step'], 'host', d['host_ms_per_step'], 'kernel_only', d['kernel_only']['res_per_s'])"
  done
done
