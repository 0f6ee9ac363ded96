#!/bin/bash
# GPU parity tests, then the kernel-only and host-to-host rates of configs 2, 3, 6 and 5.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-kb2}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E 'FAIL|Error|assert' $OUT/tests.log | head -20; exit 1; }
for cfg in ${CFGS:-2 3 6 5}; do
  timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 5 --kernel-steps 30 --no-cpu --e2e-steps 0 > $OUT/c$cfg.json 2>&1 || { tail -5 $OUT/c$cfg.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c$cfg.json').read().strip().splitlines()[-1]); print('config $cfg', 'h2h', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'serial_ms', d['kernel_only']['serial_launch_ms'])"
done
if [ -f deppy_amd/libdeppy_hip_stamps.so ]; then
  DEPPY_PHASES_FORM=packed timeout -k 10 200 python scripts/phases.py 2 10000 > $OUT/phases_c2.jsonl 2>&1 || { tail -5 $OUT/phases_c2.jsonl; exit 1; }
  python3 -c "
import json
for l in open('$OUT/phases_c2.jsonl'):
    if not l.startswith('{'): continue
    d=json.loads(l); a=d['sat_A']
    print('n', d['n'], 'kernel_ms', round(d['kernel_ms'],3), 'A total', a['total_mean'], 'init', a['init'][0], 'build', a['init_build'][0], 'count', a['build_count'][0], 'scan', a['build_scan'][0], 'fill', a['build_fill'][0], 'stage', a['init_stage'][0], 'validate', a['init_validate'][0], 'base', a['base'][0], 'rounds', a['round_total'][0], 'search', a['search'][0])
"
fi
