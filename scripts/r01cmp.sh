set -o pipefail
mkdir -p gpurun_out/r01cmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r01cmp/tests.log 2>&1 || { tail -20 gpurun_out/r01cmp/tests.log; exit 1; }
tail -1 gpurun_out/r01cmp/tests.log
for i in 1 2; do
  (cd r01tree && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu > ../gpurun_out/r01cmp/r01_$i.json 2>&1) || { tail -5 gpurun_out/r01cmp/r01_$i.json; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r01cmp/r01_$i.json').read().strip().splitlines()[-1]); print('r01 tree kernel-only value', d['value'], 'serial', d.get('serial_ms_per_step'))"
  timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 5 --kernel-steps 40 --no-cpu --e2e-steps 0 > gpurun_out/r01cmp/cur_$i.json 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r01cmp/cur_$i.json').read().strip().splitlines()[-1]); print('current h2h', d['value'], 'kernel_only', d['kernel_only']['res_per_s'], 'serial', d['kernel_only']['serial_launch_ms'])"
done
DEPPY_PHASES_FORM=packed timeout -k 10 200 python scripts/phases.py 2 10000 > gpurun_out/r01cmp/phases_c2.jsonl 2>&1 || { tail -5 gpurun_out/r01cmp/phases_c2.jsonl; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r01cmp/phases_c2.jsonl'):
    if not l.startswith('{'): continue
    d=json.loads(l); a=d['sat_A']
    print('n', d['n'], 'kernel_ms', round(d['kernel_ms'],3), 'A total', a['total_mean'], 'init', a['init'][0], 'build', a['init_build'][0], 'count', a['build_count'][0], 'scan', a['build_scan'][0], 'fill', a['build_fill'][0], 'stage', a['init_stage'][0], 'validate', a['init_validate'][0], 'base', a['base'][0], 'rounds', a['round_total'][0], 'search', a['search'][0])
"
