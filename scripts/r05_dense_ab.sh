#!/bin/bash
# Round-5 A/B: the 128-VGPR one-wavefront build (solve_lds_dense.hip, chosen
# for small catalogs) against the unbounded build alone (DEPPY_NO_DENSE=1):
# fabric writes per run (one rocprofv3 --pmc pass) and kernel-only rates,
# configs 3 and 6, interleaved.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_dense
mkdir -p $OUT
for cfg in 3 6; do
  for v in dense nodense; do
    if [ $v = nodense ]; then export DEPPY_NO_DENSE=1; else unset DEPPY_NO_DENSE; fi
    timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum \
      --output-format csv -d $OUT/c${cfg}_$v -o run -- \
      python3 bench.py --config $cfg --kernel-only --kernel-steps 6 --no-cpu > $OUT/c${cfg}_${v}_pmc.json 2> $OUT/c${cfg}_${v}_pmc.err || exit 1
  done
  for rep in 1 2; do
    for v in dense nodense; do
      if [ $v = nodense ]; then export DEPPY_NO_DENSE=1; else unset DEPPY_NO_DENSE; fi
      timeout -k 10 120 python3 bench.py --config $cfg --kernel-only --kernel-steps 30 --no-cpu > $OUT/c${cfg}_${v}_$rep.json 2> $OUT/c${cfg}_${v}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$OUT/c${cfg}_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_only']; print('config $cfg $v rep $rep kernel_only', k['res_per_s'], 'serial_ms', k['serial_launch_ms'])"
    done
  done
done
python3 - <<'PY'
import csv, glob, os
for d in sorted(glob.glob("gpurun_out/r05_dense/c*_*dense")):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    tot = {}
    n = 0
    for r in csv.DictReader(open(f[0])):
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        n += 1
    print(os.path.basename(d), {k: int(v) for k, v in tot.items()})
PY
