#!/bin/bash
# Round-5: the SQ issue/wait split of the library as built now (its digest in
# the json), then the driver's command on config 2 with it.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_sq
mkdir -p $OUT
rm -rf gpurun_out/sq
bash scripts/pmc_sq_r02.sh "2 3 6" > $OUT/sq.log 2>&1 || exit 1
python3 scripts/sq_summary.py gpurun_out/sq > $OUT/sq_split.json || exit 1
cp $OUT/sq_split.json profiles/r05_sq_split.json
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['kernel_only']['res_per_s'], d['build'], json.dumps(d['roofline']['issue'])[:300])"
