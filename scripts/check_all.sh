#!/bin/bash
# GPU parity tests, config 2/3 bench lines (short CPU baseline), config 4 at
# 256 and 1024 catalogs per launch.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --config 2 --steps 50 --kernel-steps 8 --cpu-seconds 3 > gpurun_out/c2.json 2> gpurun_out/c2.err || exit 1
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --kernel-steps 8 --cpu-seconds 3 > gpurun_out/c3.json 2> gpurun_out/c3.err || exit 1
timeout -k 10 240 python -u scripts/config4.py 256 3 > gpurun_out/c4.json 2> gpurun_out/c4.err || exit 1
timeout -k 10 300 python -u scripts/config4.py 1024 2 > gpurun_out/c4_1024.json 2>> gpurun_out/c4.err || exit 1
python - <<'PY'
import json
for c in (2, 3):
    d = json.load(open("gpurun_out/c%d.json" % c))
    print(c, d["value"], d["kernel_only"]["res_per_s"], d["pcie"]["h2d_GBs"], d["verified_bit_exact_vs_oracle"], d["cpu_baseline"]["value"])
for f in ("c4", "c4_1024"):
    d = json.load(open("gpurun_out/%s.json" % f))
    print(f, d["n"], d["kernel_ms"], d["res_per_s"], d["oracle_s_16thr"], d["parity"])
PY
