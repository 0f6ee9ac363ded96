#!/bin/bash
# Config 4 after a multi-wave change: GPU parity tests first, then the
# 256-catalog batch, single-catalog latency and phase stamps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 240 python -u scripts/config4.py 256 3 > gpurun_out/c4.json 2> gpurun_out/c4.err || exit 1
timeout -k 10 120 python -u scripts/config4.py 1 5 > gpurun_out/c4.lat.json 2>> gpurun_out/c4.err || exit 1
timeout -k 10 200 python -u scripts/phases.py 4 1,16 > gpurun_out/c4_phases.json 2> gpurun_out/c4_phases.err || exit 1
cut -c1-300 gpurun_out/c4.json gpurun_out/c4.lat.json
timeout -k 10 200 python -u scripts/phases.py 2 10000 > gpurun_out/c2_phases.json 2> gpurun_out/c2_phases.err || exit 1
timeout -k 10 300 python -u bench.py --config 2 --steps 30 --kernel-steps 8 --cpu-seconds 3 > gpurun_out/c2.json 2> gpurun_out/c2.err || exit 1
