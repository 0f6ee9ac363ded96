#!/bin/bash
# Phase stamps of config-4 catalogs (the diagnostic library): one alone, 16 together.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c4ph
timeout -k 10 300 python -u scripts/phases.py 4 1,16 > gpurun_out/c4ph/phases_c4.jsonl 2> gpurun_out/c4ph/phases_c4.err
