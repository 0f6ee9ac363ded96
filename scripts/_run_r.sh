set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in 1 4 8 16; do timeout -k 10 60 ./scripts/plan_bench 3 65536 20 $t; done > gpurun_out/plan_bench.jsonl && \
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
for c in 3 2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --no-cpu --kernel-steps 0 > gpurun_out/b$c.json 2>gpurun_out/b$c.err || exit 1
done
