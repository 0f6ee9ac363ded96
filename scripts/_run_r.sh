set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
for c in 4 5 2; do
  st=10; [ $c = 4 ] && st=4; [ $c = 2 ] && st=50
  timeout -k 10 300 python -u bench.py --config $c --steps $st --no-cpu --kernel-steps 4 > gpurun_out/b$c.json 2>gpurun_out/b$c.err || exit 1
done
