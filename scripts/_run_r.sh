set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
for c in 2 3; do
  st=50; [ $c = 3 ] && st=20
  timeout -k 10 300 python -u bench.py --config $c --steps $st --no-cpu --kernel-steps 8 > gpurun_out/b$c.json 2>gpurun_out/b$c.err || exit 1
done && rm -rf gpurun_out/prof && bash scripts/profile_r02.sh "2 3" > gpurun_out/profile.log 2>&1
