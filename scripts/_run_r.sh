set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config 2 --steps 50 --no-cpu > gpurun_out/b2.json 2>gpurun_out/b2.err && \
DEPPY_DIRECT=0 timeout -k 10 200 python -u bench.py --config 2 --steps 50 --no-cpu --kernel-steps 0 > gpurun_out/b2_staged.json 2>>gpurun_out/b2.err && \
timeout -k 10 200 python -u bench.py --config 3 --steps 20 --no-cpu > gpurun_out/b3.json 2>>gpurun_out/b2.err
