set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s3_chk
timeout -k 10 300 python -u -m pytest tests/test_device_lowering.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3_chk/dl.log 2>&1; rc=$?; tail -1 gpurun_out/s3_chk/dl.log; [ $rc -eq 0 ] || exit 1
for c in 5 4; do DEPPY_DL_TIMES=1 timeout -k 10 200 python -u scripts/dl_probe.py $c $([ $c = 4 ] && echo 64 || echo 10000) 5 2>&1 | tail -2 || exit 1; done
