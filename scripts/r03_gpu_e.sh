#!/bin/bash
# Round 3: the capped one-wavefront build without the BCP counter (3 VGPR
# spills instead of 12): GPU tests, config 3/6 PMC traffic and kernel rates.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/${TAG:-prof3}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r03_gputest_f.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r03_gputest_f.log; [ $rc -eq 0 ] || exit 1
for cfg in 3 6; do
  cmd="python3 bench.py --config $cfg --kernel-only --kernel-steps 10 --no-cpu --pmc-json none"
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG:-prof3}/c${cfg}_trace -o run -- $cmd > gpurun_out/${TAG:-prof3}/c${cfg}_trace.json 2> gpurun_out/${TAG:-prof3}/c${cfg}_trace.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG:-prof3}/c${cfg}_fetch -o run -- $cmd > /dev/null 2> gpurun_out/${TAG:-prof3}/c${cfg}_fetch.err || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG:-prof3}/c${cfg}_write -o run -- $cmd > /dev/null 2> gpurun_out/${TAG:-prof3}/c${cfg}_write.err || exit 1
  python3 scripts/pmc_traffic.py gpurun_out/${TAG:-prof3}/c${cfg}_fetch gpurun_out/${TAG:-prof3}/c${cfg}_write 11 $cfg gpurun_out/${TAG:-prof3}/c${cfg}_trace.json >> gpurun_out/${TAG:-prof3}/pmc_traffic.jsonl || exit 1
  timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --kernel-steps 30 --no-cpu --e2e-steps 0 > gpurun_out/${TAG:-prof3}_c$cfg.json 2>&1 || exit 1
done
cat gpurun_out/${TAG:-prof3}/pmc_traffic.jsonl
