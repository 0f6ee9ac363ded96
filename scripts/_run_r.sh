set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 2 3 5; do
  st=50; [ $c = 3 ] && st=20; [ $c = 5 ] && st=10
  timeout -k 10 300 python -u bench.py --config $c --steps $st --no-cpu --kernel-steps 6 > gpurun_out/b$c.json 2>gpurun_out/b$c.err || exit 1
done
