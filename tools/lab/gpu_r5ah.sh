# round-5: cfg5 bench (fp64) and section clocks of the current build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5ah}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config cfg5 --steps 10 --warmup 2 > $O/bench_cfg5.json 2> $O/bench_cfg5.err &&
timeout -k 10 200 python tools/ric_stamps.py --cfg5 > $O/ric_cfg5.txt 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
