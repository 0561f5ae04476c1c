# usage: bash tools/gpu_round.sh TAG — GPU tests, smoke, bench, rocprofv3 kernel-trace stats of the
# same bench command, and two PMC passes (FETCH_SIZE, WRITE_SIZE) for the HBM traffic figure.
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
set -o pipefail
TAG=${1:-r1}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
O=gpurun_out/$TAG
export TMPDIR=/tmp
BENCH="bench.py --steps 100 --warmup 5"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 420 python $BENCH > $O/bench.json 2> $O/bench.err &&
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $BENCH --no-cpu --no-ref > $O/bench_prof.json 2> $O/prof.err &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ref > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ref > $O/pmc_write.log 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
find $O -name "*.csv" | head -50 >> $O/rc.txt
exit $rc
