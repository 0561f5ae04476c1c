# usage: bash tools/gpu_round.sh TAG — GPU tests, smoke, bench (cfg3 default, cfg5, cfg5 --fp32), rocprofv3
# kernel-trace stats of the same bench command, and PMC passes (FETCH_SIZE, WRITE_SIZE, one each) of the
# cfg3 solver, the cfg5 Riccati kernel and its fp32 mode for the HBM traffic figures, and the
# per-section clocks of the Riccati kernel (tools/ric_stamps.py: N = 125 captured QPs, cfg5).
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
set -o pipefail
TAG=${1:-r1}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
O=gpurun_out/$TAG
export TMPDIR=/tmp
BENCH="bench.py --steps 100 --warmup 5"
C5="bench.py --config cfg5 --steps 10 --warmup 2"
C5F="bench.py --config cfg5 --fp32 --steps 10 --warmup 2"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 600 python $BENCH > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python $C5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err &&
timeout -k 10 300 python $C5F > $O/bench_cfg5_fp32.json 2> $O/bench_cfg5_fp32.err &&
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $BENCH --no-cpu --no-ref > $O/bench_prof.json 2> $O/prof.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run --output-format csv -- python3 $C5 --no-cpu > $O/bench_prof5.json 2> $O/prof5.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof5f -o run --output-format csv -- python3 $C5F --no-cpu > $O/bench_prof5f.json 2> $O/prof5f.err &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ref > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ref > $O/pmc_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc5_fetch -o run --output-format csv -- python3 bench.py --config cfg5 --steps 3 --warmup 1 --no-cpu > $O/pmc5_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc5_write -o run --output-format csv -- python3 bench.py --config cfg5 --steps 3 --warmup 1 --no-cpu > $O/pmc5_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc5f_fetch -o run --output-format csv -- python3 bench.py --config cfg5 --fp32 --steps 3 --warmup 1 --no-cpu > $O/pmc5f_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc5f_write -o run --output-format csv -- python3 bench.py --config cfg5 --fp32 --steps 3 --warmup 1 --no-cpu > $O/pmc5f_write.log 2>&1 &&
timeout -k 10 120 python tools/ric_stamps.py > $O/ric_n125.txt 2>&1 &&
timeout -k 10 120 python tools/ric_stamps.py --cfg5 > $O/ric_cfg5.txt 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
find $O -name "*.csv" | head -80 >> $O/rc.txt
exit $rc
