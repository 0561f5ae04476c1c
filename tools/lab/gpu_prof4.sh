# usage: bash tools/lab/gpu_prof4.sh TAG — round-4 evidence: SQ counter passes (tools/pmc_sq.sh), PMC traffic passes
# (FETCH_SIZE / WRITE_SIZE) and rocprofv3 kernel-trace stats of the bench commands (cfg3 default, cfg5, cfg5 fp32).
set -o pipefail
TAG=${1:-r4}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
B3="bench.py --steps 20 --warmup 3 --no-cpu --no-ref --no-cfg5"
C5="bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu"
C5F="bench.py --config cfg5 --fp32 --steps 10 --warmup 2 --no-cpu"
bash tools/pmc_sq.sh $TAG/sq all > $O/sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $B3 > $O/bench_prof.json 2> $O/prof.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run --output-format csv -- python3 $C5 > $O/bench_prof5.json 2> $O/prof5.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof5f -o run --output-format csv -- python3 $C5F > $O/bench_prof5f.json 2> $O/prof5f.err &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ref --no-cfg5 > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ref --no-cfg5 > $O/pmc_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc5_fetch -o run --output-format csv -- python3 bench.py --config cfg5 --steps 3 --warmup 1 --no-cpu > $O/pmc5_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc5_write -o run --output-format csv -- python3 bench.py --config cfg5 --steps 3 --warmup 1 --no-cpu > $O/pmc5_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc5f_fetch -o run --output-format csv -- python3 bench.py --config cfg5 --fp32 --steps 3 --warmup 1 --no-cpu > $O/pmc5f_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc5f_write -o run --output-format csv -- python3 bench.py --config cfg5 --fp32 --steps 3 --warmup 1 --no-cpu > $O/pmc5f_write.log 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
