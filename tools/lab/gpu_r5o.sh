# round-5: LPV-round kernel breakdown (rocprofv3), polish section clocks, the agent-count sweep of the cfg3 round
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5o}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/run_lpv_rounds.py --rounds 20 > $O/lpv.json 2> $O/lpv.err &&
timeout -k 10 200 python tools/polish_stamps.py 6 1 > $O/pstamps.txt 2>&1 &&
timeout -k 10 200 python bench.py --agents 512 --steps 20 --warmup 3 --no-cpu --no-ref --no-cfg5 > $O/b512.json 2> $O/b512.err &&
timeout -k 10 200 python bench.py --agents 1024 --steps 20 --warmup 3 --no-cpu --no-ref --no-cfg5 > $O/b1024.json 2> $O/b1024.err &&
timeout -k 10 200 python bench.py --agents 2048 --steps 20 --warmup 3 --no-cpu --no-ref --no-cfg5 > $O/b2048.json 2> $O/b2048.err &&
timeout -k 10 200 python bench.py --agents 4096 --steps 20 --warmup 3 --no-cpu --no-ref --no-cfg5 > $O/b4096.json 2> $O/b4096.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
