# round-5: GPU suite; the default bench line (every sub-object) at the driver's step count
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5n}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 900 python -u bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
