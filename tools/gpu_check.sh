# usage: bash tools/gpu_check.sh TAG — GPU tests, cfg5 diagnostics, cfg3 and cfg5 bench lines
# (each GPU step under its own time limit, chained with &&).
set -o pipefail
TAG=${1:-chk}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/cfg5_diag.py --rounds 10 --out $O/cfg5_diag > $O/cfg5_diag.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu > $O/bench_cfg5.json 2> $O/bench_cfg5.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
