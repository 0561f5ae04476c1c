# round 6: GPU suite, smoke, cfg5 lines (fp64 / fp32) — usage: bash tools/lab/gpu_r6a.sh TAG
set -o pipefail
TAG=${1:-r6a}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --config cfg5 --steps 10 --warmup 2 > $O/bench_cfg5.json 2> $O/bench_cfg5.err &&
timeout -k 10 300 python bench.py --config cfg5 --fp32 --steps 10 --warmup 2 > $O/bench_cfg5_fp32.json 2> $O/bench_cfg5_fp32.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
