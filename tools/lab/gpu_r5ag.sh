# round-5: GPU tests + cfg5 bench lines (fp64, fp32) of the current build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5ag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --config cfg5 --steps 10 --warmup 2 > $O/bench_cfg5.json 2> $O/bench_cfg5.err &&
timeout -k 10 300 python bench.py --config cfg5 --fp32 --steps 10 --warmup 2 > $O/bench_cfg5_fp32.json 2> $O/bench_cfg5_fp32.err &&
timeout -k 10 200 python tools/ric_stamps.py > $O/ric_n125.txt 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
