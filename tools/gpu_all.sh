# usage: bash tools/gpu_all.sh TAG  — gpu tests, smoke, bench, rocprofv3 kernel-trace stats
set -o pipefail
TAG=${1:-r1}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/${TAG}_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 &&
timeout -k 10 420 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err &&
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/${TAG}_bench_prof.json 2> gpurun_out/${TAG}_prof.err
rc=$?
echo "rc=$rc" >> gpurun_out/${TAG}_pytest_gpu.log
exit $rc
