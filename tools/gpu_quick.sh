# usage: bash tools/gpu_quick.sh TAG — GPU tests + bench (no profiling)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$1; O=gpurun_out/$1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu > $O/bench.json 2> $O/bench.err
echo rc=$? > $O/rc.txt
