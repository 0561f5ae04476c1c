# usage: bash tools/gpu_v3.sh TAG — v3 solver: section clocks, bench, solver GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$1; O=gpurun_out/$1
timeout -k 10 120 python -u tools/stamps.py > $O/stamps.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu --no-ref > $O/bench.json 2> $O/bench.err &&
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 120 --timeout-method thread -k "not riccati and not lpv_n125 and not dist" > $O/pytest.log 2>&1
echo rc=$? >> $O/stamps.txt
