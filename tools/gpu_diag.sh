# usage: bash tools/gpu_diag.sh TAG — captured-QP diagnostic (condensed and forced Riccati) + the GPU test suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$1; O=gpurun_out/$1
timeout -k 10 180 python -u tools/diag_lpv.py --riccati > $O/diag.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo rc=$? >> $O/diag.log
