set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m3 -E "gfx|Marketing" > gpurun_out/r1_rocminfo.txt || true
timeout -k 10 420 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r1d_pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r1d_pytest_gpu.log
exit $rc
