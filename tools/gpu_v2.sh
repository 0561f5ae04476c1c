# GPU tests then the per-phase stamp breakdown; stops after anything but a clean pass/fail
set -o pipefail
TAG=${1:-v2}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 420 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/${TAG}_pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/stamps.py 1024 30 > gpurun_out/${TAG}_stamps.log 2>&1
