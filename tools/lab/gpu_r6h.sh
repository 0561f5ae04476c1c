# round 6: the segmented latency mode with prefetched stage data (lab lib) — usage: bash tools/lab/gpu_r6h.sh TAG
set -o pipefail
TAG=${1:-r6h}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
SEG=$PWD/tools/mwlab/libcmpc_seg2.so
CMPC_LIB_PATH=$SEG timeout -k 10 200 python -u -m pytest tests/test_gpu.py -v -rA -p no:cacheprovider --timeout 150 --timeout-method thread -k "lpv_batch_matches_reference_optimum and n125" > $O/pytest_seg2.log 2>&1 &&
CMPC_LIB_PATH=$SEG timeout -k 10 120 python -u tools/ric_stamps.py > $O/ric_n125_seg2.txt 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
