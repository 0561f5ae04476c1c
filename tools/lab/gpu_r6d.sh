# round 6: latency-mode role clocks (piped / not piped), the fp32 path's KKT failures captured — usage: bash tools/lab/gpu_r6d.sh TAG
set -o pipefail
TAG=${1:-r6d}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/ric_stamps.py > $O/ric_n125_mw.txt 2>&1 &&
CMPC_LIB_PATH=$PWD/tools/mwlab/libcmpc_nopipe.so timeout -k 10 120 python -u tools/ric_stamps.py > $O/ric_n125_mw_nopipe.txt 2>&1 &&
timeout -k 10 180 python -u tools/f32_capture.py $O/f32_bad.npz 12 > $O/f32_capture.txt 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
