# round 6: latency mode with the piped pass's A/B prefetch (lab lib), fp32 failure replay — usage: bash tools/lab/gpu_r6e.sh TAG
set -o pipefail
TAG=${1:-r6e}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
CMPC_LIB_PATH=$PWD/tools/mwlab/libcmpc_pf.so timeout -k 10 120 python -u tools/ric_stamps.py > $O/ric_n125_mw_pf.txt 2>&1 &&

timeout -k 10 120 python -u tools/f32_replay.py tools/mwlab/f32_bad.npz > $O/f32_replay.txt 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
