# round-5 lab: two-wave mode determinism and per-iteration merits (tools/v3lab/dbg: -DCMPC_DBG_MERIT)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5k}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 120 python tools/w2_dbg.py 8 6 > $O/dbg.txt 2>&1 &&
CMPC_LIB_PATH=$PWD/tools/v3lab/dbg/libcmpc.so timeout -k 10 120 python tools/w2_dbg.py 8 8 merit > $O/merit.txt 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
