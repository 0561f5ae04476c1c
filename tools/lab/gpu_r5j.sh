# round-5 lab: where the two-wave mode departs from one wave (max_iter sweep), in-tree and with the
# predictor right-hand side kept on wave 0 (tools/v3lab/w2k, -DCMPC_W2_RHS=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5j}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 120 python tools/w2_dbg.py 8 8 > $O/dbg.txt 2>&1 &&
CMPC_LIB_PATH=$PWD/tools/v3lab/w2k/libcmpc.so timeout -k 10 120 python tools/w2_dbg.py 8 8 > $O/dbg_k.txt 2>&1 &&
CMPC_LIB_PATH=$PWD/tools/v3lab/w2k/libcmpc.so timeout -k 10 120 python tools/w2_ab.py 512 20 > $O/w2k_512.txt 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
