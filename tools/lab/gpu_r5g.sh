# round-5: polish kernel section clocks, previous library vs in-tree; polish / rescue GPU tests; LPV rounds line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5g}
O=gpurun_out/$T
mkdir -p $O
CMPC_LIB_PATH=$PWD/tools/v3lab/libcmpc_prev.so timeout -k 10 200 python tools/polish_stamps.py 6 2 > $O/pstamps_prev.txt 2>&1 &&
timeout -k 10 200 python tools/polish_stamps.py 6 2 > $O/pstamps_new.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_polish.py tests/test_rounds_gpu.py tests/test_gpu.py -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread -k "polish or rescue or infeasible or edge or scale or lpv" > $O/pytest_pol.log 2>&1 &&
timeout -k 10 200 python tools/run_lpv_rounds.py --rounds 20 > $O/lpv.json 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
