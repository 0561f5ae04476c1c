# round-5: GPU suite; LS kernel stamps (L5 contraction); LPV A/B vs tools/v3lab/libcmpc_prev.so; polish stamps; LPV rounds line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5h}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 180 python tools/stamps.py --lpv > $O/stamps_lpv.txt 2>&1 &&
CMPC_LIB_PATH=$PWD/tools/v3lab/libcmpc_prev.so timeout -k 10 200 python tools/lpv_ab.py $O/lprev.npz 10 > $O/lprev.txt 2>&1 &&
timeout -k 10 200 python tools/lpv_ab.py $O/lnew.npz 10 > $O/lnew.txt 2>&1 &&
python tools/lpv_ab.py cmp $O/lprev.npz $O/lnew.npz > $O/lcmp.txt 2>&1 &&
timeout -k 10 200 python tools/polish_stamps.py 6 1 > $O/pstamps.txt 2>&1 &&
timeout -k 10 200 python tools/run_lpv_rounds.py --rounds 20 --check > $O/lpv.json 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
