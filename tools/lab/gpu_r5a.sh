# round-5 first check: the GPU suite on the current sources, then the LPV parity-margin diagnostic
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python -u tools/lpv_margin.py --tag r5a > $O/margin.log 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
