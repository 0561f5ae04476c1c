# round-5: GPU suite with the two-wave mode opt-in; A/B one vs two waves at 512 agents
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5m}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python tools/w2_ab.py 512 20 > $O/w2_512.txt 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
