# round-5: the v3 kernel's two-wave mode — A/B against one wave (bit equality, kernel time) at 512 and 1024
# agents, then the GPU suite (small fused batches now run two waves by default), the 512-agent bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5i}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 120 python tools/w2_ab.py 512 20 > $O/w2_512.txt 2>&1 &&
timeout -k 10 120 python tools/w2_ab.py 1024 20 > $O/w2_1024.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --agents 512 --steps 20 --warmup 3 --no-cpu --no-ref --no-cfg5 > $O/bench512.json 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
