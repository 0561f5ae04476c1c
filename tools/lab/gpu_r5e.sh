# round-5: per-section clocks of the v3 kernel (cfg3 at 1024 and 512 agents, the reference-model LPV round)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5e}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 120 python tools/stamps.py 1024 > $O/stamps_1024.txt 2>&1 &&
timeout -k 10 120 python tools/stamps.py 512 > $O/stamps_512.txt 2>&1 &&
timeout -k 10 180 python tools/stamps.py --lpv > $O/stamps_lpv.txt 2>&1 &&
timeout -k 10 300 python bench.py --agents 512 --steps 20 --warmup 3 --no-cpu --no-ref --no-cfg5 > $O/bench512.json 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
