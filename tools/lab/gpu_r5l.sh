# round-5 lab: section clocks of the v3 kernel at 512 agents, one wave vs two waves per agent
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5l}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 120 python tools/stamps.py 512 --one-wave > $O/stamps_512_w1.txt 2>&1 &&
timeout -k 10 120 python tools/stamps.py 512 --two-waves > $O/stamps_512_w2.txt 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
