# round-5: polish section clocks + LPV rounds (A/B of one build of the polish kernel)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5q}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/polish_stamps.py 6 1 > $O/pstamps.txt 2>&1 &&
timeout -k 10 300 python tools/run_lpv_rounds.py --rounds 20 --check > $O/lpv.json 2> $O/lpv.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
