# round-5: LPV-round kernel breakdown (rocprofv3 --kernel-trace --stats) of the current build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5ac}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/run_lpv_rounds.py --rounds 20 > $O/lpv.json 2> $O/lpv.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
