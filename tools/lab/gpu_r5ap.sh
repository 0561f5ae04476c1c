# round-5: the compacted polish launch — polish / rescue / LPV GPU tests, LPV rounds with the C check, and the
# per-dispatch kernel trace of the rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5ap}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_polish.py tests/test_rounds_gpu.py tests/test_gpu.py -k "polish or rescue or lpv or round" > $O/pytest.log 2>&1 &&
timeout -k 10 300 python tools/run_lpv_rounds.py --rounds 20 --check > $O/lpv.json 2> $O/lpv.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/run_lpv_rounds.py --rounds 20 > $O/lpv_prof.json 2> $O/lpv_prof.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
