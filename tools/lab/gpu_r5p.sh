# round-5: the polish kernel on the one-wave accumulator Cholesky (wave_chol64): polish / rescue tests,
# polish section clocks, the LPV rounds with the C-restatement check
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5p}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_polish.py tests/test_rounds_gpu.py tests/test_gpu.py -k "polish or rescue or lpv or round" > $O/pytest.log 2>&1 &&
timeout -k 10 200 python tools/polish_stamps.py 6 1 > $O/pstamps.txt 2>&1 &&
timeout -k 10 300 python tools/run_lpv_rounds.py --rounds 20 --check > $O/lpv.json 2> $O/lpv.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
