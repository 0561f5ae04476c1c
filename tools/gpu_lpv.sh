# usage: bash tools/gpu_lpv.sh TAG [pytest -k expr] — GPU tests (optionally a subset), the LPV-rounds
# line with its oracle check, and a rocprofv3 kernel-trace summary of the LPV rounds.
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
set -o pipefail
TAG=${1:-lpv}
K=${2:-}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread ${K:+-k "$K"} > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/run_lpv_rounds.py --check > $O/lpv_rounds.json 2> $O/lpv_rounds.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/run_lpv_rounds.py --rounds 10 > $O/lpv_prof.json 2> $O/lpv_prof.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
