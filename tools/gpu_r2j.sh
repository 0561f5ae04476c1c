set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$1; O=gpurun_out/$1
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread -k "riccati or lpv or osqp or long_horizon or dist" > $O/pytest_ric.log 2>&1 &&
timeout -k 10 200 python -u tools/ric_stamps.py > $O/stamps.log 2>&1
echo rc=$? >> $O/stamps.log
