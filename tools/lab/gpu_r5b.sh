# round-5: GPU suite, the LPV parity-margin diagnostic and the default bench line after the degenerate-endpoint polish
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r5b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python -u tools/lpv_margin.py --tag ${1:-r5b} > $O/margin.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cfg5 > $O/bench.json 2> $O/bench.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
