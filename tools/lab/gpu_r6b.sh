# round 6: latency-mode check (tools/mw_dbg.py), the N = 125 tests, then the GPU suite — usage: bash tools/lab/gpu_r6b.sh TAG
set -o pipefail
TAG=${1:-r6b}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 python -u tools/mw_dbg.py 6 > $O/mw_dbg.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -rA -p no:cacheprovider --timeout 200 --timeout-method thread -k "n125 or latency_mode" > $O/pytest_n125.log 2>&1 &&
timeout -k 10 120 python -u tools/ric_stamps.py > $O/ric_n125_mw.txt 2>&1 &&
timeout -k 10 120 python -u tools/ric_stamps.py --one-wave > $O/ric_n125_one.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --config cfg5 --steps 10 --warmup 2 > $O/bench_cfg5.json 2> $O/bench_cfg5.err &&
timeout -k 10 300 python bench.py --config cfg5 --fp32 --steps 10 --warmup 2 > $O/bench_cfg5_fp32.json 2> $O/bench_cfg5_fp32.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
