# round 6: segmented latency-mode lab build (N = 125 optimum + clocks), fp32 last-pass replay, the GPU suite,
# smoke, stamps, bench — usage: bash tools/lab/gpu_r6g.sh TAG
set -o pipefail
TAG=${1:-r6g}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
SEG=$PWD/tools/mwlab/libcmpc_seg.so
CMPC_LIB_PATH=$SEG timeout -k 10 200 python -u -m pytest tests/test_gpu.py -v -rA -p no:cacheprovider --timeout 150 --timeout-method thread -k "lpv_batch_matches_reference_optimum and n125" > $O/pytest_seg.log 2>&1 &&
CMPC_LIB_PATH=$SEG timeout -k 10 120 python -u tools/ric_stamps.py > $O/ric_n125_seg.txt 2>&1
rs=$?
echo "seg rc=$rs" > $O/rc_seg.txt
# an ordinary test failure (1) goes on; a fault, abort or time limit ends the call here
if [ $rs -gt 1 ]; then echo "rc=$rs" > $O/rc.txt; exit $rs; fi
timeout -k 10 120 python -u tools/f32_replay.py tools/mwlab/f32_bad.npz > $O/f32_replay.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 120 python -u tools/ric_stamps.py > $O/ric_n125_mw.txt 2>&1 &&
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
