# round 6: fp32 last-pass replay, the GPU suite, smoke, the reference configuration — usage: bash tools/lab/gpu_r6f.sh TAG
set -o pipefail
TAG=${1:-r6f}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/f32_replay.py tools/mwlab/f32_bad.npz > $O/f32_replay.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 120 python -u tools/ric_stamps.py > $O/ric_n125_mw.txt 2>&1 &&
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
