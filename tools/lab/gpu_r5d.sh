# round-5: co-issue ubench; GPU suite, LPV margin, bench on the in-tree library; A/B of the cfg3 kernel
# against tools/v3lab/libcmpc_prev.so (tools/v3_ab.py: per-round kernel time, bit equality)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5d}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 60 tools/ubench/coexec > $O/coexec.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python -u tools/lpv_margin.py --tag $T > $O/margin.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cfg5 > $O/bench.json 2> $O/bench.err &&
CMPC_LIB_PATH=$PWD/tools/v3lab/libcmpc_prev.so timeout -k 10 200 python tools/v3_ab.py $O/prev.npz 40 > $O/prev.txt 2>&1 &&
timeout -k 10 200 python tools/v3_ab.py $O/new.npz 40 > $O/new.txt 2>&1 &&
python tools/v3_ab.py cmp $O/prev.npz $O/new.npz > $O/cmp.txt 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
