set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$1; O=gpurun_out/$1
timeout -k 10 300 python -u -m pytest tests/test_mex_gpu.py tests/test_dist_gpu.py -q -rA -p no:cacheprovider --timeout 280 --timeout-method thread > $O/pytest_mex.log 2>&1
for i in 1 2; do timeout -k 10 120 python -u tools/ric_stamps.py > $O/cur$i.log 2>&1 && CMPC_LIB_PATH=$PWD/colaborativempc-_amd/lib/var/libcmpc.so timeout -k 10 120 python -u tools/ric_stamps.py > $O/var$i.log 2>&1 || exit 1; done
