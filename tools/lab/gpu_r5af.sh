# round-5: A/B of the Riccati kernel (chunked row loops) against the previous build, and the cfg5 section clocks
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r5af}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
CMPC_LIB_PATH=tools/v3lab/libcmpc_old.so timeout -k 10 300 python tools/ric_ab.py dump /tmp/ric_a.npz > $O/dump_a.log 2>&1 &&
timeout -k 10 300 python tools/ric_ab.py dump /tmp/ric_b.npz > $O/dump_b.log 2>&1 &&
timeout -k 10 100 python tools/ric_ab.py cmp /tmp/ric_a.npz /tmp/ric_b.npz > $O/cmp.txt 2>&1 &&
timeout -k 10 200 python tools/ric_stamps.py --cfg5 > $O/ric_cfg5.txt 2>&1 &&
timeout -k 10 200 python tools/ric_stamps.py > $O/ric_n125.txt 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
