# round-5: MFMA/VALU co-issue micro-benchmark, then GPU suite + LPV margin + bench (tools/lab/gpu_r5b.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r5c}
mkdir -p $O
timeout -k 10 60 tools/ubench/coexec > $O/coexec.txt 2>&1 &&
bash tools/lab/gpu_r5b.sh ${1:-r5c}
