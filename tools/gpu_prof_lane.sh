set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lane4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/lane_check.py --agents 1024 --rounds 1 --only lane_fp32 --reps 2 > $O/fp32.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $O/pmc -o run --output-format csv -- python3 tools/lane_check.py --agents 1024 --rounds 1 --only lane_f64 --reps 1 > $O/pmc.log 2>&1
echo rc=$? >> $O/pmc.log
