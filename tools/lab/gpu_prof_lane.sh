# usage: bash tools/lab/gpu_prof_lane.sh TAG — PMC passes (instruction mix, waits, instruction cache) of the lane kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-lanepmc}
mkdir -p $O
export TMPDIR=/tmp
CMD="python3 tools/lane_check.py --agents 1024 --rounds 1 --only lane_f64 --reps 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_SALU -d $O/p1 -o run --output-format csv -- $CMD > $O/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d $O/p2 -o run --output-format csv -- $CMD > $O/p2.log 2>&1
echo rc=$? >> $O/p2.log
