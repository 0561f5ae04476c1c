# usage: bash tools/pmc_sq.sh TAG [cfg3|cfg5|cfg5f|all] — SQ instruction-mix / wave-state counter passes (one
# rocprofv3 --pmc pass per counter group, at most 8 SQ counters each, the program directly after --) over short
# bench.py runs; summarised by `python tools/prof_summary.py sq`.  Each pass has its own time limit; the passes
# are chained with && (stop at the first failure).
set -o pipefail
TAG=${1:-sq}
WHICH=${2:-all}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_WAVES"
P3="SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_VALU_MFMA_COEXEC_CYCLES"
P4="GRBM_GUI_ACTIVE GRBM_COUNT"
run() {  # run NAME "ARGS"
    local name=$1 args=$2 i=1 rc=0
    for P in "$P1" "$P2" "$P3" "$P4"; do
        timeout -s KILL 120 rocprofv3 --pmc $P -d $O/${name}_p$i -o run --output-format csv -- python3 bench.py $args \
            > $O/${name}_p$i.log 2>&1 || return $?
        i=$((i + 1))
    done
}
rc=0
if [ "$WHICH" = all ] || [ "$WHICH" = cfg3 ]; then
    run cfg3 "--steps 5 --warmup 1 --no-cpu --no-ref" || rc=$?
fi
if [ $rc = 0 ] && { [ "$WHICH" = all ] || [ "$WHICH" = cfg5 ]; }; then
    run cfg5 "--config cfg5 --steps 3 --warmup 1 --no-cpu" || rc=$?
fi
if [ $rc = 0 ] && { [ "$WHICH" = all ] || [ "$WHICH" = cfg5f ]; }; then
    run cfg5f "--config cfg5 --fp32 --steps 3 --warmup 1 --no-cpu" || rc=$?
fi
echo "rc=$rc" > $O/rc.txt
find $O -name "*counter_collection.csv" >> $O/rc.txt
exit $rc
