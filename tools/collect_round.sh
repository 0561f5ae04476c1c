# usage: bash tools/collect_round.sh TAG PTAG [COMMIT] — copy the summaries of a tools/gpu_round.sh TAG run
# (gpurun_out/TAG) into profiles/ under PTAG: pytest log, smoke, bench lines, rocprof kernel stats and the
# solver-kernel traces (tools/prof_summary.py trace), PMC traffic (tools/prof_summary.py pmc), Riccati stamps.
# Run it on the sources the GPU run used (the PMC summaries stamp their sha).
set -e
TAG=$1; P=$2; C=${3:-$(git rev-parse --short HEAD)}
O=gpurun_out/$TAG; D=profiles
cp $O/pytest_gpu.log $D/${P}_pytest_gpu.log
cp $O/smoke.log $D/${P}_smoke.log
tail -n 1 $O/bench.json > $D/${P}_bench.json
tail -n 1 $O/bench_cfg5.json > $D/${P}_cfg5_bench.json
tail -n 1 $O/bench_cfg5_fp32.json > $D/${P}_cfg5_fp32_bench.json
cp $O/prof/run_kernel_stats.csv $D/${P}_kernel_stats.csv
cp $O/prof5/run_kernel_stats.csv $D/${P}_cfg5_kernel_stats.csv
cp $O/prof5f/run_kernel_stats.csv $D/${P}_cfg5_fp32_kernel_stats.csv
python tools/prof_summary.py trace $O/prof/run_kernel_trace.csv 5 100 $D/${P}_solver_trace.json
SOLVER=mpc_riccati python tools/prof_summary.py trace $O/prof5/run_kernel_trace.csv 2 10 $D/${P}_cfg5_solver_trace.json
SOLVER=mpc_riccati python tools/prof_summary.py trace $O/prof5f/run_kernel_trace.csv 2 10 $D/${P}_cfg5_fp32_solver_trace.json
python tools/prof_summary.py pmc $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv $D/pmc_${P}.json $C
SOLVER=mpc_riccati python tools/prof_summary.py pmc $O/pmc5_fetch/run_counter_collection.csv $O/pmc5_write/run_counter_collection.csv $D/pmc_cfg5_${P}.json $C
SOLVER=mpc_riccati python tools/prof_summary.py pmc $O/pmc5f_fetch/run_counter_collection.csv $O/pmc5f_write/run_counter_collection.csv $D/pmc_cfg5fp32_${P}.json $C
cp $O/ric_n125.txt $D/${P}_riccati_n125_stamps.txt
cp $O/ric_cfg5.txt $D/${P}_riccati_cfg5_stamps.txt
