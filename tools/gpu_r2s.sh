set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$1; O=gpurun_out/$1
timeout -k 10 120 python -u tools/diag_build.py > $O/build.log 2>&1
timeout -k 10 120 python -u tools/diag_lpv.py lpv_n20_a4 > $O/diag_nb3.log 2>&1
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 400 python -u bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu > $O/bench_cfg5.json 2> $O/bench_cfg5.err
echo rc=$? > $O/rc.txt
