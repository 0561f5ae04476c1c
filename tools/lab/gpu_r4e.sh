set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 200 python tools/cfg5_sched.py > $O/sched_fp64.txt 2>&1 &&
timeout -k 10 200 python tools/cfg5_sched.py 8192 fp32 > $O/sched_fp32.txt 2>&1 &&
timeout -k 10 300 python bench.py --config cfg5 --steps 10 --warmup 2 > $O/cfg5.json 2> $O/cfg5.err &&
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -k "riccati or cfg5 or lane or n125 or lpv" -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_sub.log 2>&1
echo rc=$? > $O/rc.txt
