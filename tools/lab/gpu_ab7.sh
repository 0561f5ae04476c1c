set -o pipefail
O=gpurun_out/ab7
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err
echo rc=$? > $O/rc.txt
