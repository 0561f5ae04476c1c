set -o pipefail
O=gpurun_out/ab4
mkdir -p $O
timeout -k 10 200 python tools/v3_ab.py $O/new.npz 40 > $O/new.txt 2>&1 &&
timeout -k 10 100 python tools/stamps.py > $O/stamps_new.txt 2>&1 &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo rc=$? > $O/rc.txt
