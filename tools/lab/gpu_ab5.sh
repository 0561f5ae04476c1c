set -o pipefail
O=gpurun_out/ab5
mkdir -p $O
timeout -k 10 200 python tools/v3_ab.py $O/new.npz 40 > $O/new.txt 2>&1 &&
timeout -k 10 100 python tools/stamps.py > $O/stamps_new.txt 2>&1
echo rc=$? > $O/rc.txt
