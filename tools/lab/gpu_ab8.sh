# A/B of the in-tree library against tools/v3lab/libcmpc_prev.so: cfg3 kernel time and bit equality
# (v3_ab), the reference-model rounds (lpv_ab); usage: bash tools/lab/gpu_ab8.sh TAG
set -o pipefail
O=gpurun_out/${1:-ab8}
mkdir -p $O
CMPC_LIB_PATH=$PWD/tools/v3lab/libcmpc_prev.so timeout -k 10 200 python tools/v3_ab.py $O/prev.npz 40 > $O/prev.txt 2>&1 &&
timeout -k 10 200 python tools/v3_ab.py $O/new.npz 40 > $O/new.txt 2>&1 &&
CMPC_LIB_PATH=$PWD/tools/v3lab/libcmpc_prev.so timeout -k 10 200 python tools/lpv_ab.py $O/lprev.npz 10 > $O/lprev.txt 2>&1 &&
timeout -k 10 200 python tools/lpv_ab.py $O/lnew.npz 10 > $O/lnew.txt 2>&1 &&
python tools/v3_ab.py cmp $O/prev.npz $O/new.npz > $O/cmp.txt 2>&1 &&
python tools/lpv_ab.py cmp $O/lprev.npz $O/lnew.npz > $O/lcmp.txt 2>&1
echo rc=$? > $O/rc.txt
