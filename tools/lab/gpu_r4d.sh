set -o pipefail
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 200 python tools/cfg5_sched.py > $O/sched_fp64.txt 2>&1 &&
timeout -k 10 200 python tools/cfg5_sched.py 8192 fp32 > $O/sched_fp32.txt 2>&1 &&
timeout -k 10 200 python bench.py --agents 512 --steps 20 --warmup 3 --no-cpu --no-ref --no-cfg5 > $O/b512.json 2> $O/b512.err &&
timeout -k 10 200 python bench.py --agents 4096 --steps 10 --warmup 2 --no-cpu --no-ref --no-cfg5 > $O/b4096.json 2> $O/b4096.err &&
timeout -k 10 200 python bench.py --agents 2048 --steps 10 --warmup 2 --no-cpu --no-ref --no-cfg5 > $O/b2048.json 2> $O/b2048.err &&
timeout -k 10 200 python bench.py --agents 1024 --steps 20 --warmup 3 --no-cpu --no-ref --no-cfg5 > $O/b1024.json 2> $O/b1024.err
echo rc=$? > $O/rc.txt
mkdir -p gpurun_out/ab3 && timeout -k 10 200 python tools/v3_ab.py gpurun_out/ab3/new.npz 40 > gpurun_out/ab3/new.txt 2>&1 && timeout -k 10 100 python tools/stamps.py > gpurun_out/ab3/stamps_new.txt 2>&1
