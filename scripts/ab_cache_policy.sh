set -u
mkdir -p gpurun_out
for i in 1 2; do
for lib in libkge_hip.so libkge_hip_nt.so; do
  KGE_HIP_LIB=$PWD/customknowledgegraphembedding_amd/$lib timeout -k 10 180 python3 bench.py --no-cpu-baseline --sharded-steps 0 --steps 5 --train-steps 100 > gpurun_out/ab_$lib.$i.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['train_step']['ms_per_step'])" gpurun_out/ab_$lib.$i.json
done
done
KGE_HIP_LIB=$PWD/customknowledgegraphembedding_amd/libkge_hip_nt.so timeout -k 10 300 python3 -m pytest tests/test_train_gpu.py tests/test_run_gpu.py -m gpu -q -x -p no:cacheprovider > gpurun_out/nt_tests.log 2>&1; echo tests rc=$?; tail -2 gpurun_out/nt_tests.log
