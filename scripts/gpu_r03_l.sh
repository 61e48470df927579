#!/bin/bash
# Round-3 session L: sharded tests + the simulated 8-rank step (forward and train kernels of rank 0).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/l
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_shard_exchange_gpu.py tests/test_shard_train_gpu.py tests/test_sharded_gpu.py \
    -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 scripts/shard_sim.py > $O/sim.log 2>&1 || { tail -20 $O/sim.log; exit 1; }
tail -n 1 $O/sim.log
echo session-l done
