#!/bin/bash
# Round-3 GPU pass b: the headline-configuration parity test, hammer C3 miss states, bench parity.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03b}
mkdir -p $OUT
echo "[r03b] tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 240 --timeout-method thread -k "headline_config or forward_internals or one_env_step" > $OUT/pytest.log 2>&1
echo "[r03b] diag"
timeout -k 10 600 python -u tools/diag_tf.py hammer-v0 random 110 256 30 > $OUT/diag.log 2>&1
cp gpurun_out/diag_hammer_random.json $OUT/
echo "[r03b] bench"
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-config2 > $OUT/bench.json 2> $OUT/bench.err
echo "[r03b] done"
