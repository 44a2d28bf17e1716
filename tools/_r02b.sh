set -o pipefail
mkdir -p gpurun_out/r02f
timeout -k 10 300 python -u tools/diag_tf.py hammer-v0 random 1 64 12 0 pos > gpurun_out/r02f/diag_pos.log 2>&1
echo diag rc $?
timeout -k 10 300 python -u tools/diag_tf.py hammer-v0 random 1 64 12 0x20000 pos > gpurun_out/r02f/diag_pos64.log 2>&1
echo diag rc $?
timeout -k 10 400 python bench.py > gpurun_out/r02f/bench.json 2> gpurun_out/r02f/bench.err
echo bench rc $?
