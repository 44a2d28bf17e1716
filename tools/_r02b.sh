set -o pipefail
mkdir -p gpurun_out/r02c
timeout -k 10 300 python -u tools/diag_tf.py hammer-v0 dapg 40 64 6 > gpurun_out/r02c/diag_hammer.log 2>&1
echo diag rc $?
