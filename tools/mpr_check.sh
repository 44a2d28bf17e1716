# GPU suite + hammer (task default / forced fp64 MPR) + pen benches (run through gpurun)
set -e -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
grep -E "teacher-forced|passed|failed" gpurun_out/pytest_gpu.log
timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline > gpurun_out/ab_task.json
timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline --mpr fp64 > gpurun_out/ab_64.json
timeout -k 10 200 python bench.py --env pen-v0 --envs-per-gpu 16384 --steps 200 --no-cpu-baseline > gpurun_out/abp_task.json
for v in task 64; do python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v hammer', d['value'], d['roofline']['kernel_ms'])"; done
python -c "import json;d=json.load(open('gpurun_out/abp_task.json'));print('pen task', d['value'])"
