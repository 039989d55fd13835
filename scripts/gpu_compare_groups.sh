set -o pipefail
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_r1c.log 2>&1
echo PYTEST=$? >> gpurun_out/pytest_gpu_r1c.log
for G in 1 2; do
  NGT_AMD_GROUPS=$G timeout -k 10 400 python bench.py --steps 5 --no-cpu --eps 0.095,0.096,0.097,0.098,0.1 > gpurun_out/bench_g$G.json 2> gpurun_out/bench_g$G.log || break
done
tail -2 gpurun_out/pytest_gpu_r1c.log
