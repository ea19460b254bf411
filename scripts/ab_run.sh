set -e
mkdir -p gpurun_out/ab
B="python -u bench.py --configs encode,strains --no-cpu --steps 10 --warmup 3"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/ab/new$i.json 2> gpurun_out/ab/new$i.err
  NTC_GPU_LIB=ntcomp_amd/ab/libprev.so timeout -k 10 200 $B > gpurun_out/ab/old$i.json 2> gpurun_out/ab/old$i.err
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/gpu_tests.log 2>&1
