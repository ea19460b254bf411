# alternating A/B of device builds: bash scripts/ab_run.sh "<configs>" lib1 lib2 ...  (lib "cur" = the in-tree build)
# extra bench arguments: AB_ARGS="--err-ppm 0"
set -e
mkdir -p gpurun_out/ab
CFG=${1:-encode,strains}
shift
B="python -u bench.py --configs $CFG --no-cpu --steps 10 --warmup 3 ${AB_ARGS:-}"
for i in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    if [ "$L" = cur ]; then
      timeout -k 10 300 $B > gpurun_out/ab/$n.$i.json 2> gpurun_out/ab/$n.$i.err
    else
      NTC_GPU_LIB=$L timeout -k 10 300 $B > gpurun_out/ab/$n.$i.json 2> gpurun_out/ab/$n.$i.err
    fi
  done
done
