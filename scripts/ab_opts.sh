# alternating A/B of ctx options on the in-tree build: bash scripts/ab_opts.sh "<configs>" "opt1=v" "opt2=v" ...
# ("-" = defaults)
set -e
mkdir -p gpurun_out/ab
CFG=${1:-encode,strains}
shift
B="python -u bench.py --configs $CFG --no-cpu --steps 10 --warmup 3"
for i in 1 2; do
  for O in "$@"; do
    if [ "$O" = - ]; then A=""; n=default; else A="--opt $O"; n=$(echo "$O" | tr '=' '_'); fi
    timeout -k 10 300 $B $A > gpurun_out/ab/$n.$i.json 2> gpurun_out/ab/$n.$i.err
  done
done
