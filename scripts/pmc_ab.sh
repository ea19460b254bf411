#!/bin/bash
# PMC A/B: k_ms4 read requests and instruction counts per library (encode config only)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcab
for L in ntcomp_amd/ab/libgb1.so ntcomp_amd/ab/libgb0.so; do
  n=$(basename $L .so)
  NTC_GPU_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-include-regex 'k_ms4' --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmcab/rd_$n -o rd --output-format csv -- python3 bench.py --configs encode --no-cpu --steps 3 --warmup 0 > gpurun_out/pmcab/rd_$n.out 2>&1 || exit 1
  NTC_GPU_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-include-regex 'k_ms4' --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmcab/sq_$n -o sq --output-format csv -- python3 bench.py --configs encode --no-cpu --steps 3 --warmup 0 > gpurun_out/pmcab/sq_$n.out 2>&1 || exit 1
done
