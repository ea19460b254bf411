#!/bin/bash
# A/B of unpacker builds (segment sizes): ntc_unpack_streams on C91 blocks, 2 and 16 blocks per
# call, kernel trace per variant (VARIANTS: X = ntcomp_amd/ab/libntcomp_gpu_X.so, cur = in-tree)
set -e
O=gpurun_out/unpack_ab
mkdir -p $O
export TMPDIR=/tmp
for v in ${VARIANTS:-cur}; do
  lib=ntcomp_amd/ab/libntcomp_gpu_$v.so
  [ "$v" = cur ] && lib=ntcomp_amd/libntcomp_gpu.so
  NTC_GPU_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o unp --output-format csv -- \
      python3 scripts/unpack_sync.py --no-sim --out $O/$v.json > $O/$v.log 2>&1
done
