set -e
mkdir -p gpurun_out/e2e
timeout -k 10 400 python -u scripts/e2e_bench.py --reads 10000000 --gzip > gpurun_out/e2e/gz.json 2> gpurun_out/e2e/gz.err
rm -rf /tmp/ntc_e2e
timeout -k 10 400 python -u scripts/e2e_bench.py --reads 10000000 --gzip --bgzf > gpurun_out/e2e/bgzf.json 2> gpurun_out/e2e/bgzf.err
rm -rf /tmp/ntc_e2e
