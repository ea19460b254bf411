set -e
timeout -k 10 300 python -u scripts/e2e_bench.py --reads 1000 --deflate auto --reps 1 > /dev/null 2>&1
NTC_UPLOAD_TRACE=1 timeout -k 10 60 python -u scripts/init_cost.py /tmp/ntc_e2e/idx > gpurun_out/up_trace.log 2>&1
NTC_UPLOAD_TRACE=1 timeout -k 10 60 python -u scripts/init_cost.py /tmp/ntc_e2e/idx >> gpurun_out/up_trace.log 2>&1
rm -rf /tmp/ntc_e2e
