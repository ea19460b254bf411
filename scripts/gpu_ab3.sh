export TMPDIR=/tmp
mkdir -p gpurun_out/ab3
OUT=gpurun_out/ab3/nt CONFIGS=strains,encode VARIANTS="A B C cur" REPS=2 timeout -k 10 700 bash scripts/ab_bench.sh > gpurun_out/ab3/nt.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --configs strains --no-cpu --strain-inflight 2 > gpurun_out/ab3/s91_inflight2.json 2> gpurun_out/ab3/s91_inflight2.err || exit 1
timeout -k 10 200 python -u bench.py --configs strains --no-cpu --opt joint=0 > gpurun_out/ab3/s91_joint0.json 2> gpurun_out/ab3/s91_joint0.err || exit 1
cd /tmp/ntc_ceiling 2>/dev/null || true
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u scripts/host_ceiling.py --reads 4000000 --threads 16 --ctx 2 --reps 2 --kinds gz --out /tmp/ntc_ceiling > gpurun_out/ab3/ceil_gz.jsonl 2> gpurun_out/ab3/ceil_gz.err || exit 1
NTC_PGZ_STATS=1 timeout -k 10 100 tests/san/host_ceiling encode /tmp/ntc_ceiling/idx /tmp/ntc_ceiling/r.fq.gz /tmp/ntc_ceiling/x.dat 16 0 2 2 0 1 > gpurun_out/ab3/pgz_stats.txt 2>&1 || exit 1
for c in 1048576 4194304; do NTC_PGZ_CHUNK=$c timeout -k 10 100 tests/san/host_ceiling encode /tmp/ntc_ceiling/idx /tmp/ntc_ceiling/r.fq.gz /tmp/ntc_ceiling/x.dat 16 0 2 2 0 2 >> gpurun_out/ab3/pgz_chunk.txt 2>&1 || exit 1; done
