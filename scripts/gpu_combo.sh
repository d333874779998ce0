cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python scripts/prof_c3.py 1e9 > gpurun_out/prof_c3.log 2>&1; head -45 gpurun_out/prof_c3.log
mkdir -p gpurun_out/pq10
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pq10/trace -o run -- python3 scripts/exp_h2o.py 1e9 q10 > gpurun_out/pq10/log.txt 2>&1; grep -E "^q" gpurun_out/pq10/log.txt
python3 scripts/prof_summary.py gpurun_out/pq10 > gpurun_out/q10_summary.txt; head -25 gpurun_out/q10_summary.txt; rm -rf gpurun_out/pq10
