cd $GRAFT_REPO_ROOT
LOG=gpurun_out/pytest_combo.log TMO=600 bash scripts/gpu_tests.sh tests/test_gpu_hashagg_order.py tests/test_gpu_hashagg.py tests/test_gpu_groupby.py tests/test_gpu_h2o.py tests/test_gpu_superagg.py > /dev/null; tail -2 gpurun_out/pytest_combo.log
bash scripts/prof_h2o_ab.sh vaex_amd/libvaexhip_pair.so 1e9 q3 q5 q7
H2O_PROFILE=1 timeout -k 10 300 python scripts/exp_h2o.py 1e9 q3 > gpurun_out/h2o_prof.log 2>&1; grep -A28 "== profile q3" gpurun_out/h2o_prof.log
