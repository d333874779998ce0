cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in libvaexhip.so libvaexhip_r16.so libvaexhip_r4.so libvaexhip_t1024.so libvaexhip_tb256.so libvaexhip_tb1024.so; do echo "== $v"
VAEX_AMD_LIB=$PWD/vaex_amd/$v timeout -k 10 300 python -m pytest tests/test_gpu_superagg.py -m gpu -q -p no:cacheprovider -k "tiled_path" 2>&1 | tail -1
EXP_DEBUG=0 VAEX_AMD_LIB=$PWD/vaex_amd/$v timeout -k 10 300 python scripts/exp_tiles.py 1e9 || exit $?; done
