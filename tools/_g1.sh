set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06d; mkdir -p $O
MG_SHAPES=sq8k timeout -k 10 300 python -u tools/micro_gemm.py 2042,2052,2056,2057 > $O/mg_sq8k.log 2>&1 &&
MG_SHAPES=qkv,fc1 timeout -k 10 300 python -u tools/micro_gemm.py 3004,2040,2041,2050,2051,2052 > $O/mg_qkv_fc1.log 2>&1
