set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06h; mkdir -p $O
MG_SHAPES=proj,fc2 timeout -k 10 300 python -u tools/micro_gemm.py 3004,2015,2062,2063 > $O/mg.log 2>&1
