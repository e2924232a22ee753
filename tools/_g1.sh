set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06l; mkdir -p $O
MG_SHAPES=proj,fc2 timeout -k 10 300 python -u tools/micro_gemm.py 3004,2053,2054 > $O/mg.log 2>&1
