set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 300 python -u tools/ab_knob.py gemm_wide 0 1 > $O/ab_gemm_wide.log 2>&1
