set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06o; mkdir -p $O
timeout -k 10 300 python -u tools/ab_knob.py attn_store 0 1 > $O/ab_attn_store.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_knob.py ln_store 1 0 > $O/ab_ln_store.log 2>&1
