cd $GRAFT_REPO_ROOT && O=gpurun_out/r06k && mkdir -p $O &&
timeout -k 10 300 python -u tools/ab_knob.py gemm_group 4 2 8 4 > $O/ab_gemm_group.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_knob.py gemm4_group 5 3 8 5 > $O/ab_gemm4_group.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_knob.py ln_variant 0 2 3 0 > $O/ab_ln_variant.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_knob.py attn_tail_skip 0 1 0 > $O/ab_attn_tail.log 2>&1
