set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 300 python -u tools/ab_knob.py rows_store 0 1 > $O/ab_rows_store.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_knob.py swin_store 0 1 > $O/ab_swin_store.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_knob.py ring_store 0 1 > $O/ab_ring_store.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_knob.py cls_store 0 1 > $O/ab_cls_store.log 2>&1
