#!/bin/bash
# Round 4: -fno-slp-vectorize per source file (experiment libraries via CATSEG_HIP_LIB), same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04o}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
E=$PWD/exp_so
for rep in 1 2; do
  timeout -k 10 120 python -u tools/micro_mlp.py > $O/mlp_base_$rep.log 2>&1 && \
  CATSEG_HIP_LIB=$E/libnoslp_rp.so timeout -k 10 120 python -u tools/micro_mlp.py > $O/mlp_noslp_$rep.log 2>&1 && \
  timeout -k 10 120 python -u tools/micro_swin.py 0 > $O/swin_base_$rep.log 2>&1 && \
  CATSEG_HIP_LIB=$E/libnoslp_sw.so timeout -k 10 120 python -u tools/micro_swin.py 0 > $O/swin_noslp_$rep.log 2>&1 && \
  CA_VARIANTS=0 timeout -k 10 150 python -u tools/micro_classattn.py > $O/ca_base_$rep.log 2>&1 && \
  CA_VARIANTS=0 CATSEG_HIP_LIB=$E/libnoslp_ca.so timeout -k 10 150 python -u tools/micro_classattn.py > $O/ca_noslp_$rep.log 2>&1 && \
  timeout -k 10 150 python -u tools/micro_attn.py 200 > $O/attn_base_$rep.log 2>&1 && \
  CATSEG_HIP_LIB=$E/libnoslp_at.so timeout -k 10 150 python -u tools/micro_attn.py 200 > $O/attn_noslp_$rep.log 2>&1 || exit 1
done
