#!/bin/bash
# Round 4: probe v2 + ViT attention mode-2 A/B + decoder conv layouts vs round 3 (micro only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04c}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/probe_mfma_overlap.hip -o /tmp/probe_mfma_overlap > $O/probe_build.log 2>&1 && \
timeout -k 10 120 /tmp/probe_mfma_overlap > $O/probe.log 2>&1 && \
timeout -k 10 150 python -u tools/micro_attn.py 0,208,210 > $O/micro_attn.log 2>&1 && \
timeout -k 10 150 python -u tools/micro_upconv.py 0 > $O/upconv_new.log 2>&1 && \
CATSEG_HIP_LIB=$PWD/exp_so/libr03conv.so timeout -k 10 150 python -u tools/micro_upconv.py 0 > $O/upconv_old.log 2>&1 && \
timeout -k 10 150 python -u tools/micro_ring.py 0 > $O/ring_new.log 2>&1 && \
CATSEG_HIP_LIB=$PWD/exp_so/libr03conv.so timeout -k 10 150 python -u tools/micro_ring.py 0 > $O/ring_old.log 2>&1 && \
timeout -k 10 150 python -u tools/micro_gproj.py > $O/gproj_new.log 2>&1 && \
CATSEG_HIP_LIB=$PWD/exp_so/libr03conv.so timeout -k 10 150 python -u tools/micro_gproj.py > $O/gproj_old.log 2>&1
