#!/bin/bash
# HBM traffic of the grouped weight-gradient launches: in-step (the C2 step,
# decoder = launch 0 of 2 per step, encoder = launch 1; PICK separates them --
# round 5's file averaged both over the decoder's algorithmic bytes) and the
# decoder's launch alone (tools/wgrad_one.py)
set -o pipefail
TAG=${TAG:-r6}
TAG=wgdec_$TAG PICK=0/2 bash tools/pmc_instep.sh wgrad4_kernel 131072 "wgrad_grouped M50432 x32 N512 K2048 bf16>f32" || exit 1
TAG=wgenc_$TAG PICK=1/2 bash tools/pmc_instep.sh wgrad4_kernel 131072 "wgrad_grouped M50432 x32 N512 K2048 bf16>f32" || exit 1
TAG=wgone_$TAG bash tools/wgrad_pmc.sh || exit 1
