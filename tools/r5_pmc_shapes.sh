#!/bin/bash
# Standalone PMC traffic (tools/pmc_traffic.sh) of the fwd/dgrad shapes the
# bench line and DESIGN cite: encoder fc1 dgrad (the line's roofline_fwd_dgrad
# shape), decoder fc2 dgrad x GELU', decoder fc1 fwd + GELU' (micro-batch M).
set -o pipefail
T=${TAG:-r5ab}
TAG=${T}_encfc1dg timeout -k 10 400 bash tools/pmc_traffic.sh 6400 768 3072 0 1 0 || exit 1
TAG=${T}_decfc2dg timeout -k 10 400 bash tools/pmc_traffic.sh 25216 2048 512 0 1 5 || exit 1
TAG=${T}_decfc1fw timeout -k 10 400 bash tools/pmc_traffic.sh 25216 2048 512 0 0 4 || exit 1
