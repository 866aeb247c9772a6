#!/bin/bash
# Step-boundary idle time of the captured C2 step: loss-read modes and HIP
# runtime graph settings (tools/step_boundary_probe.py; one process each).
set -o pipefail
probe() {   # probe <read mode> [ENV=VALUE ...]
  local mode=$1; shift
  echo "== read=$mode $*"
  env MAECLIP_PROBE=1 "$@" timeout -k 10 240 python -u tools/step_boundary_probe.py --steps 40 --read "$mode" || exit 1
}
probe prev
probe none
probe sync
probe prev DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
probe prev DEBUG_HIP_GRAPH_BATCH_SIZE=8
probe prev DEBUG_HIP_GRAPH_BATCH_SIZE=1024
probe prev
