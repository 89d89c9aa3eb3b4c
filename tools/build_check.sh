#!/bin/bash
# Build libpsengine.so for gfx950 in-tree and run the CPU suite; non-zero exit
# on any failure (run before sending the tree to a GPU box).
set -euo pipefail
cd "$(dirname "$0")/.."
python3 -c "
import sys; sys.path.insert(0, 'go-libp2p-pubsub_amd')
from psengine import _build; _build.build(force=True, verbose=False)" > /tmp/psamd_build.log 2>&1 || { grep -i error -A3 /tmp/psamd_build.log | head -30; exit 1; }
timeout 900 python3 -m pytest tests -x -q -m "not gpu" -n 4 2>&1 | tail -2
