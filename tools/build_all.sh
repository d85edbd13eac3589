#!/bin/bash
# Build the extension (every csrc/*.hip for gfx950 + the bindings) into p2p_pytorch_amd/_C.
set -e
cd "$(dirname "$0")/.."
python tools/build_ext.py
