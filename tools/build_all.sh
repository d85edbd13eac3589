#!/bin/bash
# Build the extension and the kernel-experiment variants (P2P_LIB A/B builds) together, so
# an experiment library never lags the Python op schemas.
set -e
cd "$(dirname "$0")/.."
python tools/build_ext.py
python tools/build_ext.py --define P2P_EXP_NORMFRAG --out p2p_pytorch_amd/_C/exp_normfrag.so
