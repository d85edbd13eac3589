#!/bin/bash
# the Cout-64 stride-2 input gradients / ConvT: s2t halo kernel (default) vs the 512 x 64 m32 tile
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r6ah1 ROUNDS=2 bash tools/r6/ab_env.sh "X=1" "P2P_NO_S2T=1" || exit $?
echo done
