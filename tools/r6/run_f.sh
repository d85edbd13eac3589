#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r6g ROUNDS=2 BARGS="--precision fp8" bash tools/r6/ab_env.sh "P2P_S2T_F8=1" "P2P_S2T_F8=3" || exit $?
TAG=r6h ROUNDS=2 bash tools/r6/ab_env.sh "P2P_CLASS_MAJOR=0" "P2P_CLASS_MAJOR=1" || exit $?
