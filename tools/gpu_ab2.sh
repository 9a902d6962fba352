#!/bin/bash
# Two-variant pass: txsig GPU tests through each variant, then the headline A/B (in-tree vs variants)
# and a kernel trace of each.  usage: bash tools/gpu_ab2.sh <tag> <variant> [variant ...]
TAG=$1; shift
for v in "$@"; do
  CORDA_AMD_LIB=tools/variants/$v.so bash tools/gpu_tests.sh ${TAG}_$v txsig || exit 1
done
args=""; for v in "$@"; do args="$args tools/variants/$v.so"; done
bash tools/ab_lib.sh $TAG $args || exit 1
for v in "$@"; do CORDA_AMD_LIB=tools/variants/$v.so bash tools/trace_env.sh ${TAG}_$v || exit 1; done
