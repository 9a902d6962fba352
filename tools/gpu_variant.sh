#!/bin/bash
# GPU-box pass for a variant library: the whole GPU suite and smoke through it (CORDA_AMD_LIB), the
# headline A/B against the in-tree build, then headline runs of the variant under each environment
# setting given.  usage: bash tools/gpu_variant.sh <name> [NAME=VALUE ...]  (tools/variants/<name>.so)
V=${1:?variant name}; shift
CORDA_AMD_LIB=tools/variants/$V.so bash tools/gpu_tests.sh r03_$V && bash tools/ab_lib.sh $V tools/variants/$V.so || exit 1
if [ $# -gt 0 ]; then CORDA_AMD_LIB=tools/variants/$V.so bash tools/ab_env_headline.sh env_$V - "$@"; fi
