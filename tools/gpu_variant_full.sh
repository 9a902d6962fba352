#!/bin/bash
# A variant through the WHOLE GPU suite and smoke, then the headline A/B and a kernel trace.
# usage: bash tools/gpu_variant_full.sh <name>
V=${1:?variant}
CORDA_AMD_LIB=tools/variants/$V.so bash tools/gpu_tests.sh r03_$V && bash tools/ab_lib.sh $V tools/variants/$V.so && \
CORDA_AMD_LIB=tools/variants/$V.so bash tools/trace_env.sh $V
