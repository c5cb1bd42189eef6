#!/bin/bash
# r03ad: C2 A/B of the fused query's loads two calls ahead (QH_PFD=2) against one call ahead.
set -e
mkdir -p gpurun_out/r03ad
STEPS=30 bash tools/ab_libs.sh base pfd2 base pfd2 base pfd2 | tee gpurun_out/r03ad/ab.txt
