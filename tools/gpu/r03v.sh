#!/bin/bash
# r03v: C2 A/B of a phase stagger of the first-round waves of k_prep_h (slot mod 3 x D,
# D = 120 / 240 / 360 us) against the current build, interleaved.
set -e
mkdir -p gpurun_out/r03v
STEPS=30 bash tools/ab_libs.sh base st12 st24 st36 base st12 st24 st36 | tee gpurun_out/r03v/ab.txt
