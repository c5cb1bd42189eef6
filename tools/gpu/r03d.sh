#!/bin/bash
# r03d: k_prep_h A/B -- query loads two calls ahead (pfd2), and the fused kernel's XOF half alone
# (xofonly: the query's incremental cost).
set -e
STEPS=30 bash tools/ab_libs.sh base pfd2 xofonly base pfd2 xofonly
