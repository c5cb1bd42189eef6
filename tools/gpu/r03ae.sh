#!/bin/bash
# r03ae: r03ac (whole GPU suite with the executor's output copy kernel, jobs line x3) then r03ad
# (C2 A/B of the query loads two calls ahead).
set -e
bash tools/gpu/r03ac.sh
bash tools/gpu/r03ad.sh
