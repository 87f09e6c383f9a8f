#!/bin/bash
# A/B of the v3/v4 staging fetch width (SWH_TILE_FETCH) and occupancy builds.
E=swift_subtask_dev_amd/_exp
B="python bench.py --no-cpu-baseline --steps 10"
exec tools/gpu_steps.sh \
 "150:f1:SWH_LIB_PATH=$E/f1.so $B" \
 "150:f1w3:SWH_LIB_PATH=$E/f1w3.so $B --loop-variant 4" \
 "150:f4:SWH_LIB_PATH=$E/f4.so $B"
