#!/bin/bash
# A/B of the tile hit-list capacity / occupancy builds (tools/build_variant.sh).
E=swift_subtask_dev_amd/_exp
B="python bench.py --no-cpu-baseline --steps 10"
exec tools/gpu_steps.sh \
 "150:m5:$B --loop-variant 5" \
 "150:c48v3:SWH_LIB_PATH=$E/cap48.so $B --loop-variant 3" \
 "150:c48v4:SWH_LIB_PATH=$E/cap48.so $B --loop-variant 4" \
 "150:c48v6:SWH_LIB_PATH=$E/cap48.so $B --loop-variant 6" \
 "150:c64v3:SWH_LIB_PATH=$E/cap64.so $B --loop-variant 3" \
 "150:c64v4:SWH_LIB_PATH=$E/cap64.so $B --loop-variant 4" \
 "150:c64v6:SWH_LIB_PATH=$E/cap64.so $B --loop-variant 6"
