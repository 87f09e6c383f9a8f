#!/bin/bash
# A/B of tile5 register-pressure builds (tools/build_variant.sh): phase-A block
# size (SWH_T5_KB), staging candidates per lane (SWH_T5_U), waves per SIMD.
E=swift_subtask_dev_amd/_exp
B="python bench.py --no-cpu-baseline --steps 10"
exec tools/gpu_steps.sh \
 "150:base:$B" \
 "150:u1w2:SWH_LIB_PATH=$E/u1w2.so $B --loop-variant 5" \
 "150:u1w4:SWH_LIB_PATH=$E/u1w4.so $B --loop-variant 5" \
 "150:u1kb4w4:SWH_LIB_PATH=$E/u1kb4w4.so $B --loop-variant 5" \
 "150:base5f:$B --loop-variant 5"
