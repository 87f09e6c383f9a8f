tools/gpu_steps.sh \
 "150:w3v4:SWH_LIB_PATH=swift_subtask_dev_amd/_exp/wpe3.so python bench.py --no-cpu-baseline --steps 10 --loop-variant 4" \
 "150:w3v5:SWH_LIB_PATH=swift_subtask_dev_amd/_exp/wpe3.so python bench.py --no-cpu-baseline --steps 10 --loop-variant 5" \
 "150:w3v3:SWH_LIB_PATH=swift_subtask_dev_amd/_exp/wpe3.so python bench.py --no-cpu-baseline --steps 10 --loop-variant 3" \
 "150:w4v4:SWH_LIB_PATH=swift_subtask_dev_amd/_exp/wpe4.so python bench.py --no-cpu-baseline --steps 10 --loop-variant 4" \
 "150:w4v5:SWH_LIB_PATH=swift_subtask_dev_amd/_exp/wpe4.so python bench.py --no-cpu-baseline --steps 10 --loop-variant 5" \
 "150:w4v3:SWH_LIB_PATH=swift_subtask_dev_amd/_exp/wpe4.so python bench.py --no-cpu-baseline --steps 10 --loop-variant 3" \
 "150:w4v5g32:SWH_LIB_PATH=swift_subtask_dev_amd/_exp/wpe4.so python bench.py --no-cpu-baseline --steps 10 --loop-variant 5 --group-size 32"
