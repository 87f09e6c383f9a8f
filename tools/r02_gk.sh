#!/bin/bash
tools/gpu_steps.sh \
 "300:gk2:python -u bench.py --workload grav --n 256 --steps 3 --warmup 1" \
 "300:gk3:SWH_LIB_PATH=swift_subtask_dev_amd/_exp/grav_k3.so python -u bench.py --workload grav --n 256 --steps 3 --warmup 1" \
 "300:gk4:SWH_LIB_PATH=swift_subtask_dev_amd/_exp/grav_k4.so python -u bench.py --workload grav --n 256 --steps 3 --warmup 1"
