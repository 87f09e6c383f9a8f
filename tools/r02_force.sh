#!/bin/bash
tools/gpu_steps.sh \
 "600:t_f:python -u -m pytest tests/test_gpu_parity.py tests/test_dosub.py -q --timeout 300 --timeout-method thread -k 'force or chain or headline or clustered or 125'" \
 "200:fa:python -u bench.py --no-cpu-baseline" \
 "200:fb:SWH_LIB_PATH=swift_subtask_dev_amd/_exp/wpe4.so python -u bench.py --no-cpu-baseline"
