#!/bin/bash
# Odd-N PM mesh on the GPU with rocFFT's logs: the N = 15
# parity test in its own process, rocFFT trace + plan + RTC logs and the
# plans' work sizes (SWH_PM_DEBUG) under gpurun_out/, the RTC kernel cache in
# a writable directory.
set -o pipefail
out=gpurun_out/r04_pm_odd
mkdir -p $out/rtc_cache
export ROCFFT_LAYER=41 ROCFFT_LOG_TRACE_PATH=$out/rocfft_trace.log \
       ROCFFT_LOG_PLAN_PATH=$out/rocfft_plan.log ROCFFT_LOG_RTC_PATH=$out/rocfft_rtc.log \
       ROCFFT_RTC_CACHE_PATH=$out/rtc_cache/rocfft_kernel_cache.db SWH_PM_DEBUG=1
timeout -k 10 300 python -u -m pytest -v -s --timeout 240 --timeout-method thread \
  tests/test_mesh.py -k "gpu_pm" > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/pytest.log
exit $rc
