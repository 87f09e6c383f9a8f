#!/bin/bash
export TMPDIR=/tmp
tools/gpu_steps.sh "60:probe_ta:tools/probe/gather_ta" "200:diag:tools/diag_build.sh" || exit $?
tools/r03d_base.sh
