#!/bin/bash
# PM mesh: GPU parity vs the oracle, then the whole GPU suite
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300:t_mesh:python -u -m pytest tests/test_mesh.py -x -v --timeout 120 --timeout-method thread" \
 "600:t_all:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
