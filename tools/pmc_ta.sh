#!/bin/bash
# TA / TD busy of the list walks and build (is the density walk address-bound?)
export TMPDIR=/tmp
mkdir -p gpurun_out/ta
rocprofv3 --list-avail > gpurun_out/ta/avail.txt 2>&1 || true
grep -o -E "\bT[AD]_[A-Z_]*BUSY[a-z_]*\b|\bTCP_[A-Z_]*\b" gpurun_out/ta/avail.txt | sort -u | head -80 > gpurun_out/ta/names.txt
cat gpurun_out/ta/names.txt | head -40
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE --kernel-include-regex "list_build|walk_kernel" -d gpurun_out/ta/p1 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-breakdown > gpurun_out/ta/p1.log 2>&1
echo "p1 rc=$?"
