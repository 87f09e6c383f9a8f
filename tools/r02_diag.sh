#!/bin/bash
tools/ab.sh "d0:" "d1:--diag-mode 1" "d2:--diag-mode 2" "d3:--diag-mode 3"
