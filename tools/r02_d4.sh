#!/bin/bash
tools/ab.sh "d0:" "d4:--diag-mode 4"
