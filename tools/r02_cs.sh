#!/bin/bash
tools/ab.sh "c075:--cell-scale 0.75" "c125:--cell-scale 1.25" "c15:--cell-scale 1.5" "c2:--cell-scale 2"
