#!/bin/bash
# Phase stamps of the training Winograd convs (trace build) + the same steps' wall clock
set -e
mkdir -p gpurun_out
AZ_LIB=abvar/trace/libaz.so timeout -k 10 300 python -u tools/train_trace.py 3 > gpurun_out/r05k_train_trace.txt 2>&1
