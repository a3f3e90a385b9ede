#!/bin/bash
# Run each argument as one GPU step (each with its own `timeout -k 10 N` inside), in order; a step
# that fails its tests (status 1) does not stop the chain, anything else (a time limit, an abort, a
# fault) ends the call there.  Statuses go to gpurun_out/steps.log.
mkdir -p gpurun_out
for step in "$@"; do
    bash -c "$step"
    rc=$?
    echo "[gpu_steps] rc=$rc: $step" >> gpurun_out/steps.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
