#!/bin/bash
# Round-4 GPU pass R: the whole GPU suite with the headline-form test at the bench's 512-step
# launches and the relief pair's other forms.
set -o pipefail
mkdir -p gpurun_out/r
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r/suite.txt 2>&1
rc=$?; tail -2 gpurun_out/r/suite.txt; grep -E "FAILED|pair_forms|headline" gpurun_out/r/suite.txt | head -12
exit $rc
