#!/bin/bash
# Longer random-problem fuzz of every engine against the oracle (the counts
# DESIGN.md §7 quotes).  Output: gpurun_out/fz/fuzz.txt
set -o pipefail
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/fz
cd $GRAFT_REPO_ROOT
MDP_FUZZ_SMALL=80 MDP_FUZZ_LARGE=100 MDP_FUZZ_WIDE=30 MDP_FUZZ_SCN=40 MDP_FUZZ_FUT=60 \
  timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenario.py tests/test_gpu_future.py \
  -m gpu -k random -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/fz/fuzz.txt 2>&1
rc=$?; tail -3 gpurun_out/fz/fuzz.txt; exit $rc
