#!/bin/bash
# Basic-slack deactivation on every shard: its tests, the multi-shard / IPC / long-pin subset, then the
# whole GPU suite.  (experiment helper)
source "$(dirname "$0")/../gpu_step.sh"
step deact 500 python -u -m pytest tests/test_gpu_deactivate.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu || exit $?
tail -1 $O/deact.log
step suite 1000 python -u -m pytest tests -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu --deselect tests/test_gpu_deactivate.py || exit $?
tail -1 $O/suite.log
