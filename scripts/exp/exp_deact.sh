#!/bin/bash
# Basic-slack deactivation: its own tests first, then the whole GPU suite, then the bench line
# (window + whole solves) with it on and off.  (experiment helper)
source "$(dirname "$0")/../gpu_step.sh"
step deact 400 python -u -m pytest tests/test_gpu_deactivate.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu || exit $?
grep -c PASSED $O/deact.log
step suite 900 python -u -m pytest tests -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu --deselect tests/test_gpu_deactivate.py || exit $?
tail -1 $O/suite.log
step bench_on 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
tail -1 $O/bench_on.log | cut -c1-200
