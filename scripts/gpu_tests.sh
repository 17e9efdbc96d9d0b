#!/bin/bash
# Round 6: the GPU tests touched by a change (PK: pytest -k expression; FILES: test files)
source "$(dirname "$0")/gpu_step.sh"
step tests ${SECS:-900} python -u -m pytest ${FILES:-tests} -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "${PK:-}" || exit $?
grep -c PASSED $O/tests.log
