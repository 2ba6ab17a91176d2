#!/bin/bash
# Round-5 GPU step Q: the user-table RFFT tests (records built from non-library tables, host and
# device) and the whole fixed-point RFFT file.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/q1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_rfft_fixed.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log; grep -E "FAIL|Error" $O/t.log | head; exit $rc
