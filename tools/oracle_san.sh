#!/bin/bash
# the CPU restatement (oracle/src) under AddressSanitizer + UndefinedBehaviorSanitizer.
# Builds oracle/_build_san/liboracle.so (make -C oracle SAN=1) and runs every CPU test that
# calls the restatement with it preloaded; any UB report aborts the test run (halt_on_error).
# Usage: tools/oracle_san.sh [extra pytest args]      (CPU only; ~2 minutes)
set -euo pipefail
cd "$(dirname "$0")/.."
make -C oracle SAN=1 >/dev/null
export LD_PRELOAD="$(gcc -print-file-name=libasan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export CMSISDSP_ORACLE_SO="$PWD/oracle/_build_san/liboracle.so"
python -m pytest -q -m "not gpu" -p no:cacheprovider tests/test_oracle.py tests/test_golden.py tests/test_mfcc.py \
  tests/test_mfcc_q31.py tests/test_mfcc_q15.py tests/test_conv_family.py tests/test_conv_opt.py tests/test_multirate.py \
  tests/test_sparse.py tests/test_lattice.py tests/test_rfft_fixed.py tests/test_fir_long.py "$@"
