#!/bin/bash
# Round-5 final bench lines: every workload on the final library (tools/round_lines.sh).
set -e -o pipefail
export TMPDIR=/tmp
rm -rf gpurun_out/lines_r05final
bash tools/round_lines.sh r05final
echo all-ok
