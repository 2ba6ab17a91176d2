#!/bin/bash
# VALU issue-rate probes on one MI355X (tools/probes/op_rate.hip, valu_rate.hip).
set -o pipefail
mkdir -p gpurun_out/probes
timeout -k 10 120 tools/probes/op_rate > gpurun_out/probes/op_rate.txt 2>&1 || exit $?
cat gpurun_out/probes/op_rate.txt
timeout -k 10 120 tools/probes/valu_rate > gpurun_out/probes/valu_rate.txt 2>&1 || exit $?
cat gpurun_out/probes/valu_rate.txt
