#!/bin/bash
# Round-5 profile of the fused inverse fixed-point RFFT (tools/rfft_inv_ab.py 1024 8192): one
# --kernel-trace --stats pass, then separate --pmc passes for the HBM read / write bytes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pinv; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/rfft_inv_ab.py 1024 8192 > $O/trace.txt 2> $O/trace.err || { echo "trace rc=$?"; exit 1; }
cat $O/trace.txt
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc1 -o run -- python3 tools/rfft_inv_ab.py 1024 8192 > $O/pmc1.txt 2> $O/pmc1.err || { echo "pmc1 rc=$?"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc2 -o run -- python3 tools/rfft_inv_ab.py 1024 8192 > $O/pmc2.txt 2> $O/pmc2.err || { echo "pmc2 rc=$?"; exit 1; }
echo all-ok
