#!/bin/bash
# round 5: exit-time SIGSEGV re-check (the round-4 command: CU-masked split streams under
# rocprofv3 --kernel-trace), then the whole GPU test suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/prof_cumask -o cumask -- python3 scripts/diag_split_streams.py cumask > $O/rocprof_cumask.log 2>&1
echo "rocprof cumask rc=$?" >> $O/rocprof_cumask.log
timeout -k 10 120 python3 scripts/diag_split_streams.py cumask > $O/plain_cumask.log 2>&1
echo "plain cumask rc=$?" >> $O/plain_cumask.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
