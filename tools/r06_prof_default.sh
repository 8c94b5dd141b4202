#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench command (the committed profiles/r06_cfg2_kernel_stats.csv)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r06v}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_default -o run -- python3 $R/bench.py > $O/bench_under_rocprof.log 2>&1 || exit 1
grep '^{' $O/bench_under_rocprof.log | cut -c1-200
